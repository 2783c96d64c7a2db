"""numpy restatement of the MPVAE probit ELBO -- TEST INFRASTRUCTURE ONLY.

Restates reference ``mpvae.py`` lines 103-210 (``build_multi_classification_loss``,
``pairwise_and``/``pairwise_sub``, ``compute_loss``) as explicit forward and
*analytic* backward formulas, organised the way the build shards the Monte-Carlo
sample axis S:

  shard_forward   per-shard statistics      (rowstat, bstat, colsum)
  combine_bstats  exact cross-shard combine (log-sum-exp + sums)
  finalize        the 8-tuple of compute_loss
  shard_backward  per-shard gradients       (dfe, dfx, dR) given global stats

Numerics: the probit probability E = Phi(u)(1-1e-6) + 0.5e-6 is evaluated in
float32 with the reference's own operation order (mpvae.py:171-180, torch
``Normal.cdf`` = 0.5*(1+erf(x/sqrt 2))), because that is the ill-conditioned
step (1+erf near -1) and the reference computes it in fp32.  Everything after E
(logs, exps, sums, log-sum-exp, gradients) runs in float64.

Degenerate label rows (no positive or no negative label) follow the reference:
ranking loss 0 in the forward (mpvae.py:119-121); in the backward the whole
row's gradient is NaN whenever the ranking term of that branch receives a
gradient (0/0 in the ``div`` backward of mpvae.py:118).
"""
import math

import numpy as np
from scipy import special

F32 = np.float32
C1 = F32(1.0) - F32(1e-6)          # (1 - eps1), eps1 = tensor([1e-6]).float()  mpvae.py:156,177
C0 = F32(1e-6) * F32(0.5)          # eps1 * 0.5
INV_SQRT_2PI = 1.0 / math.sqrt(2.0 * math.pi)
KL_EPS = 1e-6                      # mpvae.py:148
KL_WEIGHT = 1.1                    # mpvae.py:208


# --------------------------------------------------------------------------- E
def probit_prob(u32):
    """E = Normal(0,1).cdf(u)*(1-eps1) + eps1*0.5 in float32 (mpvae.py:171-180)."""
    u32 = np.asarray(u32, F32)
    x = (u32 / F32(math.sqrt(2.0))).astype(F32)
    cdf = F32(0.5) * (F32(1.0) + special.erf(x).astype(F32))
    return (cdf.astype(F32) * C1 + C0).astype(F32)


def noise_product(noise, R, t_fp32=False):
    """t = tensordot(noise, R.T.float()) -> (S,B,L) float32 (mpvae.py:165-170),
    accumulated in fp64 and rounded once; t_fp32: by an fp32 GEMM, as the
    reference's own tensordot computes it (to measure how far fp32 arithmetic
    alone moves the results)."""
    if t_fp32:
        Rt32 = np.asarray(R).astype(F32).T
        return np.asarray(noise, F32) @ Rt32
    Rt = np.asarray(R).astype(F32).astype(np.float64).T          # (z, L)
    t = np.asarray(noise, np.float64) @ Rt
    return t.astype(F32)


def label_sets(y):
    """pos / neg masks (exact 1 / exact 0, mpvae.py:107-108) and n = |pos|*|neg|."""
    y = np.asarray(y, F32)
    pos, neg = (y == 1.0), (y == 0.0)
    n = pos.sum(1).astype(np.float64) * neg.sum(1).astype(np.float64)
    return pos, neg, n


# ------------------------------------------------------------------- forward
def branch_rows(E, y, ranking="factorized"):
    """Per-(s,b) statistics of one branch: log-prob, P, N, ranking loss c[s,b].

    logp[s,b] = sum_l y log E + (1-y) log(1-E)                  (mpvae.py:184-185)
    c[s,b]    = sum_{j in pos, k in neg} exp(-5(E_j-E_k)) / (5 n)  (mpvae.py:110-118)
              = P*N / (5 n),  P = sum_pos exp(-5E), N = sum_neg exp(5E)
    NaN/inf (n == 0) -> 0                                       (mpvae.py:119-121)
    """
    E = np.asarray(E, np.float64)
    y64 = np.asarray(y, np.float64)
    pos, neg, n = label_sets(y)
    logp = (y64 * np.log(E) + (1.0 - y64) * np.log(1.0 - E)).sum(-1)
    P = (np.exp(-5.0 * E) * pos).sum(-1)
    N = (np.exp(5.0 * E) * neg).sum(-1)
    if ranking == "naive":
        diff = E[..., :, None] - E[..., None, :]                   # [j,k] = E_j - E_k
        truth = (pos[:, :, None] & neg[:, None, :])
        sums = (np.exp(-5.0 * diff) * truth).sum((-2, -1))
    else:
        sums = P * N
    with np.errstate(divide="ignore", invalid="ignore"):
        c = sums / (5.0 * n)
    c = np.where(np.isfinite(c), c, 0.0)
    return logp, P, N, c


def shard_forward(y, fe_out, fx_out, R, noise, ranking="factorized", t_fp32=False):
    """Statistics of one S-shard (noise = this shard's (S_loc,B,z) slice).

    Returns dict with
      rowstat (6,B,S_loc) = [logp_e, logp_x, P_e, N_e, P_x, N_x]
      bstat   (6,B)       = [m_e, Z_e, m_x, Z_x, csum_e, csum_x]  (local max / sum-exp)
      colsum  (2,B,L)     = [sum_s E, sum_s E_x]
      E, Ex, t            (S_loc,B,L) for the backward
    """
    t = noise_product(noise, R, t_fp32)
    E = probit_prob(t + np.asarray(fe_out, F32))
    Ex = probit_prob(t + np.asarray(fx_out, F32))
    le, Pe, Ne, ce = branch_rows(E, y, ranking)
    lx, Px, Nx, cx = branch_rows(Ex, y, ranking)
    rowstat = np.stack([le.T, lx.T, Pe.T, Ne.T, Px.T, Nx.T])       # (6,B,S_loc)
    me, mx = le.max(0), lx.max(0)
    bstat = np.stack([me, np.exp(le - me).sum(0), mx, np.exp(lx - mx).sum(0),
                      ce.sum(0), cx.sum(0)])
    colsum = np.stack([E.astype(np.float64).sum(0), Ex.astype(np.float64).sum(0)])
    return dict(rowstat=rowstat, bstat=bstat, colsum=colsum, E=E, Ex=Ex, t=t)


def combine_bstats(bstats):
    """Exact cross-shard combine: M = max m_r, Z = sum Z_r exp(m_r - M), sums add."""
    b = np.stack(bstats)                                           # (R,6,B)
    out = np.empty(b.shape[1:])
    for m_i, z_i in ((0, 1), (2, 3)):
        M = b[:, m_i].max(0)
        out[m_i] = M
        out[z_i] = (b[:, z_i] * np.exp(b[:, m_i] - M)).sum(0)
    out[4:] = b[:, 4:].sum(0)
    return out


def kl_term(mu_e, lv_e, mu_x, lv_x):
    """KL(q_label || p_feat) averaged over the batch (mpvae.py:147-148)."""
    mu_e, lv_e, mu_x, lv_x = (np.asarray(a, np.float64) for a in (mu_e, lv_e, mu_x, lv_x))
    per = (lv_x - lv_e) - 1.0 + np.exp(lv_e - lv_x) + (mu_x - mu_e) ** 2 / (np.exp(lv_x) + KL_EPS)
    return float(np.mean(0.5 * per.sum(1)))


def finalize(bstat, colsum, S_total, kl, nll_coeff, c_coeff):
    """The 8-tuple of compute_loss (mpvae.py:186-210) from global statistics."""
    B = bstat.shape[1]
    nll = float(np.mean(-np.log(bstat[1] / S_total) - bstat[0]))
    nll_x = float(np.mean(-np.log(bstat[3] / S_total) - bstat[2]))
    c = float(bstat[4].sum() / (S_total * B))
    c_x = float(bstat[5].sum() / (S_total * B))
    total = (nll + nll_x) * nll_coeff + (c + c_x) * c_coeff + kl * KL_WEIGHT
    return dict(total=total, nll=nll, nll_x=nll_x, c=c, c_x=c_x, kl=kl,
                indiv_prob=colsum[1] / S_total, indiv_prob_label=colsum[0] / S_total)


# ------------------------------------------------------------------ backward
def upstream(g_total=None, g_nll=None, g_nll_x=None, g_c=None, g_c_x=None, g_kl=None,
             nll_coeff=0.0, c_coeff=0.0):
    """Fold d total into the component gradients; a component is 'live' when any
    gradient (even 0) reaches it -- that is what triggers the reference's NaN rows."""
    def add(g, extra):
        if g is None and extra is None:
            return None
        return (0.0 if g is None else g) + (0.0 if extra is None else extra)
    gt = g_total
    return dict(
        nll=add(g_nll, None if gt is None else nll_coeff * gt),
        nll_x=add(g_nll_x, None if gt is None else nll_coeff * gt),
        c=add(g_c, None if gt is None else c_coeff * gt),
        c_x=add(g_c_x, None if gt is None else c_coeff * gt),
        kl=add(g_kl, None if gt is None else KL_WEIGHT * gt))


def row_coefficients(rowstat, bstat_global, y, S_total, g):
    """coef (6,B,S_loc) = [alpha_e, betaP_e, betaN_e, alpha_x, betaP_x, betaN_x].

    dE[s,b,l] = alpha*(y/E - (1-y)/(1-E)) - [y==1] betaP e^{-5E} + [y==0] betaN e^{5E}
      alpha = -g_nll * softmax_s(logp)[s,b] / B
      betaP = g_c * N[s,b] / (n_b S B),  betaN = g_c * P[s,b] / (n_b S B)
    """
    _, B, _ = rowstat.shape
    _, _, n = label_sets(y)
    coef = np.zeros(rowstat.shape)
    for br, (li, pi, ni, mi, zi, gn, gc) in enumerate(
            [(0, 2, 3, 0, 1, g["nll"], g["c"]), (1, 4, 5, 2, 3, g["nll_x"], g["c_x"])]):
        if gn is not None:
            w = np.exp(rowstat[li] - bstat_global[mi][:, None]) / bstat_global[zi][:, None]
            coef[3 * br] = -gn * w / B
        if gc is not None:
            with np.errstate(divide="ignore", invalid="ignore"):
                scale = gc / (n[:, None] * S_total * B)
                coef[3 * br + 1] = scale * rowstat[ni]
                coef[3 * br + 2] = scale * rowstat[pi]
            dead = n == 0
            coef[3 * br:3 * br + 3, dead, :] = np.nan
    return coef


def shard_backward(fwd, y, fe_out, fx_out, noise, coef, S_total, g_I=None, g_IL=None):
    """(dfe, dfx, dR) contributions of one shard, with coef from row_coefficients."""
    y64 = np.asarray(y, np.float64)
    pos, neg, _ = label_sets(y)
    t = fwd["t"].astype(np.float64)
    out = []
    gus = []
    for br, (E, base, gind) in enumerate([(fwd["E"], fe_out, g_IL), (fwd["Ex"], fx_out, g_I)]):
        E = E.astype(np.float64)
        a = coef[3 * br].T[:, :, None]                 # (S_loc,B,1)
        bP = coef[3 * br + 1].T[:, :, None]
        bN = coef[3 * br + 2].T[:, :, None]
        gE = a * (y64 / E - (1.0 - y64) / (1.0 - E))
        gE = gE - np.where(pos, bP * np.exp(-5.0 * E), 0.0) + np.where(neg, bN * np.exp(5.0 * E), 0.0)
        # NaN rows must poison every label of the row, including non-0/1 labels
        gE = np.where(np.isnan(bP) | np.isnan(bN), np.nan, gE)
        if gind is not None:
            gE = gE + np.asarray(gind, np.float64)[None] / S_total
        u = (t.astype(F32) + np.asarray(base, F32)).astype(np.float64)
        gu = gE * float(C1) * INV_SQRT_2PI * np.exp(-0.5 * u * u)
        gus.append(gu)
        out.append(gu.sum(0))
    G = gus[0] + gus[1]
    # dR[l, k] = sum_{s,b} G[s,b,l] eps[s,b,k]: one fp64 BLAS product over the
    # S*B sample rows (np.einsum's loop would take minutes at S*B ~ 1e5)
    L, z = G.shape[-1], np.shape(noise)[-1]
    dR = G.reshape(-1, L).T @ np.asarray(noise, np.float64).reshape(-1, z)
    return out[0], out[1], dR


def kl_backward(mu_e, lv_e, mu_x, lv_x, g_kl):
    mu_e, lv_e, mu_x, lv_x = (np.asarray(a, np.float64) for a in (mu_e, lv_e, mu_x, lv_x))
    B = mu_e.shape[0]
    s = 0.5 * g_kl / B
    ex = np.exp(lv_x)
    den = ex + KL_EPS
    d = mu_x - mu_e
    r = np.exp(lv_e - lv_x)
    return dict(fe_mu=s * (-2.0 * d / den), fx_mu=s * (2.0 * d / den),
                fe_logvar=s * (-1.0 + r), fx_logvar=s * (1.0 - r - d * d * ex / den ** 2))


# ---------------------------------------------------------------- one-shot API
def elbo_forward(y, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar, R, noise,
                 nll_coeff, c_coeff, ranking="factorized", shards=1, t_fp32=False):
    """Whole compute_loss forward; ``shards`` > 1 splits S and combines exactly;
    ``t_fp32``: t from an fp32 GEMM (noise_product)."""
    S = noise.shape[0]
    edges = np.linspace(0, S, shards + 1).astype(int)
    parts = [shard_forward(y, fe_out, fx_out, R, noise[a:b], ranking, t_fp32)
             for a, b in zip(edges[:-1], edges[1:])]
    bstat = combine_bstats([p["bstat"] for p in parts])
    colsum = sum(p["colsum"] for p in parts)
    kl = kl_term(fe_mu, fe_logvar, fx_mu, fx_logvar)
    out = finalize(bstat, colsum, S, kl, nll_coeff, c_coeff)
    out["_parts"], out["_edges"], out["_bstat"] = parts, edges, bstat
    return out


def elbo_backward(fwd, y, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar, noise,
                  nll_coeff, c_coeff, g_total=None, g_nll=None, g_nll_x=None, g_c=None,
                  g_c_x=None, g_kl=None, g_I=None, g_IL=None):
    """Analytic gradients of sum_i g_i * output_i w.r.t. the 7 tensor inputs."""
    g = upstream(g_total, g_nll, g_nll_x, g_c, g_c_x, g_kl, nll_coeff, c_coeff)
    S = noise.shape[0]
    B, L = np.asarray(y).shape
    dfe, dfx = np.zeros((B, L)), np.zeros((B, L))
    dR = 0.0
    for p, a, b in zip(fwd["_parts"], fwd["_edges"][:-1], fwd["_edges"][1:]):
        coef = row_coefficients(p["rowstat"], fwd["_bstat"], y, S, g)
        e, x, r = shard_backward(p, y, fe_out, fx_out, noise[a:b], coef, S, g_I, g_IL)
        dfe, dfx, dR = dfe + e, dfx + x, dR + r
    grads = dict(fe_out=dfe, fx_out=dfx, r_sqrt_sigma=dR)
    gk = 0.0 if g["kl"] is None else g["kl"]
    grads.update(kl_backward(fe_mu, fe_logvar, fx_mu, fx_logvar, gk))
    return grads
