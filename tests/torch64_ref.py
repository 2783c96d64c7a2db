"""oracle/probit_elbo.py restated in torch fp64, S-chunked -- TEST INFRASTRUCTURE.

The numpy oracle holds the whole (S, B, L) problem on the host and runs its
transcendentals on one core: fine up to ~1e8 label-samples, minutes beyond.
The headline configuration (C4: S = 4096, B = 512, L = z = 1024, 2.1e9
label-samples, a noise GEMM of 4.4e12 flop) is out of its reach, yet it is the
size at which the product's dR GEMM reduces its longest split-K chunks
(131072 sample rows per fp32 accumulator).  This module evaluates the same
formulas -- E in float32 in the reference's op order (mpvae.py:171-180), every
other quantity in float64 -- as torch ops on whatever device the inputs live
on, in chunks of the sample axis, so the full C4 problem runs in seconds on
the GPU box with a few GB of scratch.

It is a restatement of ``oracle.probit_elbo`` (same function names, same
numerics) and is pinned to it: ``tests/test_torch64_ref.py`` (CPU) compares
the two on random and degenerate cases.  Only tests import it; the product
never does.  References: mpvae.py:103-210 (via oracle/probit_elbo.py).
"""
import math

import torch

F32, F64 = torch.float32, torch.float64
_C1 = torch.tensor(1.0, dtype=F32) - torch.tensor(1e-6, dtype=F32)   # 1 - eps1
_C0 = torch.tensor(1e-6, dtype=F32) * torch.tensor(0.5, dtype=F32)   # eps1 * 0.5
_SQRT2 = torch.tensor(math.sqrt(2.0), dtype=F32)
INV_SQRT_2PI = 1.0 / math.sqrt(2.0 * math.pi)
KL_EPS, KL_WEIGHT = 1e-6, 1.1


def probit_prob(u32, erf_fp64=False):
    """E = Normal(0,1).cdf(u)(1-eps1) + eps1/2 in float32, op by op (oracle.probit_prob).
    erf_fp64: erf(x) evaluated in float64 and rounded once to float32 (a
    correctly rounded fp32 erf) in place of torch's fp32 erf -- the same
    formula with another legitimate fp32 erf, to measure what one-ulp
    differences of E alone do to the gradients."""
    d = u32.device
    x = u32 / _SQRT2.to(d)
    erf = torch.erf(x.to(F64)).to(F32) if erf_fp64 else torch.erf(x)
    cdf = 0.5 * (1.0 + erf)
    return cdf * _C1.to(d) + _C0.to(d)


# The product's erf (mpvae-1_amd/csrc/mpv_common.h), restated op by op in fp32:
# the same formula E = 0.5 (1 + erf(u / sqrt 2)) (1 - eps1) + eps1 / 2 with
# erf = +-(1 - erfc(|z|)) from a Numerical-Recipes-form erfc, in the two forms
# the kernels use -- "p" (forward: t exp2(P(t) - zq^2)) and "q" (element pass:
# (t exp2(-zq^2)) Q(t)).  fp32 fmas are emulated in fp64 (exact product, then
# rounded), the hardware reciprocal and exp2 as correctly rounded fp32 -- so
# this is the kernels' erf up to those two instructions' last-bit error.
def _f32(v):
    import numpy as np
    return float(np.float32(v))


_KZQ = _f32(_f32(0.70710678118654752440) * _f32(1.2011224087864498))      # kZq
_HALF_SQ = _f32(0.5 / _f32(1.2011224087864498))                            # 0.5f / kSqL2e
_L2E = _f32(1.4426950408889634)
_ERFC_P = [_f32(_f32(c) * _L2E) for c in (-0.139353514, 0.777093824, -1.58356997, 1.19629222,
                                           -0.0702797193, 1.09342452, -1.27360696)]
_ERFC_Q = [_f32(c) for c in (0.0899837102, -0.359859836, 0.38748431, 0.0453561664, 0.275197459,
                             0.279788422, 0.282049996)]
_KEH = _f32(0.5 * float(_C1))


def _fma(a, b, c):
    return (a.to(F64) * b + c).to(F32) if torch.is_tensor(b) else (a.to(F64) * float(b) + c).to(F32)


def kernel_probit_prob(t32, base32, form):
    """E of the kernels' arithmetic from t and fe/fx (fp32): zq = fma(t, kZq,
    base kZq), w = 1 + erf through the form-p or form-q erfc, E = w kEh + C0
    rounded twice (contract off), as probit_w2xN_zq / probit_dw2xN_zq and their
    callers compute it."""
    zq = _fma(t32, _KZQ, (base32.to(F64) * _KZQ).to(F32).to(F64))
    den = _fma(zq.abs(), _HALF_SQ, 1.0)
    t = (1.0 / den.to(F64)).to(F32).to(F64)
    c = _ERFC_P if form == "p" else _ERFC_Q
    p = _fma(t, c[0], c[1])
    for ck in c[2:]:
        p = _fma(t, p.to(F64), ck)
    z64 = zq.to(F64)
    # om = 1 - erfc as one fma of the unrounded product (MPV_OM_FMA)
    if form == "p":
        a = (-z64 * z64 + p.to(F64)).to(F32)
        om = _fma(-t, torch.exp2(a.to(F64)).to(F32).to(F64), 1.0)
    else:
        ez = torch.exp2((-z64 * z64).to(F32).to(F64)).to(F32)
        om = _fma(-(t * ez.to(F64)).to(F32).to(F64), p.to(F64), 1.0)
    w = (1.0 + torch.copysign(om, zq).to(F64)).to(F32)
    return ((w.to(F64) * _KEH).to(F32).to(F64) + float(_C0)).to(F32)


def label_sets(y):
    pos, neg = (y == 1.0), (y == 0.0)
    n = pos.sum(1).to(F64) * neg.sum(1).to(F64)
    return pos, neg, n


class ChunkedElbo:
    """compute_loss (mpvae.py:145-210) forward and analytic backward over
    S-chunks.  ``noise(s0, s1)`` returns the (s1-s0, B, z) float32 noise of
    samples [s0, s1) on the inputs' device (it is called twice per chunk:
    forward and backward, and must return the same values)."""

    def __init__(self, y, fe_out, fx_out, R, noise, S, chunk=256, t_fp32=False, erf_fp64=False,
                 t_src=None, kernel_erf=False):
        self.y, self.fe, self.fx = y.to(F32), fe_out.to(F32), fx_out.to(F32)
        self.Rt = R.to(F32).to(F64).t().contiguous()          # R.T.float() (mpvae.py:165)
        self.noise, self.S, self.chunk = noise, int(S), int(chunk)
        # t_fp32: t from an fp32 GEMM, as the reference's own tensordot computes
        # it (mpvae.py:168-170), instead of fp64 accumulation rounded once --
        # measures how far fp32 arithmetic alone moves the results
        self.t_fp32 = bool(t_fp32)
        self.erf_fp64 = bool(erf_fp64)
        # kernel_erf: E by the product's own erf (kernel_probit_prob; form p in
        # the forward, form q in the backward, as the kernels use them)
        self.kernel_erf = bool(kernel_erf)
        # t_src(s0, s1) -> (s1-s0, B, L) float32: t supplied from outside (e.g.
        # the product's own T stash) instead of computed here -- the
        # reference's formulas evaluated on another implementation's t, to
        # separate what t's rounding does to the gradients from what the
        # arithmetic after t does
        self.t_src = t_src
        self.pos, self.neg, self.n = label_sets(self.y)
        self.y64 = self.y.to(F64)

    def _chunks(self):
        for s0 in range(0, self.S, self.chunk):
            yield s0, min(self.S, s0 + self.chunk)

    def _t(self, s0, s1):
        eps = self.noise(s0, s1)
        B, z = eps.shape[1], eps.shape[2]
        if self.t_src is not None:
            return self.t_src(s0, s1).to(F32), eps
        if self.t_fp32:
            t = eps.to(F32).reshape(-1, z) @ self.Rt.to(F32)
            return t.reshape(s1 - s0, B, -1), eps
        return (eps.to(F64).reshape(-1, z) @ self.Rt).reshape(s1 - s0, B, -1).to(F32), eps

    def _E(self, t, base, form):
        if self.kernel_erf:
            return kernel_probit_prob(t, base.expand_as(t), form)
        return probit_prob(t + base, self.erf_fp64)

    def _rows(self, E):
        E = E.to(F64)
        logp = (self.y64 * torch.log(E) + (1.0 - self.y64) * torch.log(1.0 - E)).sum(-1)
        P = (torch.exp(-5.0 * E) * self.pos).sum(-1)
        N = (torch.exp(5.0 * E) * self.neg).sum(-1)
        c = P * N / (5.0 * self.n)
        c = torch.where(torch.isfinite(c), c, torch.zeros_like(c))
        return logp, P, N, c

    def forward(self, fe_mu, fe_logvar, fx_mu, fx_logvar, nll_coeff, c_coeff):
        B, L = self.y.shape
        dev = self.y.device
        rows = torch.empty((6, B, self.S), dtype=F64, device=dev)   # oracle rowstat layout
        csum = torch.zeros((2,), dtype=F64, device=dev)
        colsum = torch.zeros((2, B, L), dtype=F64, device=dev)
        for s0, s1 in self._chunks():
            t, _ = self._t(s0, s1)
            for br, base in enumerate((self.fe, self.fx)):
                E = self._E(t, base, "p")
                logp, P, N, c = self._rows(E)
                rows[br, :, s0:s1] = logp.t()
                rows[2 + 2 * br, :, s0:s1] = P.t()
                rows[3 + 2 * br, :, s0:s1] = N.t()
                csum[br] += c.sum()
                colsum[br] += E.to(F64).sum(0)
        self.rowstat = rows
        m = rows[:2].amax(-1)                                      # (2, B)
        Z = torch.exp(rows[:2] - m[..., None]).sum(-1)
        self.m, self.Z = m, Z
        nll = (-torch.log(Z / self.S) - m).mean(-1)                # (2,)
        c = csum / (self.S * B)
        mu_e, lv_e, mu_x, lv_x = (a.to(F64) for a in (fe_mu, fe_logvar, fx_mu, fx_logvar))
        per = (lv_x - lv_e) - 1.0 + torch.exp(lv_e - lv_x) + (mu_x - mu_e) ** 2 / (
            torch.exp(lv_x) + KL_EPS)
        kl = (0.5 * per.sum(1)).mean()
        total = (nll[0] + nll[1]) * nll_coeff + (c[0] + c[1]) * c_coeff + kl * KL_WEIGHT
        return dict(total=total, nll=nll[0], nll_x=nll[1], c=c[0], c_x=c[1], kl=kl,
                    indiv_prob=colsum[1] / self.S, indiv_prob_label=colsum[0] / self.S)

    def backward(self, nll_coeff, c_coeff, g_total=1.0, g_I=None, g_IL=None):
        """Gradients of g_total * total (+ <g_I, indiv_prob> + <g_IL, indiv_prob_label>)
        w.r.t. fe_out, fx_out and r_sqrt_sigma (oracle.row_coefficients +
        oracle.shard_backward), float64."""
        B, L = self.y.shape
        dev = self.y.device
        gn, gc = nll_coeff * g_total, c_coeff * g_total
        dfe = torch.zeros((B, L), dtype=F64, device=dev)
        dfx = torch.zeros((B, L), dtype=F64, device=dev)
        dR = None
        scale = gc / (self.n * self.S * B)                          # (B,), inf where n == 0
        dead = self.n == 0
        for s0, s1 in self._chunks():
            t, eps = self._t(s0, s1)
            G = None
            for br, (base, gind, out) in enumerate(((self.fe, g_IL, dfe), (self.fx, g_I, dfx))):
                E = self._E(t, base, "q").to(F64)
                w = torch.exp(self.rowstat[br, :, s0:s1] - self.m[br][:, None]) / self.Z[br][:, None]
                a = (-gn * w / B).t()[..., None]                    # (s, B, 1)
                bP = (scale[:, None] * self.rowstat[3 + 2 * br, :, s0:s1]).t()[..., None]
                bN = (scale[:, None] * self.rowstat[2 + 2 * br, :, s0:s1]).t()[..., None]
                gE = a * (self.y64 / E - (1.0 - self.y64) / (1.0 - E))
                gE = gE - torch.where(self.pos, bP * torch.exp(-5.0 * E), 0.0) \
                    + torch.where(self.neg, bN * torch.exp(5.0 * E), 0.0)
                if dead.any():
                    gE = torch.where(dead[None, :, None], float("nan"), gE)
                if gind is not None:
                    gE = gE + gind.to(F64)[None] / self.S
                u = (t + base).to(F64)
                gu = gE * float(_C1) * INV_SQRT_2PI * torch.exp(-0.5 * u * u)
                out += gu.sum(0)
                G = gu if G is None else G + gu
            part = G.reshape(-1, L).t() @ eps.to(F64).reshape(-1, eps.shape[-1])
            dR = part if dR is None else dR + part
        return dict(fe_out=dfe, fx_out=dfx, r_sqrt_sigma=dR)
