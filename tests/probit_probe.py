"""The product's probit E, read back through the product forward on controlled
arguments -- TEST INFRASTRUCTURE.

The forward kernels never publish E itself; what they publish is
indiv_prob_label = (1/S) sum_s E[s, b, l] (and indiv_prob for the feature
branch), the column sums of the very E they feed into the BCE and ranking
terms (probit_fwd.hip, fwd_tile_epilogue_t: ce += wr * E4).  With n_sample
S = 1 that column sum is one E, and dividing by S = 1 is exact, so

    indiv_prob_label[b, l] = E(t[b, l], fe_out[b, l])

bit for bit, where t is the noise product the kernel computed.  Two ways to
control t:

* ``product_E(base)``: r_sqrt_sigma = 0, so t = 0 exactly and the kernel's
  argument is zq = fma(0, kZq, fe_out kZq) = fl(fe_out kZq) -- the E of u =
  fe_out (mpvae.py:168-180 with a zero residual covariance factor);
* ``product_E(base, t)``: an arbitrary fp32 t, made exact on the f16 matrix
  cores: z = 2L noise columns, r_sqrt_sigma[l, l] = r_sqrt_sigma[l, L+l] = 1
  (2^-k, with t scaled by 2^k, for the small |t|: product_E),
  noise[.., l] = t with its 2 low mantissa bits cleared (22 significant bits:
  its hi and lo f16 halves hold it exactly), noise[.., L+l] = those 2 bits.
  Each MFMA then adds at most one nonzero exact product per output (the two
  pieces sit in different 32-wide K blocks; R's lo half is zero), and every
  partial sum is a sum of disjoint bit pieces of t, so the kernel's t is the
  given t.  (With both pieces in one K block the MFMA's internal alignment of
  its products dropped the 2-bit piece.)  The T stash is read back and
  compared bit for bit, so the claim is checked, not assumed.

Reference values: ``cr_E`` (the exact E = Phi(u)(1 - eps1) + eps1/2 with the
reference's fp32 constants, from float64 ndtr, rounded once to fp32: correctly
rounded up to a double rounding at a fp32 midpoint, probability ~2^-29 per
value) and ``ref_E`` (the reference's own fp32 op order with torch's erf,
tests/torch64_ref.probit_prob).  Only tests import this module.
"""
import argparse

import torch

import mpvae
from mpvae_ops import HipShardBackend
from torch64_ref import _C0, _C1, probit_prob

F32, F64 = torch.float32, torch.float64


def cr_E(u64):
    """Correctly rounded fp32 E of an exact (float64) argument u."""
    return (torch.special.ndtr(u64) * float(_C1) + float(_C0)).to(F32)


def ref_E(u32):
    """The reference's fp32 E of an fp32 argument (mpvae.py:171-180, torch erf)."""
    return probit_prob(u32)


def ulps(a, b):
    """|a - b| in fp32 ulps for positive fp32 tensors (E is always >= eps1/2)."""
    return (a.view(torch.int32).to(torch.int64) - b.view(torch.int32).to(torch.int64)).abs()


def _exact_t_operands(t, B, L, k):
    """(R (L, 2L) fp64, noise (1, B, 2L) fp32) whose 3xf16 product is t (B, L)
    exactly, for |t| within 2^13 of the call's max |t| (see product_E):
    noise holds t 2^k, r_sqrt_sigma 2^-k (k a multiple of 12, exact scalings)."""
    ts = t * (2.0 ** k)                             # exact (fp32 power of two, k <= 120)
    hi = (ts.view(torch.int32) & ~0x3).view(F32)   # 2 low mantissa bits cleared
    lo = ts - hi                                    # exact: the cleared bits
    noise = torch.cat((hi, lo), -1).reshape(1, B, 2 * L).contiguous()
    R = torch.zeros((L, 2 * L), dtype=F64, device=t.device)
    idx = torch.arange(L, device=t.device)
    R[idx, idx] = 2.0 ** -k
    R[idx, L + idx] = 2.0 ** -k
    return R, noise


def _product_E_once(base, t, L, gemm, k):
    N = base.numel()
    B = N // L
    dev = base.device
    fe = base.reshape(B, L).contiguous()
    y = torch.zeros((B, L), device=dev)
    mu = torch.zeros((B, 1), device=dev)
    if t is None:
        z = 32
        R = torch.zeros((L, z), dtype=F64, device=dev)
        noise = torch.zeros((1, B, z), device=dev)
    else:
        z = 2 * L
        R, noise = _exact_t_operands(t.reshape(B, L), B, L, k)
        be = HipShardBackend(gemm)
        shape = be.shape(1, 1, 0, B, L, z)
        T = be.forward_local(shape, y, fe, fe, be.prepare_R(R), be.prepare_noise(noise, shape),
                             keep_T=True)["T"]
        got = T[:, 0, :L].reshape(-1)
        bad = got.view(torch.int32) != t.reshape(-1).view(torch.int32)
        assert not bool(bad.any()), ("the crafted operands did not reproduce t exactly", k,
                                     int(bad.sum()), t.reshape(-1)[bad][:4].tolist(),
                                     got[bad][:4].tolist())
        del T, got
    args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=1, n_test_sample=1,
                              mode="test", nll_coeff=0.5, c_coeff=10.0, mpvae_noise=noise,
                              mpvae_gemm=gemm)
    out = mpvae.compute_loss(y, fe, mu, mu, fe, mu, mu, R, args)
    return out[7].reshape(-1), out[6].reshape(-1)


def product_E(base, t=None, L=1024, gemm="f16x3"):
    """E(t, base) of the product forward for fp32 device tensors base (N,) and
    t (N,) or None (t = 0), N a multiple of L when t is None.  Returns (E label
    branch, E feature branch); both branches get the same base, so they must
    agree.  t given: the T stash is checked to hold t bit for bit.

    The split operands hold a value exactly only down to 2^-14 of their
    operand's max |x| (fp16 subnormals below), so the elements go in windows
    of 12 binades of |t|, one launch per window present, each with t scaled
    by 2^12j into the top window and r_sqrt_sigma by 2^-12j (exact)."""
    N = base.numel()
    if t is None:
        assert N % L == 0, (N, L)
        return _product_E_once(base, None, L, gemm, 0)
    t = t.reshape(-1).contiguous()
    e = torch.frexp(t).exponent
    e_max = int(e[t != 0].max()) if bool((t != 0).any()) else 0
    # windows below 2^-60 of the max would need scalings beyond fp32's range
    # in the GEMM's operand scales; no such t has been met (the T stash check
    # below would say so)
    j = torch.where(t != 0, torch.div(e_max - e, 12, rounding_mode="floor"), 0).clamp_max(5)
    E = torch.empty((N,), dtype=F32, device=base.device)
    Ex = torch.empty_like(E)
    for jj in torch.unique(j).tolist():
        idx = torch.nonzero(j == jj).flatten()
        n = idx.numel()
        npad = (n + L - 1) // L * L
        bb = torch.zeros((npad,), dtype=F32, device=base.device)
        tt = torch.zeros((npad,), dtype=F32, device=base.device)
        bb[:n], tt[:n] = base.reshape(-1)[idx], t[idx]
        a, ax = _product_E_once(bb, tt, L, gemm, 12 * int(jj))
        E[idx], Ex[idx] = a[:n], ax[:n]
    return E, Ex


def steps(a, e_cr):
    """|a - e_cr| in steps of the fp32 grid the reference's formula puts E on
    (mpvae.py:171-180): cdf = 0.5 (1 + erf(x)) with erf rounded to fp32, so
    below E = 0.5 the grid of E is half an fp32 ulp of |erf| = |1 - 2 cdf|
    (up to 2^19 ulps of E near the eps1/2 floor), above it one ulp of E."""
    e = e_cr.to(F64)
    ulp_e = torch.ldexp(torch.ones_like(e), torch.frexp(e).exponent - 24)
    a_erf = (1.0 - 2.0 * e).abs().clamp_min(1e-300)
    ulp_erf = torch.ldexp(torch.ones_like(e), torch.frexp(a_erf).exponent - 24)
    step = torch.where(e < 0.5, torch.maximum(ulp_e, 0.5 * ulp_erf), ulp_e)
    return (a.to(F64) - e).abs() / step


STEP_BINS = (0.0, 0.5, 1.0, 1.5, 2.0, 4.0, 1e30)


def hist_steps(d):
    edges = torch.tensor(STEP_BINS, device=d.device, dtype=F64)
    return torch.bincount(torch.bucketize(d, edges), minlength=len(STEP_BINS)).cpu()


# ulp histogram bins (upper edges, inclusive)
BINS = (0, 1, 2, 3, 4, 8, 16, 32, 64, 128, 256, 1 << 30)


def hist(d):
    """Counts of ulp distances d per BINS bucket."""
    edges = torch.tensor(BINS, device=d.device, dtype=torch.int64)
    return torch.bincount(torch.bucketize(d, edges), minlength=len(BINS)).cpu()


def bands(e_cr):
    """Masks of the three E bands: floor (E < 1e-4), mid, top (1 - E < 1e-4:
    where one fp32 ulp of E is >= 6e-4 of 1 - E and BCE's log(1 - E) sees it)."""
    lo = e_cr < 1e-4
    hi = (1.0 - e_cr.to(F64)) < 1e-4
    return {"floor": lo, "mid": ~(lo | hi), "top": hi}


# Stated bounds on the kernels' E against the correctly rounded E, per band
# (measured on the MI355X over every fp32 u in [-9, 9]:
# tests/test_gpu_probit_ulp.py, profiles/r06_probit_ulp.json):
#   top   1 - E < 1e-4 (u > 3.72), where the C4 / C5 gradients are sensitive
#         to one ulp of E: <= 1 fp32 ulp of E, as the
#         reference's own fp32 arithmetic (torch's erf, CPU and GPU: 1);
#   floor E < 1e-4 (u < -3.72): in steps of the fp32 grid the reference's
#         formula puts E on (``steps``: 0.5 (1 + erf) with erf in fp32 holds E
#         to half an ulp of |erf|, up to 2^19 ulps of E at the eps1/2 floor):
#         <= 0.51 (measured 0.503; the reference's fp32 0.504 GPU, 0.545 CPU);
#   mid   the rest: <= 14 steps (13 over the sweep on the 256-label tile,
#         12 / 7 on the others; 14 on the C5 rows of test_gpu_parity.py,
#         where the argument is fma(t, kZq, base kZq) with t != 0; the
#         reference's fp32: 2.25).  The kernels form erf as 1 - erfc, so near
#         u = 0 (E ~ 0.5) E carries erfc's fp32 rounding: <= 4.5e-7 absolute,
#         9e-7 relative; a degree-8 fit still leaves 9 (tools/fit_erfc.py),
#         so it is the form, not the fit.  Where one ulp matters (top) the
#         form is as exact as the reference's arithmetic: 1 ulp.
BOUNDS = {"top": ("ulp", 1), "mid": ("step", 14.0), "floor": ("step", 0.51)}


def band_max(a, e_cr):
    """{band/unit: max distance} of fp32 E values a from the correctly rounded e_cr."""
    out = {}
    for band, m in bands(e_cr).items():
        out[f"{band}/ulp"] = float(ulps(a[m], e_cr[m]).max()) if m.any() else 0.0
        out[f"{band}/step"] = float(steps(a[m], e_cr[m]).max()) if m.any() else 0.0
    return out


def within_bounds(mx):
    """The band maxima mx (band_max) within BOUNDS: list of violations."""
    return [(band, unit, mx[f"{band}/{unit}"], bound) for band, (unit, bound) in BOUNDS.items()
            if bound is not None and mx[f"{band}/{unit}"] > bound]


def elem_outside(c):
    """One element record (E, E_ref, E_cr, ulp_*, step_*): is either fp32
    evaluation outside BOUNDS for its band?"""
    band = "top" if 1.0 - c["E_cr"] < 1e-4 else ("floor" if c["E_cr"] < 1e-4 else "mid")
    unit, bound = BOUNDS[band]
    if bound is None:
        return False
    return max(c[f"{unit}_kernel"], c[f"{unit}_ref"]) > bound
