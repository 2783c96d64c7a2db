"""The erfc fits of the probit kernels (mpv_common.h).

Two forms, both with t = 1 / (1 + z/2), z = |u| / sqrt 2:
  p: erfc(z) = t exp(-z^2 + P(t))   (forward epilogue, probit_w2xN_zq: one
     exponential, P in log2 units)
  q: erfc(z) = t exp(-z^2) Q(t)     (element pass, probit_dw2xN_zq: exp(-z^2)
     is needed for phi anyway, so Q = erfcx(z) / t saves the second one)
Fits the polynomial of a given degree over t >= tmin (the |u| range where
E = C0 + C1 Phi(u) is not C0-dominated) toward the minimax error, emulates
the kernel's fp32 evaluation (one rounding per fma) and reports E's relative
error over |u| <= 40 next to the degree-9 Numerical Recipes fit (form p).

usage: python tools/fit_erfc.py [p|q] [deg tmin]   (defaults: the kernels' fits)
"""
import sys

import numpy as np
from scipy.special import erfc, erfcx

L2E = 1.4426950408889634
NR = [0.17087277, -0.82215223, 1.48851587, -1.13520398, 0.27886807,
      -0.18628806, 0.09678418, 0.37409196, 1.00002368, -1.26551223]
f32 = np.float32


def target(t, form="p"):
    z = 2.0 * (1.0 / t - 1.0)
    if form == "q":
        return erfcx(z) / t
    return np.log(erfcx(z)) - np.log(t)


def fit(deg, tmin, form="p", iters=200, n=20000):
    """Lawson-style reweighted least squares on a Chebyshev grid (relative
    error for form q); the best max-error iterate."""
    x = np.cos(np.pi * (np.arange(n) + 0.5) / n) * 0.5 * (1 - tmin) + 0.5 * (1 + tmin)
    y = target(x, form)
    scale = np.abs(y) if form == "q" else np.ones_like(y)
    w = 1.0 / scale
    V = np.vander(x, deg + 1)
    best = None
    for _ in range(iters):
        c, *_ = np.linalg.lstsq(V * w[:, None], y * w, rcond=None)
        e = np.abs(V @ c - y) / scale
        if best is None or e.max() < best[0]:
            best = (e.max(), c)
        w = w * (e / e.max() + 1e-4) ** 0.5
        w /= w.max()
    return best[1]


def kernel_erfc(u, coef, form="p"):
    """fp32 emulation of the kernels: zq = u kZq, t = rcp(fma(0.5/sqrt(log2 e),
    |zq|, 1)), Horner in fp32 fmas; form p: erfc = t exp2(fma(-zq, zq, P)),
    form q: erfc = (t exp2(-zq^2)) Q."""
    sq = f32(1.2011224087864498)
    kz = f32(0.70710678118654752440) * sq
    zq = (u.astype(f32) * kz).astype(f32)
    den = (f32(0.5) / sq * np.abs(zq).astype(np.float64) + 1.0).astype(f32)
    t = (1.0 / den.astype(np.float64)).astype(f32).astype(np.float64)
    c = [float(f32(x * (L2E if form == "p" else 1.0))) for x in coef]
    p = (t * c[0] + c[1]).astype(f32)
    for k in range(2, len(c)):
        p = (t * p + c[k]).astype(f32)
    if form == "q":
        ez = np.exp2((-(zq.astype(np.float64)) * zq).astype(f32)).astype(f32)
        return ((t * ez).astype(f32).astype(np.float64) * p).astype(f32).astype(np.float64)
    a = (-(zq.astype(np.float64)) * zq + p).astype(f32)
    return t * np.exp2(a.astype(np.float64)).astype(f32)


DEFAULTS = {"p": (6, 0.38), "q": (6, 0.38)}


def e_rel_err(u, coef, form="p"):
    c1, c0 = float(f32(1 - 1e-6)), float(f32(0.5e-6))
    e_true = c0 + c1 * 0.5 * erfc(u / np.sqrt(2))
    return np.abs((c0 + c1 * 0.5 * kernel_erfc(u, coef, form)) / e_true - 1)


def main():
    form = sys.argv[1] if len(sys.argv) > 1 else "p"
    deg, tmin = DEFAULTS[form]
    if len(sys.argv) > 3:
        deg, tmin = int(sys.argv[2]), float(sys.argv[3])
    coef = fit(deg, tmin, form)
    u = np.linspace(0, 40, 800001)  # E at -u (the small side)
    for name, cf, fm in (("NR degree 9 (p)", NR, "p"), (f"{form} degree {deg}, t >= {tmin}", coef, form)):
        e = e_rel_err(u, cf, fm)
        print(f"{name:24s} E rel err: max {e.max():.2e}, |u|<=3 {e[u <= 3].max():.2e}, "
              f"3<|u|<=6 {e[(u > 3) & (u <= 6)].max():.2e}, |u|>6 {e[u > 6].max():.2e}")
    print("coefficients (highest degree first):", ", ".join("%.9g" % x for x in coef))


if __name__ == "__main__":
    main()
