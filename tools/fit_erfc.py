"""The erfc fit of the probit kernels (mpv_common.h, probit_w2xN_zq).

erfc(z) = t exp(-z^2 + P(t)), t = 1 / (1 + z/2).  Fits P of a given degree
over t >= tmin (the |u| range where E = C0 + C1 Phi(u) is not C0-dominated)
toward the minimax error, then emulates the kernel's fp32 evaluation (folded
log2 e constants, one rounding per fma) and reports E's relative error over
|u| <= 40 next to the degree-9 Numerical Recipes fit the kernels used before.

usage: python tools/fit_erfc.py [deg tmin]      (default: 6 0.38, the kernels' fit)
"""
import sys

import numpy as np
from scipy.special import erfc, erfcx

L2E = 1.4426950408889634
NR = [0.17087277, -0.82215223, 1.48851587, -1.13520398, 0.27886807,
      -0.18628806, 0.09678418, 0.37409196, 1.00002368, -1.26551223]
f32 = np.float32


def target(t):
    z = 2.0 * (1.0 / t - 1.0)
    return np.log(erfcx(z)) - np.log(t)


def fit(deg, tmin, iters=200, n=20000):
    """Lawson-style reweighted least squares on a Chebyshev grid; the best
    max-error iterate."""
    x = np.cos(np.pi * (np.arange(n) + 0.5) / n) * 0.5 * (1 - tmin) + 0.5 * (1 + tmin)
    y = target(x)
    w = np.ones_like(x)
    V = np.vander(x, deg + 1)
    best = None
    for _ in range(iters):
        c, *_ = np.linalg.lstsq(V * w[:, None], y * w, rcond=None)
        e = np.abs(V @ c - y)
        if best is None or e.max() < best[0]:
            best = (e.max(), c)
        w = w * (e / e.max() + 1e-4) ** 0.5
        w /= w.max()
    return best[1]


def kernel_erfc(u, coef):
    """fp32 emulation of the kernel: zq = u kZq, t = rcp(fma(0.5/sqrt(log2 e),
    |zq|, 1)), Horner in fp32 fmas, erfc = t exp2(fma(-zq, zq, P))."""
    sq = f32(1.2011224087864498)
    kz = f32(0.70710678118654752440) * sq
    zq = (u.astype(f32) * kz).astype(f32)
    den = (f32(0.5) / sq * np.abs(zq).astype(np.float64) + 1.0).astype(f32)
    t = (1.0 / den.astype(np.float64)).astype(f32).astype(np.float64)
    c = [float(f32(x * L2E)) for x in coef]
    p = (t * c[0] + c[1]).astype(f32)
    for k in range(2, len(c)):
        p = (t * p + c[k]).astype(f32)
    a = (-(zq.astype(np.float64)) * zq + p).astype(f32)
    return t * np.exp2(a.astype(np.float64)).astype(f32)


def main():
    deg = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    tmin = float(sys.argv[2]) if len(sys.argv) > 2 else 0.38
    coef = fit(deg, tmin)
    c1, c0 = float(f32(1 - 1e-6)), float(f32(0.5e-6))
    u = np.linspace(0, 40, 800001)  # E at -u (the small side)
    e_true = c0 + c1 * 0.5 * erfc(u / np.sqrt(2))
    for name, cf in (("NR degree 9", NR), (f"degree {deg}, t >= {tmin}", coef)):
        e = np.abs((c0 + c1 * 0.5 * kernel_erfc(u, cf)) / e_true - 1)
        print(f"{name:22s} E rel err: max {e.max():.2e}, |u|<=3 {e[u <= 3].max():.2e}, "
              f"3<|u|<=6 {e[(u > 3) & (u <= 6)].max():.2e}, |u|>6 {e[u > 6].max():.2e}")
    print("coefficients (highest degree first):", ", ".join("%.9g" % x for x in coef))


if __name__ == "__main__":
    main()
