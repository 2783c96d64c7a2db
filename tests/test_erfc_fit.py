"""The erfc polynomials the probit kernels use (mpv_common.h: kErfcDeg for the
forward's P form, kErfcxDeg for the element pass's Q form) hold the stated
accuracy: E = C0 + C1 Phi(u) from an fp32 emulation of the kernels'
evaluation, relative error <= 3e-6 over |u| <= 40 (NR's degree-9 fit in the
same emulation: 2.46e-6; all are set by the fp32 rounding of zq^2)."""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fit_erfc  # noqa: E402


def kernel_coefficients(fn, deg_name, scaled):
    src = open(os.path.join(ROOT, "mpvae-1_amd", "csrc", "mpv_common.h")).read()
    deg = int(re.search(r"constexpr int %s = (\d+);" % deg_name, src).group(1))
    body = src[src.index("MPV_DEV void %s" % fn):]
    arr = re.search(r"constexpr float c\[%s \+ 1\] = \{(.*?)\};" % deg_name, body, re.S).group(1)
    pat = r"(-?[0-9.]+(?:e-?[0-9]+)?)f \* kL2e" if scaled else r"(-?[0-9.]+(?:e-?[0-9]+)?)f"
    coef = [float(x) for x in re.findall(pat, arr)]
    assert len(coef) == deg + 1
    return coef


def test_forward_erfc_polynomial_accuracy():
    u = np.linspace(0, 40, 400001)
    ours = fit_erfc.e_rel_err(u, kernel_coefficients("probit_w2xN_zq", "kErfcDeg", True), "p")
    nr = fit_erfc.e_rel_err(u, fit_erfc.NR, "p")
    assert nr.max() < 2.6e-6
    assert ours.max() <= 3e-6, ours.max()
    # beyond the fitted range E is C0-dominated: no growth there
    assert ours[u > 6].max() < 1e-7


def test_backward_erfcx_polynomial_accuracy():
    u = np.linspace(0, 40, 400001)
    ours = fit_erfc.e_rel_err(u, kernel_coefficients("probit_dw2xN_zq", "kErfcxDeg", False), "q")
    assert ours.max() <= 3e-6, ours.max()
    assert ours[u > 6].max() < 1e-7
