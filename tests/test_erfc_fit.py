"""The erfc polynomial the probit kernels use (mpv_common.h, kErfcDeg) holds
the stated accuracy: E = C0 + C1 Phi(u) from an fp32 emulation of the
kernel's evaluation, relative error <= 3e-6 over |u| <= 40 (NR's degree-9 fit
in the same emulation: 2.46e-6; both are set by the fp32 rounding of zq^2)."""
import os
import re
import sys

import numpy as np
from scipy.special import erfc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fit_erfc  # noqa: E402


def kernel_coefficients():
    src = open(os.path.join(ROOT, "mpvae-1_amd", "csrc", "mpv_common.h")).read()
    deg = int(re.search(r"constexpr int kErfcDeg = (\d+);", src).group(1))
    body = src[src.index("MPV_DEV void probit_w2xN_zq"):]
    arr = re.search(r"constexpr float c\[kErfcDeg \+ 1\] = \{(.*?)\};", body, re.S).group(1)
    coef = [float(x) for x in re.findall(r"(-?[0-9.]+(?:e-?[0-9]+)?)f \* kL2e", arr)]
    assert len(coef) == deg + 1
    return coef


def e_rel_err(coef, u):
    f32 = np.float32
    c1, c0 = float(f32(1 - 1e-6)), float(f32(0.5e-6))
    e_true = c0 + c1 * 0.5 * erfc(u / np.sqrt(2))
    return np.abs((c0 + c1 * 0.5 * fit_erfc.kernel_erfc(u, coef)) / e_true - 1)


def test_kernel_erfc_polynomial_accuracy():
    u = np.linspace(0, 40, 400001)
    ours = e_rel_err(kernel_coefficients(), u)
    nr = e_rel_err(fit_erfc.NR, u)
    assert nr.max() < 2.6e-6
    assert ours.max() <= 3e-6, ours.max()
    # beyond the fitted range E is C0-dominated: no growth there
    assert ours[u > 6].max() < 1e-7


def test_both_dw_and_w_use_the_same_coefficients():
    src = open(os.path.join(ROOT, "mpvae-1_amd", "csrc", "mpv_common.h")).read()
    arrs = re.findall(r"constexpr float c\[kErfcDeg \+ 1\] = \{(.*?)\};", src, re.S)
    assert len(arrs) == 2 and arrs[0] == arrs[1]
