"""The kernels' probit E pinned on the device, value by value (VERDICT r05
item 1; reference mpvae.py:171-180).

Every fp32 u in [-9, 9] (2.18e9 values; E is within 1.2e-19 of eps1/2 or of
1 - eps1/2 beyond) goes through the product forward as fe_out with a zero
r_sqrt_sigma and n_sample = 1, so that indiv_prob_label is the kernels' E of u
(tests/probit_probe.py).  Each E is compared, in fp32 ulps, with

  * the correctly rounded E (float64 ndtr, rounded once), and
  * the reference's own fp32 arithmetic (torch's erf in mpvae.py's op order)
    on the device, and on the host CPU for the two tails |u| > 3.7 in full
    plus every 61st value between;
  * the op-by-op restatement of the kernels' erf that tests/torch64_ref.py
    uses (kernel_probit_prob, form p), to pin that emulation to the device.

The histograms go to $MPVAE_RECORD_ERRS; the asserted bounds per E band are
probit_probe.BOUNDS ("The probit, pinned").  The 256-label
tile (C4, C5) takes the whole sweep; the other forward tiles (48-, 96-,
128-label, and the exact-fp32 mode's) a 1-in-257 subset plus the whole top
band, where one ulp of E is the largest part of 1 - E.
"""
import json

import pytest
import torch

from probit_probe import (BINS, BOUNDS, F32, F64, STEP_BINS, bands, cr_E, hist, hist_steps, product_E,
                          ref_E, steps, ulps)
from tolerances import record
from torch64_ref import kernel_probit_prob

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
U_MAX_BITS = 0x41100000          # 9.0f
CHUNK = 1 << 24

def _assert_bounds(s, tag="kernel_vs_cr"):
    for band, (unit, bound) in BOUNDS.items():
        if bound is None:
            continue
        got = s["max"][f"{tag}/{band}/{unit}"]
        assert got <= bound, (band, unit, got, bound, s["max"])


def _values(lo_bits, hi_bits, sign):
    x = torch.arange(lo_bits, hi_bits, dtype=torch.int32, device=DEV).view(F32)
    return -x if sign else x


def _sweep_chunks(stride=1):
    for sign in (0, 1):
        for a in range(0, U_MAX_BITS + 1, CHUNK):
            b = min(a + CHUNK, U_MAX_BITS + 1)
            u = _values(a, b, sign)
            if stride > 1:
                u = u[::stride]
            yield u


def _top_band(sign=0):
    """Every fp32 u in (3.7, 9]: 1 - E < 1.1e-4."""
    a = int(torch.tensor(3.7, dtype=F32).view(torch.int32))
    return _values(a, U_MAX_BITS + 1, sign)


def _pad(u, L):
    n = (u.numel() + L - 1) // L * L
    return torch.cat((u, torch.zeros(n - u.numel(), dtype=F32, device=DEV))) if n > u.numel() \
        else u


class _Stats:
    def __init__(self):
        self.h = {}
        self.mx = {}
        self.n = 0

    def add(self, tag, band, d, unit="ulp"):
        key = f"{tag}/{band}/{unit}"
        h = hist(d) if unit == "ulp" else hist_steps(d)
        self.h[key] = self.h.get(key, torch.zeros_like(h)) + h
        m = float(d.max()) if d.numel() else 0.0
        self.mx[key] = max(self.mx.get(key, 0.0), m)

    def add_cr(self, tag, band, a, e_cr):
        """ulps and reference-grid steps of a against the correctly rounded E."""
        self.add(tag, band, ulps(a, e_cr))
        self.add(tag, band, steps(a, e_cr), "step")

    def summary(self):
        return {"max": self.mx, "hist_bins_le": {"ulp": list(BINS), "step": list(STEP_BINS)},
                "hist": {k: [int(x) for x in v] for k, v in self.h.items()}, "n": self.n}


def _compare(st, u, L, gemm="f16x3", emul=True, cpu_ref=False):
    up = _pad(u, L)
    E, Ex = product_E(up, L=L, gemm=gemm)
    E, Ex = E[:u.numel()], Ex[:u.numel()]
    assert torch.equal(E.view(torch.int32), Ex.view(torch.int32)), "branches differ"
    ecr = cr_E(u.to(F64))
    eref = ref_E(u)
    em = kernel_probit_prob(torch.zeros_like(u), u, "p") if emul else None
    st.n += u.numel()
    for band, m in bands(ecr).items():
        st.add_cr("kernel_vs_cr", band, E[m], ecr[m])
        st.add_cr("ref_gpu_vs_cr", band, eref[m], ecr[m])
        st.add("kernel_vs_ref_gpu", band, ulps(E[m], eref[m]))
        if em is not None:
            st.add("kernel_vs_emulation", band, ulps(E[m], em[m]))
    if cpu_ref:
        sel = (u.abs() > 3.7) | (torch.arange(u.numel(), device=DEV) % 61 == 0)
        ecpu = ref_E(u[sel].cpu()).to(DEV)
        for band, m in bands(ecr[sel]).items():
            st.add_cr("ref_cpu_vs_cr", band, ecpu[m], ecr[sel][m])
            st.add("kernel_vs_ref_cpu", band, ulps(E[sel][m], ecpu[m]))


@pytest.mark.timeout(900)
def test_probit_every_fp32_argument_256_label_tile():
    """All 2.18e9 fp32 u in [-9, 9] through the C4 / C5 forward tile."""
    st = _Stats()
    for u in _sweep_chunks():
        _compare(st, u, 1024, cpu_ref=True)
    s = st.summary()
    print(json.dumps(s["max"]))
    record("probit_ulp_fwd16a", s["max"])
    record("probit_ulp_fwd16a_hist", {f"{k}|{i}": float(c) for k, h in s["hist"].items()
                                      for i, c in enumerate(h)})
    _assert_bounds(s)
    assert s["n"] == 2 * (U_MAX_BITS + 1)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("L,gemm,tile", [(38, "f16x3", "fwd16"), (81, "f16x3", "fwd16t"),
                                         (128, "f16x3", "fwd16a_128"), (1024, "f32", "fwd_f32")])
def test_probit_other_forward_tiles(L, gemm, tile):
    """The other forward tiles on a 1-in-257 subset of [-9, 9] plus the whole
    top band (both signs of it: u > 3.7 and u < -3.7)."""
    st = _Stats()
    for u in _sweep_chunks(stride=257):
        _compare(st, u, L, gemm=gemm, emul=False)
    for sign in (0, 1):
        _compare(st, _top_band(sign), L, gemm=gemm, emul=False)
    s = st.summary()
    print(tile, json.dumps(s["max"]))
    record(f"probit_ulp_{tile}", s["max"])
    _assert_bounds(s)


@pytest.mark.timeout(300)
def test_probit_with_exact_noise_product():
    """E(t, base) for an arbitrary fp32 t (the kernels' argument is then
    fma(t, kZq, base kZq), not fl(base kZq)): t made exact on the matrix cores
    (probit_probe._exact_t_operands; the T stash is checked bit for bit), E
    against the correctly rounded E of the exact u = t + base."""
    g = torch.Generator(device=DEV).manual_seed(606)
    L, B = 1024, 2048
    t = torch.randn((B * L,), device=DEV, generator=g)
    base = torch.randn((B * L,), device=DEV, generator=g) * 2.0
    E, Ex = product_E(base, t=t, L=L)
    assert torch.equal(E.view(torch.int32), Ex.view(torch.int32))
    ecr = cr_E(t.to(F64) + base.to(F64))
    st = _Stats()
    eref = ref_E(t + base)
    for band, m in bands(ecr).items():
        st.add_cr("kernel_vs_cr", band, E[m], ecr[m])
        st.add_cr("ref_gpu_vs_cr", band, eref[m], ecr[m])
    s = st.summary()
    print(json.dumps(s["max"]))
    record("probit_ulp_exact_t", s["max"])
    _assert_bounds(s)
