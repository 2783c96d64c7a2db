"""CPU: the S-chunked torch fp64 restatement (tests/torch64_ref.py, used by the
full-C4 GPU parity test) against the numpy oracle it restates
(oracle/probit_elbo.py), which is itself pinned to the reference's golden
vectors (tests/test_oracle_golden.py)."""
import numpy as np
import pytest
import torch

from oracle import probit_elbo as pe
from tolerances import rel_err
from torch64_ref import ChunkedElbo

OUTS = ["total", "nll", "nll_x", "c", "c_x", "kl", "indiv_prob", "indiv_prob_label"]


def _case(L, z, B, S, d, seed, degenerate=False):
    rng = np.random.default_rng(seed)
    y = (rng.random((B, L)) < 0.25).astype(np.float32)
    y[:, 0], y[:, 1] = 1, 0
    if degenerate:
        y[1] = 0.0
        y[2] = 1.0
    f32 = lambda a: a.astype(np.float32)
    inp = dict(y=y, fe_out=f32(rng.standard_normal((B, L))), fx_out=f32(rng.standard_normal((B, L))),
               fe_mu=f32(rng.standard_normal((B, d))), fe_logvar=f32(0.3 * rng.standard_normal((B, d))),
               fx_mu=f32(rng.standard_normal((B, d))), fx_logvar=f32(0.3 * rng.standard_normal((B, d))),
               r_sqrt_sigma=rng.uniform(-1, 1, (L, z)) * np.sqrt(6.0 / (L + z)))
    noise = f32(rng.standard_normal((S, B, z)))
    return inp, noise


@pytest.mark.parametrize("L,z,B,S,chunk,degenerate", [(38, 38, 8, 40, 16, False),
                                                      (100, 37, 5, 33, 7, False),
                                                      (25, 10, 6, 20, 20, True)])
@pytest.mark.parametrize("with_gI", [False, True])
def test_chunked_torch64_matches_numpy_oracle(L, z, B, S, chunk, degenerate, with_gI):
    inp, noise = _case(L, z, B, S, 8, L + S, degenerate)
    rng = np.random.default_rng(1)
    g_I = rng.standard_normal((B, L)).astype(np.float32) if with_gI else None
    g_IL = rng.standard_normal((B, L)).astype(np.float32) if with_gI else None
    ref = pe.elbo_forward(inp["y"], inp["fe_out"], inp["fe_mu"], inp["fe_logvar"], inp["fx_out"],
                          inp["fx_mu"], inp["fx_logvar"], inp["r_sqrt_sigma"], noise, 0.1, 200.0)
    rg = pe.elbo_backward(ref, inp["y"], inp["fe_out"], inp["fe_mu"], inp["fe_logvar"],
                          inp["fx_out"], inp["fx_mu"], inp["fx_logvar"], noise, 0.1, 200.0,
                          g_total=1.0, g_I=g_I, g_IL=g_IL)
    t = {k: torch.from_numpy(v) for k, v in inp.items()}
    nz = torch.from_numpy(noise)
    ce = ChunkedElbo(t["y"], t["fe_out"], t["fx_out"], t["r_sqrt_sigma"], lambda a, b: nz[a:b], S,
                     chunk)
    out = ce.forward(t["fe_mu"], t["fe_logvar"], t["fx_mu"], t["fx_logvar"], 0.1, 200.0)
    # torch's fp32 erf and scipy's differ by one ulp on ~1.5 % of the elements
    # (measured: forward <= 1.1e-8, gradients <= 3.6e-8), 100x below the
    # product's tolerances (tolerances.py)
    for k in OUTS:
        assert rel_err(out[k].numpy(), ref[k]) <= 5e-8, k
    g = ce.backward(0.1, 200.0, 1.0, None if g_I is None else torch.from_numpy(g_I),
                    None if g_IL is None else torch.from_numpy(g_IL))
    for k in ("fe_out", "fx_out", "r_sqrt_sigma"):
        assert rel_err(g[k].numpy(), rg[k]) <= 2e-7, k


def test_external_t_source_reproduces_own_t():
    """t_src (the reference's formulas on another implementation's t, used by
    the full-size GPU tests on the product's T stash): fed the restatement's
    own fp64-accumulated t, chunk by chunk, it gives the same results bit for
    bit; fed the fp32-GEMM t, the same as t_fp32=True."""
    L, z, B, S = 40, 24, 6, 30
    inp, noise = _case(L, z, B, S, 8, 7)
    t = {k: torch.from_numpy(v) for k, v in inp.items()}
    nz = torch.from_numpy(noise)
    mk = lambda **kw: ChunkedElbo(t["y"], t["fe_out"], t["fx_out"], t["r_sqrt_sigma"],
                                  lambda a, b: nz[a:b], S, 8, **kw)
    for kw in ({}, {"t_fp32": True}):
        own = mk(**kw)
        ext = mk(t_src=lambda a, b, o=own: o._t(a, b)[0])
        mus = (t["fe_mu"], t["fe_logvar"], t["fx_mu"], t["fx_logvar"], 0.1, 200.0)
        fa, fb = own.forward(*mus), ext.forward(*mus)
        for k in OUTS:
            assert torch.equal(fa[k], fb[k]), (kw, k)
        ga, gb = own.backward(0.1, 200.0), ext.backward(0.1, 200.0)
        for k in ("fe_out", "fx_out", "r_sqrt_sigma"):
            assert torch.equal(ga[k], gb[k]), (kw, k)


def test_kernel_erf_restatement_is_the_same_probit():
    """kernel_probit_prob (the product's erf and argument rounding, both forms)
    is the reference's E up to its fp32 rounding: the kernels round the
    probit's argument differently (zq = fma(t, kZq, base kZq) instead of
    u = t + base, then u / sqrt 2), which moves E by phi(u) times an ulp or two
    of u (<= 5e-7 absolute, <= 5e-6 relative for 0.01 < E < 0.99)."""
    from torch64_ref import kernel_probit_prob, probit_prob
    g = torch.Generator().manual_seed(0)
    t = torch.randn(200000, generator=g) * 1.2
    base = torch.randn(200000, generator=g)
    E = probit_prob(t + base).double()
    for form in ("p", "q"):
        Ek = kernel_probit_prob(t, base, form).double()
        assert float((Ek - E).abs().max()) <= 5e-7
        mid = (E > 0.01) & (E < 0.99)
        assert float(((Ek - E).abs() / E)[mid].max()) <= 5e-6
