"""Pin the CPU oracle against the reference's own outputs (golden vectors made
by importing /root/reference/mpvae.py, tests/golden/make_golden.py) and the
Philox oracle against the published Random123 known-answer vectors."""
import numpy as np
import pytest

from golden_io import OUTS, PART_KEYS, fixtures
from oracle import philox, probit_elbo as pe
from tolerances import (EXTREME_FWD_RTOL, EXTREME_GRAD_RTOL, FWD_RTOL, GRAD_RTOL, rel_err)

FIX = fixtures()


def _fwd(f, ranking, shards):
    return pe.elbo_forward(f["y"], f["fe_out"], f["fe_mu"], f["fe_logvar"], f["fx_out"],
                           f["fx_mu"], f["fx_logvar"], f["r_sqrt_sigma"], f["noise"],
                           f.nll_coeff, f.c_coeff, ranking=ranking, shards=shards)


@pytest.mark.parametrize("f", FIX, ids=[f.name for f in FIX])
@pytest.mark.parametrize("ranking", ["naive", "factorized"])
@pytest.mark.parametrize("shards", [1, 3])
def test_oracle_forward_matches_reference(f, ranking, shards):
    if shards > f.S:
        pytest.skip("fewer samples than shards")
    out = _fwd(f, ranking, shards)
    tol = EXTREME_FWD_RTOL if f.extreme else FWD_RTOL
    for k in OUTS:
        assert rel_err(out[k], f["out_" + k]) <= tol, (k, rel_err(out[k], f["out_" + k]))


@pytest.mark.parametrize("f", [f for f in FIX if f.mode == "train"],
                         ids=[f.name for f in FIX if f.mode == "train"])
@pytest.mark.parametrize("kind", ["gtot", "gpart"])
def test_oracle_backward_matches_reference(f, kind):
    out = _fwd(f, "factorized", 2 if f.S >= 2 else 1)
    if kind == "gtot":
        up = dict(g_total=1.0, g_I=f["g_I"], g_IL=f["g_IL"])
    else:
        up = dict(zip(PART_KEYS, f["a_parts"]))
    g = pe.elbo_backward(out, f["y"], f["fe_out"], f["fe_mu"], f["fe_logvar"], f["fx_out"],
                         f["fx_mu"], f["fx_logvar"], f["noise"], f.nll_coeff, f.c_coeff, **up)
    ref = f.grads(kind)
    assert ref, "fixture has no gradients"
    tol = EXTREME_GRAD_RTOL if f.extreme else GRAD_RTOL
    for k, v in ref.items():
        assert np.array_equal(np.isnan(g[k]), np.isnan(v)), f"NaN pattern of d{k}"
        assert rel_err(g[k], v) <= tol, (k, rel_err(g[k], v))


def test_degenerate_rows_nan_pattern():
    """All-0 / all-1 label rows: ranking loss 0 forward, whole-row NaN gradient
    (mpvae.py:117-121 under autograd) -- pinned by fixture f2."""
    f = next(f for f in FIX if f.name == "f2_degenerate")
    g = f.grads("gtot")
    rows = np.isnan(g["fe_out"]).all(1)
    assert rows.tolist() == [False, True, False, False, True, False, False, False]
    assert np.isnan(g["r_sqrt_sigma"]).all()
    assert not np.isnan(g["fe_mu"]).any()


def test_philox_known_answers():
    """Random123 kat_vectors for philox4x32_10."""
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = philox.philox4x32_10(*ctr, *key)
        assert tuple(int(x) for x in got) == want


def test_philox_noise_is_standard_normal_and_shard_invariant():
    n = philox.normal_noise(64, 16, 24, seed=77)
    assert abs(n.mean()) < 0.01 and abs(n.std() - 1.0) < 0.01
    a = philox.normal_noise(40, 16, 24, seed=77, s_offset=24)
    np.testing.assert_array_equal(a, n[24:64])


@pytest.mark.parametrize("f", [f for f in FIX if f.mode == "train"][:4],
                         ids=[f.name for f in FIX if f.mode == "train"][:4])
def test_torch_restatement_matches_reference(f):
    """oracle.torch_ref (the bench CPU baseline) reproduces the golden outputs
    and gradients: it is the reference algorithm, op for op."""
    import torch
    from oracle import torch_ref
    from golden_io import DIFF
    t = {k: torch.from_numpy(f[k].copy()) for k in ["y", "fe_out", "fe_mu", "fe_logvar",
                                                     "fx_out", "fx_mu", "fx_logvar",
                                                     "r_sqrt_sigma", "noise"]}
    for k in DIFF:
        t[k].requires_grad_(True)
    out = torch_ref.elbo_naive(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"], t["fx_out"],
                               t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"], t["noise"],
                               f.nll_coeff, f.c_coeff)
    for k, o in zip(OUTS, out):
        assert rel_err(o.detach().numpy(), f["out_" + k]) <= 1e-6, k
    obj = out[0] + (out[6] * torch.from_numpy(f["g_I"])).sum() + \
        (out[7] * torch.from_numpy(f["g_IL"])).sum()
    obj.backward()
    for k in DIFF:
        assert rel_err(t[k].grad.numpy(), f["gtot_" + k]) <= 1e-5, k


def test_long_k_gradient_conditioning():
    """Rationale of LONG_K_GRAD_RTOL: at z = 4096 an fp32 noise GEMM (the
    reference's own precision) alone moves the oracle's gradients by ~1e-4."""
    from oracle import probit_elbo as pe
    from tolerances import LONG_K_GRAD_RTOL, rel_err
    L, z, B, S, d = 4096, 4096, 1, 40, 8
    rng = np.random.default_rng(L * 7 + S)   # the GPU test's case
    y = (rng.random((B, L)) < 0.25).astype(np.float32)
    y[:, 0], y[:, 1] = 1, 0
    f32 = lambda a: a.astype(np.float32)
    # the GPU test's draw order (dict literal: fe_out, fx_out, fe_mu, fe_logvar, fx_mu, fx_logvar)
    fe_out, fx_out = f32(rng.standard_normal((B, L))), f32(rng.standard_normal((B, L)))
    fe_mu, fe_logvar = f32(rng.standard_normal((B, d))), f32(0.3 * rng.standard_normal((B, d)))
    fx_mu, fx_logvar = f32(rng.standard_normal((B, d))), f32(0.3 * rng.standard_normal((B, d)))
    inp = [y, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar]
    R = rng.uniform(-1, 1, (L, z)) * np.sqrt(6.0 / (L + z))
    noise = f32(rng.standard_normal((S, B, z)))
    g_I, g_IL = f32(rng.standard_normal((B, L))), f32(rng.standard_normal((B, L)))

    def grads(t_fp32):
        ref = pe.elbo_forward(*inp, R, noise, 0.5, 10.0, t_fp32=t_fp32)
        return pe.elbo_backward(ref, *inp, noise, 0.5, 10.0, g_total=1.0, g_I=g_I, g_IL=g_IL)

    a = grads(False)
    b = grads(True)  # t from an fp32 GEMM, as the reference's tensordot
    spread = max(rel_err(b[k], a[k]) for k in ("fe_out", "fx_out", "r_sqrt_sigma"))
    assert 5e-5 < spread < LONG_K_GRAD_RTOL / 2, spread


def test_torch_port_spread_at_headline_coefficients():
    """What bench.py's elbo_rel_err measures (GPU vs the torch-CPU restatement of
    the reference, oracle/torch_ref.py) is mostly the reference's own fp32
    conditioning, pinned here on the CPU: at L = z = 1024, B = 64, nll_coeff 0.1,
    c_coeff 200 the torch-CPU port and the fp64-reduction oracle agree on the
    loss to < 1e-6 but differ in d fe_out by ~2e-3.  The gap sits on label-0
    elements with E -> 1 (u ~ 4.9, 1 - E ~ 1e-6): there one fp32 ulp of E
    (6e-8, from t's fp32 sgemm rounding) is ~6 % of 1 - E, and d log(1 - E)
    = -1/(1 - E) carries it into the gradient.  The GPU is held to the oracle
    at HEADLINE_GRAD_RTOL (half this spread) on such slices
    (test_gpu_parity.py::test_headline_*)."""
    import torch
    from oracle import torch_ref
    B, L, z, S, d = 64, 1024, 1024, 1, 50
    rng = np.random.default_rng(5)
    y = (rng.random((B, L)) < 0.15).astype(np.float32)
    y[:, 0], y[:, 1] = 1, 0
    f32 = lambda a: a.astype(np.float32)
    inp = dict(y=y, fe_out=f32(rng.standard_normal((B, L))),
               fe_mu=f32(rng.standard_normal((B, d))), fe_logvar=f32(0.1 * rng.standard_normal((B, d))),
               fx_out=f32(rng.standard_normal((B, L))),
               fx_mu=f32(rng.standard_normal((B, d))), fx_logvar=f32(0.1 * rng.standard_normal((B, d))),
               r_sqrt_sigma=rng.uniform(-1, 1, (L, z)) * np.sqrt(6.0 / (L + z)))
    noise = f32(rng.standard_normal((S, B, z)))
    keys = ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar"]
    ref = pe.elbo_forward(*[inp[k] for k in keys], inp["r_sqrt_sigma"], noise, 0.1, 200.0)
    rg = pe.elbo_backward(ref, *[inp[k] for k in keys], noise, 0.1, 200.0, g_total=1.0)
    t = {k: torch.from_numpy(v) for k, v in inp.items()}
    for k in ("fe_out", "fx_out", "r_sqrt_sigma"):
        t[k].requires_grad_(True)
    out = torch_ref.elbo_naive(*[t[k] for k in keys], t["r_sqrt_sigma"], torch.from_numpy(noise),
                               0.1, 200.0)
    out[0].backward()
    for i, k in enumerate(OUTS):
        assert rel_err(out[i].detach().numpy(), ref[k]) <= 2e-6, k
    e = {k: rel_err(t[k].grad.numpy(), rg[k]) for k in ("fe_out", "fx_out", "r_sqrt_sigma")}
    # measured: d fe_out 1.94e-3, d fx_out 7.7e-4, dR 3.9e-4
    assert 5e-4 <= e["fe_out"] <= 5e-3, e
    assert max(e.values()) <= 5e-3, e
    g = t["fe_out"].grad.numpy().astype(np.float64)
    i = np.unravel_index(np.abs(g - rg["fe_out"]).argmax(), g.shape)
    u = pe.noise_product(noise, inp["r_sqrt_sigma"])[0][i] + inp["fe_out"][i]
    E = float(pe.probit_prob(u))
    assert inp["y"][i] == 0.0 and 1.0 - E < 1e-5, (u, E)
