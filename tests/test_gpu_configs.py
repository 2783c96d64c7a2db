"""Every BASELINE.json configuration at its stated size on the HIP path.

* C1 (mirflickr L = z = 38, batch 32, n_train_sample 10, feature_dim 1000,
  nll_coeff 0.5, c_coeff 10, lr 7.5e-4; BASELINE configs[0],
  /root/reference/script/run_train_mirflickr.sh:1): the drop-in training loop
  of fairsoft_train.py:45-146 (forward -> compute_loss -> backward -> clip ->
  finite gate -> Adam) tracks the reference-order torch restatement step by
  step on the same device.
* C2 (L = z = 38, B = 128, S = 1000) and C3 (L = z = 81, B = 256, S = 2000):
  forward outputs and gradients at the full size against the numpy oracle
  (oracle/probit_elbo.py, pinned to the reference's own golden vectors).
* The evaluation call at n_test_sample = 10000 (fairsoft_evaluate.py:40,72-74,
  mode 'test', no T stash, several sample tiles per batch row) against the
  oracle, and with the whole batch of 512 at L = 1024 and 4096 against the
  fp64 restatement (tests/torch64_ref.py).
The full-size properties of C3, C4 and C5 (shard invariance, determinism,
finiteness) are in test_gpu_parity.py."""
import argparse

import numpy as np
import pytest
import torch

import mpvae
from golden_io import OUTS
from oracle import probit_elbo as pe
from test_gpu_parity import _against_oracle, _np
from tolerances import FWD_RTOL, GRAD_RTOL, HEADLINE_GRAD_RTOL, params_track, record, rel_err
from test_gpu_vae import _train_steps

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_c1_dropin_training_loop_tracks_reference():
    """C1 at its stated size, 4 optimizer steps (batch 32 of a 1000-feature
    synthetic mirflickr-shaped set)."""
    cfg = dict(feature_dim=1000, label_dim=38, z_dim=38, latent_dim=50, batch=32,
               n_train_sample=10, nll_coeff=0.5, c_coeff=10.0, lr=7.5e-4, steps=4)
    l1, p1 = _train_steps(True, **cfg)
    l2, p2 = _train_steps(False, **cfg)
    errs = {"loss": float(np.max(np.abs(np.array(l1) - l2) / np.abs(l2)))}
    errs.update({"param_" + k: rel_err(_np(p1[k]), _np(p2[k])) for k in p1})
    record("c1_dropin_loop", errs)
    np.testing.assert_allclose(l1, l2, rtol=1e-4)
    params_track("c1_dropin_loop", p1, p2, cfg["lr"], cfg["steps"])


FULL = {  # (L, z, B, S, d, nll_coeff, c_coeff): bench.py CONFIGS
    "c2": (38, 38, 128, 1000, 50, 0.5, 10.0),
    "c3": (81, 81, 256, 2000, 50, 0.1, 200.0),
}


@pytest.mark.parametrize("with_gI", [True, False], ids=["with_gI", "total_only"])
@pytest.mark.parametrize("cfg", sorted(FULL))
def test_full_size_against_oracle(cfg, with_gI):
    L, z, B, S, d, nllc, cc = FULL[cfg]
    ferr, gerr = _against_oracle(L, z, B, S, d, "f16x3", nllc, cc, 31 + L, with_gI=with_gI)
    record(f"{cfg}_full_{'with_gI' if with_gI else 'total_only'}",
           {**ferr, **{"d" + k: v for k, v in gerr.items()}})
    for k, e in ferr.items():
        assert e <= FWD_RTOL, (k, e)
    gtol = GRAD_RTOL if with_gI else HEADLINE_GRAD_RTOL
    for k, e in gerr.items():
        assert e <= gtol, (k, e)


@pytest.mark.parametrize("L,B", [(38, 16), (81, 8), (1024, 1)])
def test_eval_10000_samples_against_oracle(L, B):
    """mode 'test', n_test_sample = 10000, explicit noise, under no_grad (the
    evaluation call): all 8 outputs against the oracle."""
    S, d = 10000, 50
    rng = np.random.default_rng(L + B)
    y = (rng.random((B, L)) < 0.25).astype(np.float32)
    y[:, 0], y[:, 1] = 1, 0
    f32 = lambda *s: rng.standard_normal(s).astype(np.float32)
    inp = [y, f32(B, L), f32(B, d), 0.3 * f32(B, d), f32(B, L), f32(B, d), 0.3 * f32(B, d)]
    R = rng.uniform(-1, 1, (L, L)) * np.sqrt(6.0 / (2 * L))
    noise = f32(S, B, L)
    ref = pe.elbo_forward(*inp, R, noise, 0.5, 10.0, shards=4)
    args = argparse.Namespace(label_dim=L, z_dim=L, n_train_sample=10, n_test_sample=S,
                              mode="test", nll_coeff=0.5, c_coeff=10.0,
                              mpvae_noise=torch.from_numpy(noise))
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in inp]
    with torch.no_grad():
        out = mpvae.compute_loss(*t, torch.from_numpy(R).to(DEV), args)
    errs = {k: rel_err(_np(o), ref[k]) for k, o in zip(OUTS, out)}
    record(f"eval10000_L{L}_B{B}", errs)
    for k, e in errs.items():
        assert e <= FWD_RTOL, (k, e)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("L", [1024, 4096], ids=["c4", "c5"])
def test_eval_10000_samples_full_batch_against_fp64_reference(L):
    """The evaluation call (mode 'test', n_test_sample = 10000, no_grad) at the
    headline and C5 label dims with the whole batch of 512, philox noise: all
    8 outputs against the fp64 restatement (tests/torch64_ref.py) evaluated on
    the noise planes the kernels read (redrawn from the same key)."""
    from torch64_ref import ChunkedElbo
    from mpvae_ops import HipShardBackend
    from test_gpu_parity import _plane_noise
    B, S, d, key = 512, 10000, 50, 777 + L
    g = torch.Generator(device=DEV).manual_seed(L + 7)
    y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
    y[:, 0], y[:, 1] = 1, 0
    fe = torch.randn((B, L), device=DEV, generator=g)
    fx = torch.randn((B, L), device=DEV, generator=g)
    mus = [torch.randn((B, d), device=DEV, generator=g) * s for s in (1.0, 0.1, 1.0, 0.1)]
    R = ((torch.rand((L, L), device=DEV, generator=g, dtype=torch.float64) * 2 - 1)
         * (6.0 / (2 * L)) ** 0.5)
    args = argparse.Namespace(label_dim=L, z_dim=L, n_train_sample=10, n_test_sample=S,
                              mode="test", nll_coeff=0.1, c_coeff=200.0, mpvae_noise="philox",
                              mpvae_seed=key)
    with torch.no_grad():
        out = mpvae.compute_loss(y, fe, mus[0], mus[1], fx, mus[2], mus[3], R, args)
    got = [_np(o) for o in out]
    del out
    torch.cuda.empty_cache()
    be = HipShardBackend()
    pl = be.make_noise(be.shape(S, S, 0, B, L, L), DEV, key, 0)
    ref = ChunkedElbo(y, fe, fx, R, _plane_noise(pl, B, S, L), S, chunk=64 if L > 1024 else 256)
    rf = ref.forward(*mus, 0.1, 200.0)
    del ref, pl
    torch.cuda.empty_cache()
    errs = {k: rel_err(o, _np(rf[k])) for k, o in zip(OUTS, got)}
    record(f"eval10000_full_batch_L{L}_fp64ref", errs)
    for k, e in errs.items():
        assert e <= FWD_RTOL, (k, e)
