"""BASELINE configs[0] on the CPU: compute_loss on CPU tensors through the host
C++ backend (libmpvae_host.so, mpvae_host.py), checked against the reference's
own golden vectors (tests/golden, made by importing the reference's mpvae.py)
and the reference's VAE -- without the oracle: nothing under oracle/ is
imported by the product on this path (asserted)."""
import argparse
import sys

import numpy as np
import pytest
import torch

import mpvae
from golden_io import DIFF, OUTS, fixtures
from tolerances import EXTREME_FWD_RTOL, EXTREME_GRAD_RTOL, FWD_RTOL, GRAD_RTOL, rel_err

FIX = fixtures()


def _inputs(f):
    t = {k: torch.from_numpy(f[k].copy()) for k in
         ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar", "r_sqrt_sigma"]}
    if f.mode == "train":
        for k in DIFF:
            t[k].requires_grad_(True)
        if f.trainable_r:
            t["r_sqrt_sigma"].requires_grad_(True)
    return t


def _call(t, args):
    return mpvae.compute_loss(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"], t["fx_out"],
                              t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"], args)


@pytest.mark.parametrize("f", FIX, ids=[f.name for f in FIX])
@pytest.mark.parametrize("kind", ["gtot", "gpart"])
def test_golden_on_the_cpu_backend(f, kind):
    """Every golden fixture, forward and both gradient objectives, on CPU tensors:
    the same tolerances as the GPU path (tests/tolerances.py)."""
    t = _inputs(f)
    out = _call(t, f.args(mpvae_noise=torch.from_numpy(f["noise"])))
    ftol = EXTREME_FWD_RTOL if f.extreme else FWD_RTOL
    for k, o in zip(OUTS, out):
        assert o.device.type == "cpu" and o.dtype == torch.float32
        e = rel_err(o.detach().double().numpy(), f["out_" + k])
        assert e <= ftol, (k, e)
    if f.mode != "train":
        return
    if kind == "gtot":
        obj = out[0] + (out[6] * torch.from_numpy(f["g_I"])).sum() + \
            (out[7] * torch.from_numpy(f["g_IL"])).sum()
    else:
        obj = sum(float(a) * o for a, o in zip(f["a_parts"], out[1:6]))
    obj.backward()
    gtol = EXTREME_GRAD_RTOL if f.extreme else GRAD_RTOL
    for k, v in f.grads(kind).items():
        g = t[k].grad
        assert g.dtype == t[k].dtype, k
        g = g.double().numpy()
        assert np.array_equal(np.isnan(g), np.isnan(v)), f"NaN pattern of d{k}"
        assert rel_err(g, v) <= gtol, (k, rel_err(g, v))


def test_default_noise_is_the_reference_cpu_draw():
    """mpvae_noise unset: the reference's CPU draw (mpvae.py:162), seeded."""
    f = next(f for f in FIX if f.name == "f1_l38")
    t = {k: v.detach() for k, v in _inputs(f).items()}
    torch.manual_seed(1000 + 11)  # the seed make_golden.py used for f1
    out = _call(t, f.args())
    for k, o in zip(OUTS, out):
        assert rel_err(o.double().numpy(), f["out_" + k]) <= FWD_RTOL, k


def test_results_do_not_depend_on_the_thread_count():
    import mpvae_host
    lib = mpvae_host.load_library()
    f = next(f for f in FIX if f.name == "f6_l81")
    res = []
    for n in (1, 4, 0):
        assert lib.mpvh_set_threads(n) == 0
        t = _inputs(f)
        out = _call(t, f.args(mpvae_noise=torch.from_numpy(f["noise"])))
        out[0].backward()
        res.append([o.detach().clone() for o in out] + [t["fe_out"].grad.clone(),
                                                        t["fx_out"].grad.clone()])
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


def test_c1_training_steps_on_the_cpu():
    """BASELINE configs[0] (mirflickr L = 38, batch 32, n_train_sample 10) end to
    end on the CPU: the VAE (the reference's ops on CPU tensors) + compute_loss
    on the host backend + Adam, five steps; the loss is finite and falls, the
    VAE's eval forward matches the reference's golden init/forward, and no
    module under oracle/ was imported by any of it."""
    before = set(sys.modules)
    args = argparse.Namespace(feature_dim=1000, latent_dim=50, label_dim=38, z_dim=38,
                              keep_prob=0.5, scale_coeff=1.0, residue_sigma="", n_train_sample=10,
                              n_test_sample=10, mode="train", nll_coeff=0.5, c_coeff=10.0)
    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(args).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(3)
    label = (torch.rand(32, 38, generator=g) < 0.1).float()
    label[:, 0], label[:, 1] = 1, 0
    feat = torch.randn(32, 1000, generator=g)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        out = model(label, feat)
        res = mpvae.compute_loss(label, *out, model.r_sqrt_sigma, args)
        res[0].backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 10.0)
        opt.step()
        losses.append(float(res[0].detach()))
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses
    assert model.r_sqrt_sigma.grad is not None and model.r_sqrt_sigma.grad.dtype == torch.float64
    new = set(sys.modules) - before
    assert not any(m == "oracle" or m.startswith("oracle.") for m in new), sorted(new)
    assert "mpvae_host" in sys.modules


def test_vae_cpu_forward_matches_reference_golden(golden_dir):
    """The VAE's eval forward on CPU tensors (the reference's own ops) against
    the record of the reference's VAE itself (tests/golden/vae_small.npz: same
    seeds, eval mode, the label eps then the feature eps)."""
    import os
    z = np.load(os.path.join(golden_dir, "vae_small.npz"))
    args = argparse.Namespace(feature_dim=20, latent_dim=8, label_dim=6, z_dim=4, keep_prob=0.5,
                              scale_coeff=1.0, residue_sigma="")
    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(args).eval()
    torch.manual_seed(1)
    with torch.no_grad():
        out = model(torch.from_numpy(z["label"]), torch.from_numpy(z["feat"]))
    for k, o in zip(["label_out", "label_mu", "label_logvar", "feat_out", "feat_mu",
                     "feat_logvar"], out):
        np.testing.assert_allclose(o.numpy(), z["eval_" + k], rtol=1e-5, atol=1e-6, err_msg=k)
