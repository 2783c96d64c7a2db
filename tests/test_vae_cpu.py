"""VAE drop-in on CPU (construction only -- no kernel runs): same parameter
names, order, shapes, dtypes and seeded init as the reference (golden
fingerprints from tests/golden/make_golden.py), checkpoint round trip."""
import argparse
import os

import numpy as np
import pytest
import torch

import mpvae
from golden_io import GOLDEN


def _args(residue_sigma=""):
    return argparse.Namespace(feature_dim=20, latent_dim=8, label_dim=6, z_dim=4, keep_prob=0.5,
                              scale_coeff=1.0, residue_sigma=residue_sigma)


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(GOLDEN, "vae_small.npz"))
    return {k: z[k] for k in z.files}


def test_state_dict_layout_and_seeded_init(gold):
    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(_args())
    sd = model.state_dict()
    assert list(sd.keys()) == list(gold["sd_names"])
    assert len(sd) == 31
    for i, (k, v) in enumerate(sd.items()):
        shp = [s for s in gold["sd_shapes"][i] if s] or []
        assert list(v.shape) == shp[:v.dim()] or list(v.shape) == shp, k
        assert str(v.dtype) == gold["sd_dtypes"][i], k
        np.testing.assert_allclose(v.double().sum().item(), gold["sd_sums"][i], rtol=1e-9,
                                   atol=1e-9, err_msg=k)
        np.testing.assert_allclose(v.reshape(-1)[:4].double().numpy(), gold["sd_head"][i],
                                   rtol=0, atol=0, err_msg=k)


def test_shared_decoder_and_r_sqrt_sigma_modes():
    m = mpvae.VAE(_args())
    assert m.fd1 is m.fd_x1 and m.fd2 is m.fd_x2
    assert m.r_sqrt_sigma.dtype == torch.float64 and m.r_sqrt_sigma.requires_grad
    r = mpvae.VAE(_args("random")).r_sqrt_sigma
    assert r.dtype == torch.float64 and not r.requires_grad
    zr = mpvae.VAE(_args("zero")).r_sqrt_sigma
    assert zr.dtype == torch.float32 and not zr.requires_grad and float(zr.abs().sum()) == 0.0
    assert m.dropout.p == 0.5


def test_checkpoint_round_trip(tmp_path):
    torch.manual_seed(1)
    np.random.seed(1)
    a = mpvae.VAE(_args())
    p = tmp_path / "vae.pkl"
    torch.save(a.state_dict(), p)
    b = mpvae.VAE(_args())
    b.load_state_dict(torch.load(p, weights_only=True))
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_batched_step_syncs_match_the_reference_semantics():
    """mpvae_step: has_finite_grad gives the reference's
    per-parameter answer (fairsoft_utils.py:28-41) with one sync, step_scalars
    the .item() values with one copy."""
    import mpvae_step as ms

    def ref_has_finite_grad(model):  # fairsoft_utils.py:28-41, restated
        if isinstance(model, torch.Tensor):
            return not (torch.isnan(model.grad).any() or torch.isinf(model.grad).any())
        ok = True
        for p in model.parameters():
            if p.grad is not None:
                ok = ok and not (torch.isnan(p.grad).any() or torch.isinf(p.grad).any())
        return ok

    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(_args())
    assert ms.has_finite_grad(model) is True  # no gradients yet
    for p in model.parameters():
        p.grad = torch.randn_like(p)
    assert ms.has_finite_grad(model) == ref_has_finite_grad(model) is True
    for bad in (float("nan"), float("inf"), -float("inf")):
        model.fd2.weight.grad[1, 2] = bad
        assert ms.has_finite_grad(model) == ref_has_finite_grad(model) is False
        model.fd2.weight.grad[1, 2] = 0.0
    model.r_sqrt_sigma.grad = None
    assert ms.has_finite_grad(model) is True
    t = torch.zeros(3, requires_grad=True)
    t.grad = torch.tensor([1.0, float("nan"), 0.0])
    assert ms.has_finite_grad(t) is False
    vals = dict(total_loss=torch.tensor(1.5), nll_loss=torch.tensor(0.25, dtype=torch.float64),
                macro_f1=torch.tensor([0.75]).reshape(()), success_updates=3)
    got = ms.step_scalars(**vals)
    assert got == {"total_loss": 1.5, "nll_loss": 0.25, "macro_f1": 0.75, "success_updates": 3}
    assert all(type(got[k]) is float for k in ("total_loss", "nll_loss", "macro_f1"))


@pytest.mark.parametrize("scale", [1e-3, 1e2])
def test_train_step_clip_matches_torch(scale):
    """TrainStep._clip (coefficient cast per gradient dtype, multi-tensor fast
    path) against torch.nn.utils.clip_grad_norm_(params, 10) on the same
    gradients, fp32 and fp64 (r_sqrt_sigma) mixed: equal when the norm is
    under 10, within one fp32 ulp when it clips."""
    import types

    import mpvae_step
    args = argparse.Namespace(feature_dim=20, latent_dim=8, label_dim=6, z_dim=4, keep_prob=0.5,
                              scale_coeff=1.0, residue_sigma="", n_train_sample=4,
                              n_test_sample=4, mode="train", nll_coeff=0.5, c_coeff=10.0)
    torch.manual_seed(0)
    np.random.seed(0)
    m1 = mpvae.VAE(args)
    m2 = mpvae.VAE(args)
    m2.load_state_dict(m1.state_dict())
    g = torch.Generator().manual_seed(1)
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        gr = torch.randn(p1.shape, generator=g, dtype=torch.float64).to(p1.dtype) * scale
        p1.grad, p2.grad = gr.clone(), gr.clone()
    fake_opt = types.SimpleNamespace(defaults={"fused": True}, param_groups=[])
    ts = mpvae_step.TrainStep(m1, fake_opt, args)
    ts._clip()
    torch.nn.utils.clip_grad_norm_(m2.parameters(), 10.0)
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        if scale < 1:
            assert torch.equal(p1.grad, p2.grad), k
        else:
            torch.testing.assert_close(p1.grad, p2.grad, rtol=2 ** -23, atol=0, msg=k)


def test_device_steplr_contract():
    """Host-side contract of TrainStep's device StepLR (mpvae_step.DeviceStepLR):
    only the reference's torch.optim.lr_scheduler.StepLR, wrapping TrainStep's
    own optimizer, on the native Adam path; the device state starts from the
    scheduler's and sync() writes it back (fairsoft_jaccard.py:64-68)."""
    import mpvae_step
    args = argparse.Namespace(feature_dim=6, latent_dim=4, label_dim=5, z_dim=3, keep_prob=0.5,
                              scale_coeff=1.0, residue_sigma="", mpvae_linear="torch")
    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(args)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    other = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    sched = torch.optim.lr_scheduler.StepLR(opt, 37.5, 0.5)
    with pytest.raises(ValueError, match="StepLR"):
        mpvae_step.DeviceStepLR(torch.optim.lr_scheduler.ExponentialLR(opt, 0.9), opt)
    with pytest.raises(ValueError, match="wrap"):
        mpvae_step.DeviceStepLR(torch.optim.lr_scheduler.StepLR(other, 2), opt)
    # CPU parameters: not the native (device) Adam path, so no device scheduler
    with pytest.raises(ValueError, match="native Adam"):
        mpvae_step.TrainStep(model, opt, args, scheduler=sched)
    d = mpvae_step.DeviceStepLR(sched, opt)
    assert d.lr.dtype == torch.float64 and d.lr.tolist() == [1e-3]
    assert int(d.last_epoch) == sched.last_epoch == 0
    assert d.step_size == 37.5 and d.gamma == 0.5
    # a device step that decayed (as mpv_adam_finish does at a multiple of step_size)
    d.last_epoch.fill_(75)
    d.lr.mul_(0.5)
    assert d.sync() == [5e-4]
    assert opt.param_groups[0]["lr"] == 5e-4 and sched.last_epoch == 75
    assert sched.get_last_lr() == [5e-4]


def test_device_steplr_keeps_host_objects_consistent():
    """while TrainStep owns the StepLR, (1) opt.state_dict() and
    sched.state_dict() carry the device lr / epoch (synced first), (2) a host
    scheduler.step() raises instead of stepping twice, (3) a host edit of a
    param group's lr is adopted by the device state (with a warning), and
    release() hands the scheduler back (its step() works again)."""
    import warnings

    import mpvae_step
    p = torch.nn.Parameter(torch.zeros(3))
    opt = torch.optim.Adam([p], lr=1e-3, fused=True)
    sched = torch.optim.lr_scheduler.StepLR(opt, 2, 0.5)
    d = mpvae_step.DeviceStepLR(sched, opt)
    d.last_epoch.fill_(2)  # as if two applied updates decayed it on the device
    d.lr.mul_(0.5)
    assert opt.state_dict()["param_groups"][0]["lr"] == 5e-4
    assert sched.state_dict()["last_epoch"] == 2 and opt.param_groups[0]["lr"] == 5e-4
    with pytest.raises(RuntimeError, match="stepped on the device"):
        sched.step()
    opt.param_groups[0]["lr"] = 1e-2
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        d.adopt_host_lr()
    assert d.lr.tolist() == [1e-2] and any("adopts" in str(x.message) for x in w)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        d.adopt_host_lr()  # unchanged since: nothing to adopt, no warning
    assert not w
    assert d.release() == [1e-2]
    sched.step()  # host control again
    assert sched.last_epoch == 3


def test_device_steplr_follows_a_loaded_scheduler_checkpoint():
    """sched.load_state_dict while TrainStep owns the StepLR moves
    the device epoch and lr to the checkpoint's (decay boundaries from the
    checkpoint), and the next sync() does not write a stale epoch back."""
    import mpvae_step
    p = torch.nn.Parameter(torch.zeros(3))
    opt = torch.optim.Adam([p], lr=1e-3, fused=True)
    sched = torch.optim.lr_scheduler.StepLR(opt, 2, 0.5)
    # a checkpoint taken after 5 host scheduler steps
    p2 = torch.nn.Parameter(torch.zeros(3))
    opt2 = torch.optim.Adam([p2], lr=1e-3, fused=True)
    sched2 = torch.optim.lr_scheduler.StepLR(opt2, 2, 0.5)
    for _ in range(5):
        opt2.step()
        sched2.step()
    ckpt_opt, ckpt_sched = opt2.state_dict(), sched2.state_dict()
    d = mpvae_step.DeviceStepLR(sched, opt)
    opt.load_state_dict(ckpt_opt)
    sched.load_state_dict(ckpt_sched)
    assert int(d.last_epoch) == 5 and d.lr.tolist() == [opt2.param_groups[0]["lr"]] == [2.5e-4]
    assert d.sync() == [2.5e-4] and sched.last_epoch == 5
    assert sched.state_dict()["last_epoch"] == 5
    d.release()
    assert sched.load_state_dict.__func__ is torch.optim.lr_scheduler.StepLR.load_state_dict


def test_sharded_reference_noise_guard(monkeypatch):
    """args.mpvae_noise='torch_cpu' under sample sharding
    draws the whole (n_sample, B, z) tensor on every rank's host; above
    SHARDED_CPU_NOISE_MAX elements compute_loss's noise source refuses (before
    drawing anything), above SHARDED_CPU_NOISE_WARN it warns; unsharded it is
    the reference's draw as before."""
    import warnings
    from types import SimpleNamespace
    ex = SimpleNamespace(world=8)
    args = argparse.Namespace(mpvae_noise="torch_cpu")
    big = SimpleNamespace(S_local=1024, s_offset=0, exchange=ex)
    # C5: n_sample 8192, B 512, z 4096 -> 1.7e10 normals per rank per step
    with pytest.raises(ValueError, match="philox"):
        mpvae._noise_source(args, 8192, 512, 4096, big, "cpu")
    monkeypatch.setattr(mpvae, "SHARDED_CPU_NOISE_WARN", 1000)
    small = SimpleNamespace(S_local=4, s_offset=4, exchange=ex)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        noise, kw = mpvae._noise_source(args, 32, 8, 5, small, "cpu")
    assert any("philox" in str(x.message) for x in w)
    assert tuple(noise.shape) == (4, 8, 5) and kw == dict(noise="explicit")
    unsharded = SimpleNamespace(S_local=32, s_offset=0, exchange=None)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        torch.manual_seed(3)
        noise, _ = mpvae._noise_source(args, 32, 8, 5, unsharded, "cpu")
    assert not w
    torch.manual_seed(3)
    assert torch.equal(noise, torch.normal(0, 1, size=(32, 8, 5)))
