"""GPU: the VAE module (fused two-encoder reparameterisation kernel) and the
drop-in training step, against the reference's golden eval outputs and a
reference-order torch restatement (oracle/torch_ref.py) on the same device."""
import argparse
import os

import numpy as np
import pytest
import torch

import mpvae
from golden_io import GOLDEN
from tolerances import params_track
from oracle import torch_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _args(**kw):
    a = argparse.Namespace(feature_dim=20, latent_dim=8, label_dim=6, z_dim=4, keep_prob=0.5,
                           scale_coeff=1.0, residue_sigma="", n_train_sample=16,
                           n_test_sample=16, mode="train", nll_coeff=0.5, c_coeff=10.0)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _seeded_model(args, seed=0):
    torch.manual_seed(seed)
    np.random.seed(seed)
    return mpvae.VAE(args)


def test_eval_forward_matches_reference_golden():
    z = np.load(os.path.join(GOLDEN, "vae_small.npz"))
    model = _seeded_model(_args()).to(DEV).eval()
    eps = iter([torch.from_numpy(z["eps_label"]).to(DEV), torch.from_numpy(z["eps_feat"]).to(DEV)])
    model.reparam_noise = lambda like: next(eps)
    with torch.no_grad():
        out = model(torch.from_numpy(z["label"]).to(DEV), torch.from_numpy(z["feat"]).to(DEV))
    names = ["label_out", "label_mu", "label_logvar", "feat_out", "feat_mu", "feat_logvar"]
    for n, o in zip(names, out):
        np.testing.assert_allclose(o.cpu().numpy(), z["eval_" + n], rtol=1e-4, atol=1e-5,
                                   err_msg=n)


@pytest.mark.parametrize("train", [False, True])
def test_forward_and_grads_match_reference_order(train):
    """Same cuda seed -> same dropout masks and eps as the reference's forward
    order; outputs and all parameter gradients agree with torch autograd."""
    args = _args()
    model = _seeded_model(args).to(DEV).train(train)
    label = (torch.rand(7, 6, device=DEV) < 0.4).float()
    feat = torch.randn(7, 20, device=DEV)
    torch.cuda.manual_seed(123)
    ours = model(label, feat)
    w = [torch.randn_like(o) for o in ours]
    sum((o * wi).sum() for o, wi in zip(ours, w)).backward()
    g_ours = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
    model.zero_grad()
    torch.cuda.manual_seed(123)
    ref = torch_ref.vae_forward_reference_order(model, label, feat)
    sum((o * wi).sum() for o, wi in zip(ref, w)).backward()
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for k, p in model.named_parameters():
        if p.grad is None:
            assert k not in g_ours
            continue
        torch.testing.assert_close(g_ours[k], p.grad, rtol=1e-4, atol=1e-6, msg=k)


def _has_finite_grad(model):  # fairsoft_utils.py:28-41
    return all(torch.isfinite(p.grad).all() for p in model.parameters() if p.grad is not None)


def _train_steps(use_ours, steps=3, feature_dim=30, label_dim=12, z_dim=12, latent_dim=8,
                 batch=16, n_train_sample=32, nll_coeff=0.5, c_coeff=10.0, lr=1e-3,
                 trainstep=False, linear="torch", step_size=None, gamma=0.5):
    """The live loop body of fairsoft_train.py:45-146 (penalty-free): forward ->
    compute_loss -> backward -> clip 10 -> finite gate -> Adam step (and, with
    step_size, the StepLR step of fairsoft_jaccard.py:67-68 after an applied
    update, fairsoft_train.py:143-145).
    trainstep: ours through mpvae_step.TrainStep (fused Adam, device gate,
    device StepLR).  linear: our VAE's Linear backend (the shipped default is
    "hip"; "torch" keeps nn.Linear to compare the ELBO path and the step logic
    alone)."""
    args = _args(feature_dim=feature_dim, label_dim=label_dim, z_dim=z_dim, latent_dim=latent_dim,
                 n_train_sample=n_train_sample, nll_coeff=nll_coeff, c_coeff=c_coeff,
                 mpvae_linear=linear)
    model = _seeded_model(args, seed=7).to(DEV).train()
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=1e-5, fused=trainstep)
    sched = None if step_size is None else torch.optim.lr_scheduler.StepLR(opt, step_size, gamma)
    if trainstep:
        import mpvae_step
        ts = mpvae_step.TrainStep(model, opt, args, scheduler=sched)
    g = torch.Generator().manual_seed(11)
    X = torch.randn(steps * batch, feature_dim, generator=g)
    Y = (torch.rand(steps * batch, label_dim, generator=g) < 0.3).float()
    Y[:, 0], Y[:, 1] = 1, 0
    torch.manual_seed(5)
    torch.cuda.manual_seed(5)
    losses = []
    for i in range(steps):
        opt.zero_grad()
        sl = slice(batch * i, batch * (i + 1))
        feat, label = X[sl].to(DEV), Y[sl].to(DEV)
        if trainstep:
            res = ts(label, feat)
            losses.append(float(res[0].detach()))
            continue
        if use_ours:
            out = model(label, feat)
            res = mpvae.compute_loss(label, *out, model.r_sqrt_sigma, args)
        else:
            out = torch_ref.vae_forward_reference_order(model, label, feat)
            noise = torch.normal(0, 1, size=(n_train_sample, batch, z_dim)).to(DEV)  # mpvae.py:162
            res = torch_ref.elbo_naive(label, *out, model.r_sqrt_sigma, noise, args.nll_coeff,
                                       args.c_coeff)
        res[0].backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 10.0)
        if _has_finite_grad(model):
            opt.step()
            if sched is not None:
                sched.step()
        losses.append(float(res[0].detach()))
    if trainstep:
        ts.sync_scheduler()
    if sched is not None:
        losses.append(opt.param_groups[0]["lr"])
    return losses, {k: v.detach().clone() for k, v in model.state_dict().items()}


def test_dropin_training_loop_tracks_reference():
    l1, p1 = _train_steps(True)
    l2, p2 = _train_steps(False)
    np.testing.assert_allclose(l1, l2, rtol=1e-4)
    params_track("dropin_loop", p1, p2, 1e-3, 3)


def test_has_finite_grad_multi_tensor_path_on_device():
    """mpvae_step.has_finite_grad on CUDA grads (the fused multi-tensor
    _foreach_norm path training uses), mixed fp32 / fp64 gradients, against the
    reference's per-parameter isnan / isinf answer (fairsoft_utils.py:28-41)."""
    import mpvae_step
    args = _args()
    model = _seeded_model(args).to(DEV)
    for p in model.parameters():
        if p.requires_grad:
            p.grad = torch.randn_like(p)
    ref = lambda: all(not (torch.isnan(p.grad).any() or torch.isinf(p.grad).any())
                      for p in model.parameters() if p.grad is not None)
    assert model.r_sqrt_sigma.grad.dtype == torch.float64
    assert mpvae_step.has_finite_grad(model) is True and ref()
    for name, bad in (("fx1.weight", float("nan")), ("fe2.bias", float("inf")),
                      ("r_sqrt_sigma", float("-inf")), ("r_sqrt_sigma", float("nan")),
                      ("label_mp_mu.weight", float("-inf"))):
        p = dict(model.named_parameters())[name]
        keep = p.grad.clone()
        p.grad.view(-1)[p.grad.numel() // 2] = bad
        assert mpvae_step.has_finite_grad(model) is False and not ref(), (name, bad)
        p.grad.copy_(keep)
        assert mpvae_step.has_finite_grad(model) is True
    # a huge-but-finite gradient must not overflow the reduction
    model.fx1.weight.grad.fill_(3e38)
    assert mpvae_step.has_finite_grad(model) is True and ref()


def test_train_step_device_gate_tracks_reference_loop():
    """mpvae_step.TrainStep (fused Adam skipping on a device found_inf, no host
    sync) follows the reference loop at C1's shapes."""
    cfg = dict(feature_dim=1000, label_dim=38, z_dim=38, latent_dim=50, batch=32,
               n_train_sample=10, nll_coeff=0.5, c_coeff=10.0, lr=7.5e-4, steps=4)
    l1, p1 = _train_steps(True, trainstep=True, **cfg)
    l2, p2 = _train_steps(False, **cfg)
    np.testing.assert_allclose(l1, l2, rtol=1e-4)
    params_track("trainstep_gate_loop", p1, p2, cfg["lr"], cfg["steps"])


def test_train_step_hip_linear_tracks_torch_linear():
    """The drop-in step at C1's shapes with the Linear layers on mpv_linear
    against nn.Linear, 4 Adam steps.  Adam's first steps move every parameter
    by +-lr (m / sqrt(v) = sign(g)), so an element whose gradient sits at the
    rounding level of two fp32 GEMM orders (or behind a ReLU flip) may move
    the other way: the check is that losses agree, that almost no element
    differs and that none differs by more than those sign flips allow."""
    cfg = dict(feature_dim=1000, label_dim=38, z_dim=38, latent_dim=50, batch=32,
               n_train_sample=10, nll_coeff=0.5, c_coeff=10.0, lr=7.5e-4, steps=4)
    l1, p1 = _train_steps(True, trainstep=True, linear="hip", **cfg)
    l2, p2 = _train_steps(True, trainstep=True, linear="torch", **cfg)
    np.testing.assert_allclose(l1, l2, rtol=1e-4)
    params_track("trainstep_hip_vs_torch_linear", p1, p2, cfg["lr"], cfg["steps"], (l1, l2))


def test_shipped_default_train_step_tracks_reference_loop():
    """The shipped default end to end -- mpv_linear Linear layers with folded
    dropout, FusedReparam, the ELBO kernels, TrainStep's device gate and clip,
    mpv_adam_step and the device StepLR -- against the reference loop restated
    op for op (oracle/torch_ref: nn.Linear, the (S,B,L,L) ranking tensor,
    foreach Adam, host-gated StepLR) at C1's shapes (BASELINE configs[0]),
    across two lr decays.  Losses agree; parameters are bounded by the
    Adam-flip rule (tolerances.params_track: ReLU pre-activations within
    rounding of 0 flip between two fp32 GEMM orders); the lr equals."""
    cfg = dict(feature_dim=1000, label_dim=38, z_dim=38, latent_dim=50, batch=32,
               n_train_sample=10, nll_coeff=0.5, c_coeff=10.0, lr=7.5e-4, steps=5, step_size=2)
    l1, p1 = _train_steps(True, trainstep=True, linear="hip", **cfg)
    l2, p2 = _train_steps(False, **cfg)
    assert l1[-1] == l2[-1] == 7.5e-4 * 0.25  # decayed at updates 2 and 4
    np.testing.assert_allclose(l1[:-1], l2[:-1], rtol=1e-4)
    params_track("shipped_default_vs_reference_loop", p1, p2, cfg["lr"], cfg["steps"],
                 (l1[:-1], l2[:-1]))


@pytest.mark.parametrize("step_size", [2, 1.5])
def test_train_step_device_steplr_matches_host_loop(step_size):
    """The reference's Adam + StepLR (fairsoft_jaccard.py:64-68) stepped by its
    host-gated loop (fairsoft_train.py:140-146: the scheduler steps only after
    an applied update) against TrainStep with the scheduler on the device,
    across lr decays and a skipped (NaN) update: lr, parameters, Adam state,
    the scheduler's last_epoch and the update count equal, bit for bit.  Both
    sides run the same model code, so only the step logic differs; clipping
    at 1e9 multiplies by exactly 1 on both sides.  A float step_size (the
    reference passes one_epoch_iter * max_epoch / lr_decay_times) decays
    where Python's `last_epoch % step_size` is 0."""
    import mpvae_step

    def run(ours):
        args = _args(feature_dim=30, label_dim=12, z_dim=12, latent_dim=8, n_train_sample=32)
        model = _seeded_model(args, seed=7).to(DEV).train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5, fused=True)
        sched = torch.optim.lr_scheduler.StepLR(opt, step_size, 0.5)
        ts = mpvae_step.TrainStep(model, opt, args, max_grad_norm=1e9, scheduler=sched) \
            if ours else None
        g = torch.Generator().manual_seed(11)
        torch.manual_seed(5)
        torch.cuda.manual_seed(5)
        lrs, updates = [], 0
        for i in range(7):
            y = (torch.rand(16, 12, generator=g) < 0.3).float()
            y[:, 0], y[:, 1] = 1, 0
            if i == 3:
                y[5] = 0.0  # no positive label: NaN ranking gradient, update skipped
            label, feat = y.to(DEV), torch.randn(16, 30, generator=g).to(DEV)
            if ours:
                ts(label, feat)
                lrs.append(float(ts.sched.lr[0]))
                continue
            opt.zero_grad()
            out = model(label, feat)
            res = mpvae.compute_loss(label, *out, model.r_sqrt_sigma, args)
            res[0].backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1e9)
            if _has_finite_grad(model):
                opt.step()
                sched.step()
                updates += 1
            lrs.append(opt.param_groups[0]["lr"])
        if ours:
            assert ts.sync_scheduler() == [opt.param_groups[0]["lr"]]
            updates = int(ts.updates)
        st = [(k, opt.state[p]) for k, p in model.named_parameters()]
        return lrs, updates, sched.last_epoch, sched.get_last_lr(), model.state_dict(), st

    ours, ref = run(True), run(False)
    assert ours[0] == ref[0], (ours[0], ref[0])
    assert len(set(ref[0])) >= 3  # at least two decays happened
    assert ours[1:4] == ref[1:4] and ref[1] == 6
    for (k, a), b in zip(ours[4].items(), ref[4].values()):
        assert torch.equal(a, b), k
    for (k, sa), (_, sb) in zip(ours[5], ref[5]):
        for key in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[key], sb[key]), (k, key)


def test_train_step_skips_nonfinite_update_on_device():
    """A degenerate label row (no positive label) makes the ranking gradient
    NaN (mpvae.py:118): the step must leave every parameter and the Adam step
    count untouched, like the reference's has_finite_grad gate."""
    import mpvae_step
    args = _args(n_train_sample=8)
    model = _seeded_model(args).to(DEV).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    ts = mpvae_step.TrainStep(model, opt, args)
    label = (torch.rand(5, 6, device=DEV) < 0.5).float()
    label[:, 0], label[:, 1] = 1, 0
    feat = torch.randn(5, 20, device=DEV)
    ts(label, feat)
    assert int(ts.updates) == 1
    before = {k: v.clone() for k, v in model.state_dict().items()}
    bad = label.clone()
    bad[2] = 0.0
    ts(bad, feat)
    assert int(ts.updates) == 1 and float(ts.found_inf) == 1.0
    for k, v in model.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert all(int(s["step"]) == 1 for s in opt.state.values())


def test_train_step_graph_replays_match_eager():
    """The whole step (VAE forward, compute_loss, backward, clip, gate, Adam)
    captured in one HIP graph: replays on new batches equal eager TrainStep
    calls (reparameterisation noise switched off, dropout off, philox probit
    noise keyed by a device seed the step advances)."""
    import mpvae_step
    B, F_, L = 24, 40, 10

    def make():
        a = _args(feature_dim=F_, label_dim=L, z_dim=L, latent_dim=8, keep_prob=0.0,
                  n_train_sample=64, mpvae_noise="philox",
                  mpvae_seed=torch.tensor([99], dtype=torch.int64, device=DEV))
        m = _seeded_model(a, seed=3).to(DEV).train()
        m.reparam_noise = torch.zeros_like
        o = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5, fused=True,
                             capturable=True)
        # the reference's StepLR, on the device inside the graph
        sch = torch.optim.lr_scheduler.StepLR(o, 2, 0.5)
        return m, mpvae_step.TrainStep(m, o, a, scheduler=sch)

    g = torch.Generator().manual_seed(2)
    batches = []
    for _ in range(4):
        y = (torch.rand(B, L, generator=g) < 0.3).float()
        y[:, 0], y[:, 1] = 1, 0
        batches.append((y.to(DEV), torch.randn(B, F_, generator=g).to(DEV)))
    mg, tg = make()
    me, te = make()
    tg.capture(*batches[0], warmup=1)
    te(*batches[0])
    for y, x in batches[1:]:
        og = [o.clone() for o in tg(y, x)]
        oe = te(y, x)
        torch.cuda.synchronize()
        for a, b in zip(og, oe):
            torch.testing.assert_close(a, b.detach(), rtol=1e-6, atol=0)
    for (k, a), b in zip(mg.state_dict().items(), me.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-9, msg=k)
    assert int(tg.updates) == int(te.updates) == 4
    assert tg.sync_scheduler() == te.sync_scheduler() == [1e-3 * 0.5 * 0.5]


def test_release_scheduler_drops_the_captured_graph():
    """a graph captured while TrainStep owned the StepLR steps the
    device lr inside its Adam launch.  release_scheduler() drops it, so the
    next call runs eagerly on the host's param_groups lr: with lr set to 0
    on the host the parameters stay as they are (a replay would have moved
    them by the device lr)."""
    import mpvae_step
    B, F_, L = 16, 30, 8
    a = _args(feature_dim=F_, label_dim=L, z_dim=L, latent_dim=8, keep_prob=0.0,
              n_train_sample=32, mpvae_noise="philox",
              mpvae_seed=torch.tensor([5], dtype=torch.int64, device=DEV))
    m = _seeded_model(a, seed=4).to(DEV).train()
    o = torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True)
    sch = torch.optim.lr_scheduler.StepLR(o, 2, 0.5)
    ts = mpvae_step.TrainStep(m, o, a, scheduler=sch)
    g = torch.Generator().manual_seed(3)
    y = (torch.rand(B, L, generator=g) < 0.3).float()
    y[:, 0], y[:, 1] = 1, 0
    batch = (y.to(DEV), torch.randn(B, F_, generator=g).to(DEV))
    ts.capture(*batch, warmup=1)
    ts(*batch)  # a replay: the device lr is in use
    assert ts.release_scheduler() == [o.param_groups[0]["lr"]]
    assert ts.graph is None
    o.param_groups[0]["lr"] = 0.0
    before = {k: v.clone() for k, v in m.state_dict().items()}
    ts(*batch)
    torch.cuda.synchronize()
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    sch.step()  # the host scheduler is usable again


def test_native_adam_matches_torch_fused_adam():
    """mpvae_step.adam_step (csrc/adam.hip, one launch) against torch's fused
    capturable Adam on the same parameters and gradients: fp32 tensors of the
    VAE's shapes and ragged ones plus an fp64 one (r_sqrt_sigma), L2 weight
    decay, six steps with a skipped (found_inf) update in the middle.  The
    per-element arithmetic is torch's adam_math, so parameters and moments
    agree to the last bit or within one rounding."""
    import copy

    import mpvae_step
    from tolerances import record
    torch.manual_seed(11)
    shapes = [((512, 1038), torch.float32), ((512,), torch.float32), ((38, 512), torch.float32),
              ((7,), torch.float32), ((3, 2049), torch.float32), ((1,), torch.float32),
              ((38, 38), torch.float64)]
    ps = [torch.nn.Parameter(torch.randn(s, dtype=dt, device=DEV)) for s, dt in shapes]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    kw = dict(lr=7.5e-4, weight_decay=1e-5, fused=True, capturable=True)
    ref = torch.optim.Adam(ps, **kw)
    mine = torch.optim.Adam(qs, **kw)
    assert mpvae_step._native_adam(mine)
    sref = torch.optim.lr_scheduler.StepLR(ref, 2, 0.3)
    dsched = mpvae_step.DeviceStepLR(torch.optim.lr_scheduler.StepLR(mine, 2, 0.3), mine)
    found = torch.zeros((), dtype=torch.float32, device=DEV)
    worst = 0.0
    for it in range(6):
        found.fill_(1.0 if it == 3 else 0.0)
        for p, q in zip(ps, qs):
            g = torch.randn_like(p) * (10.0 if it == 0 else 1.0)
            p.grad, q.grad = g.clone(), g.clone()
        ref.found_inf = found
        ref.step()
        del ref.found_inf
        if it != 3:
            sref.step()  # the reference's scheduler steps after applied updates only
        mpvae_step.adam_step(mine, found, sched=dsched)
        assert float(dsched.lr[0]) == ref.param_groups[0]["lr"], it
        for p, q in zip(ps, qs):
            sp, sq = ref.state[p], mine.state[q]
            assert torch.equal(sp["step"], sq["step"]), (it, sp["step"], sq["step"])
            for a, b in ((p, q), (sp["exp_avg"], sq["exp_avg"]), (sp["exp_avg_sq"], sq["exp_avg_sq"])):
                d = ((a.detach().double() - b.detach().double()).abs()
                     / a.detach().double().abs().clamp_min(1e-30)).max().item()
                worst = max(worst, d)
                assert torch.equal(a, b), (it, tuple(a.shape), d)
    record("native_adam_vs_torch_fused", {"max_rel": worst})
    assert ref.param_groups[0]["lr"] == 7.5e-4 * 0.3 * 0.3
    # the state is torch's own: a state_dict round trip restores it
    sd = copy.deepcopy(mine.state_dict())
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


def test_fused_reparam_passthrough_grads_bit_equal():
    """FusedReparam's mu / logvar pass-through outputs: a gradient reaching
    them (compute_loss's KL) is added inside mpv_reparam_bwd, and equals, bit
    for bit, autograd adding it to the reparameterisation gradient when the
    original mu / logvar tensors are used instead."""
    from mpvae_ops import FusedReparam
    torch.manual_seed(4)
    shp = [(128, 50), (128, 50)]
    leaves = [torch.randn(s, device=DEV, requires_grad=True) for s in shp + shp]
    mu_e, lv_e, mu_x, lv_x = leaves
    eps_e, eps_x = torch.randn(shp[0], device=DEV), torch.randn(shp[1], device=DEV)
    w = [torch.randn(shp[0], device=DEV) for _ in range(6)]

    def grads(passthrough):
        h = [t * 1.0 for t in leaves]  # non-leaf heads, as the encoders' outputs
        out = FusedReparam.apply(h[0], h[1], eps_e, h[2], h[3], eps_x)
        z_e, z_x = out[:2]
        m = out[2:] if passthrough else h
        loss = sum((a * b).sum() for a, b in zip((z_e, z_x) + tuple(m), w))
        return torch.autograd.grad(loss, leaves)
    for a, b in zip(grads(True), grads(False)):
        assert torch.equal(a, b)
    # the returned mu / logvar are fresh tensors, not views of the heads: a
    # caller may modify them in place, as it may the reference's
    h = [t * 1.0 for t in leaves]
    out = FusedReparam.apply(h[0], h[1], eps_e, h[2], h[3], eps_x)
    assert all(o._base is None and o.data_ptr() != x.data_ptr() for o, x in zip(out[2:], h))
    assert all(torch.equal(o, x) for o, x in zip(out[2:], h))
    out[2].clamp_(-1.0, 1.0)
    (out[2].sum() + out[0].sum()).backward()
    assert torch.isfinite(leaves[0].grad).all()


@pytest.mark.parametrize("linear", ["hip", "torch"])
def test_empty_batch_forward_and_backward(linear):
    """A batch of 0 rows through VAE.forward (train and eval) and compute_loss
    and back: the reference's nn.Linear / randn_like / compute_loss give (0, n)
    outputs, NaN losses and zero parameter gradients (tests/golden/edge_cases.json
    for compute_loss); no kernel may be launched with an empty grid."""
    args = _args(mpvae_linear=linear)
    model = _seeded_model(args).to(DEV)
    for train in (True, False):
        model.train(train)
        out = model(torch.zeros(0, 6, device=DEV), torch.zeros(0, 20, device=DEV))
        assert [tuple(o.shape) for o in out] == [(0, 6), (0, 8), (0, 8), (0, 6), (0, 8), (0, 8)]
        if train:
            loss = mpvae.compute_loss(torch.zeros(0, 6, device=DEV), *out, model.r_sqrt_sigma,
                                      args)
            assert torch.isnan(loss[0]).item()
            loss[0].backward()
            torch.cuda.synchronize()
            for n, p in model.named_parameters():
                assert p.grad is None or not p.grad.any(), n
