"""GPU: mpv_linear (csrc/linear.hip), the VAE's Linear layers on the fp32
matrix cores, against an fp64 torch restatement of nn.Linear (+ ReLU, + the
scale_coeff multiply) and its backward, through the C ABI (mpvae_linear)."""
import numpy as np
import pytest
import torch

import mpvae_linear
from tolerances import LINEAR_RTOL, LINEAR_VAE_RTOL, record, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (M batch rows, K in features, N out features): the reference's layer shapes
# at B = 32 / 128 / 256 / 512 (mpvae.py:14-32 with feature_dim 1000, latent 50,
# label 38 / 81 / 1024) plus ragged and degenerate ones
SHAPES = [(32, 1000, 256), (128, 1038, 512), (256, 1050, 256), (256, 256, 512),
          (512, 512, 1024), (128, 256, 50), (7, 20, 6), (1, 1, 1), (33, 17, 65),
          (257, 129, 3), (5, 2100, 70)]


def _layer(K, N, bias=True, seed=0):
    torch.manual_seed(seed)
    return torch.nn.Linear(K, N, bias=bias).to(DEV)


@torch.no_grad()
def _ref(x, layer, relu, alpha, gy, mask):
    """fp64: y = act(alpha (x W^T + b)); grads of <y, gy> with the ReLU mask
    taken from the kernel's own output (boundary elements agree by fiat)."""
    xd, wd = x.double(), layer.weight.double()
    y = xd @ wd.T
    if layer.bias is not None:
        y = y + layer.bias.double()
    y = alpha * y
    if relu:
        y = torch.clamp_min(y, 0.0)
    g = gy.double() * alpha
    if mask is not None:
        g = g * (mask > 0)
    gx = g @ wd
    gw = g.T @ xd
    gb = g.sum(0) if layer.bias is not None else None
    return y, gx, gw, gb


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("relu,alpha,bias", [(True, 1.0, True), (False, 1.7, True),
                                             (False, 1.0, False)])
def test_linear_matches_fp64(M, K, N, relu, alpha, bias):
    layer = _layer(K, N, bias)
    g = torch.Generator(device=DEV).manual_seed(M * 7 + K + N)
    x = torch.randn((M, K), device=DEV, generator=g).requires_grad_(True)
    y = mpvae_linear.linear(x, layer, relu, alpha)
    gy = torch.randn((M, N), device=DEV, generator=g)
    y.backward(gy)
    yr, gxr, gwr, gbr = _ref(x.detach(), layer, relu, alpha, gy, y.detach() if relu else None)
    errs = {"y": rel_err(y.detach().cpu(), yr.cpu()), "dx": rel_err(x.grad.cpu(), gxr.cpu()),
            "dW": rel_err(layer.weight.grad.cpu(), gwr.cpu())}
    if bias:
        errs["db"] = rel_err(layer.bias.grad.cpu(), gbr.cpu())
    else:
        assert layer.bias is None
    record(f"linear_{M}_{K}_{N}_{int(relu)}_{alpha}_{int(bias)}", errs)
    for k, e in errs.items():
        assert e < LINEAR_RTOL, (k, e)


def test_linear_strided_input_and_deterministic():
    """x a column slice of a wider tensor (row stride != K), as torch.cat
    views are not; repeated launches are bitwise equal (fixed chunk order)."""
    layer = _layer(300, 200)
    big = torch.randn((128, 512), device=DEV)
    x = big[:, 100:400]
    assert x.stride(0) == 512
    outs = [mpvae_linear.linear(x, layer, True, 1.0) for _ in range(3)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    with torch.no_grad():
        ref = torch.relu(torch.nn.functional.linear(x.double(), layer.weight.double(),
                                                    layer.bias.double()))
    assert rel_err(outs[0].detach().cpu(), ref.cpu()) < LINEAR_RTOL


def test_linear_graph_capture():
    """Forward + backward captured in a HIP graph replay bit-equal to eager
    calls."""
    layer = _layer(1000, 256)
    x = torch.randn((128, 1000), device=DEV, requires_grad=True)
    gy = torch.randn((128, 256), device=DEV)

    def step():
        y = mpvae_linear.linear(x, layer, True, 1.0)
        dx, dw, db = torch.autograd.grad(y, (x, layer.weight, layer.bias), gy)
        return y.detach(), dx, dw, db
    eager = step()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        captured = step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for a, b in zip(captured, eager):
        assert torch.equal(a, b)


def test_linear_nan_and_relu_semantics():
    """torch.relu passes NaN; its backward (threshold_backward) zeroes the
    gradient only where the output is <= 0, so a NaN output passes it: the
    kernel's ReLU mask does the same."""
    layer = _layer(8, 4)
    x = torch.randn((3, 8), device=DEV)
    x[1, 2] = float("nan")
    x.requires_grad_(True)
    y = mpvae_linear.linear(x, layer, True, 1.0)
    y_t = torch.relu(torch.nn.functional.linear(x.detach(), layer.weight, layer.bias))
    assert torch.equal(torch.isnan(y), torch.isnan(y_t))
    assert torch.isnan(y[1]).all()
    y.backward(torch.ones_like(y))
    xt = x.detach().clone().requires_grad_(True)
    lt = _layer(8, 4)
    torch.relu(torch.nn.functional.linear(xt, lt.weight, lt.bias)).backward(torch.ones_like(y))
    # row 1's output is NaN everywhere and torch passes the gradient through it
    assert torch.isfinite(x.grad[1]).all() and x.grad[1].abs().max() > 0
    torch.testing.assert_close(x.grad, xt.grad, rtol=2e-6, atol=1e-6)
    assert torch.equal(torch.isnan(layer.weight.grad), torch.isnan(lt.weight.grad))
    assert torch.isnan(layer.weight.grad).any()  # x's NaN reaches dW (as in torch)


def test_linear_rejects_cpu_and_bad_shapes():
    layer = torch.nn.Linear(4, 3)
    with pytest.raises(RuntimeError):
        mpvae_linear.linear(torch.randn(2, 4), layer)
    layer = layer.to(DEV)
    with pytest.raises(ValueError):
        mpvae_linear.linear(torch.randn(2, 5, device=DEV), layer)


def test_vae_linear_backends_agree():
    """The VAE's forward + gradients with mpvae_linear='hip' against the same
    VAE on nn.Linear, same dropout masks and reparameterisation noise, with the
    nn.Linear run's ReLU masks forced to the hip run's.  (Without the forcing a
    pre-activation within rounding of 0 -- 1.5e-8 in this case -- flips its
    ReLU between any two fp32 GEMMs and moves the decoder's weight gradient
    by 3.4e-3: tools/studies/vae_linear_probe.py.)"""
    import argparse

    import mpvae
    args = argparse.Namespace(feature_dim=1000, latent_dim=50, label_dim=38, z_dim=38,
                              keep_prob=0.5, scale_coeff=1.3, residue_sigma="",
                              n_train_sample=16, n_test_sample=16, mode="train",
                              nll_coeff=0.5, c_coeff=10.0)
    masks, res = [], {}
    # the ReLU masks are taken from VAE._lin, which the folded dropout path
    # bypasses (its own test: test_vae_dropout_fold_bit_equal)
    fold, mpvae.FOLD_DROPOUT = mpvae.FOLD_DROPOUT, False
    try:
        _backends_run(args, masks, res)
    finally:
        mpvae.FOLD_DROPOUT = fold
    assert len(masks) == 7  # encoders 2 + 3 ReLU layers, the stacked decoder pass of 2
    errs = {}
    for i, (a, b) in enumerate(zip(res["hip"][0], res["torch"][0])):
        errs[f"out{i}"] = rel_err(a.cpu(), b.cpu())
    for k, v in res["torch"][1].items():
        errs["param_" + k] = rel_err(res["hip"][1][k].cpu(), v.cpu())
    record("vae_linear_hip_vs_torch", errs)
    for k, e in errs.items():
        assert e < LINEAR_VAE_RTOL, (k, e)


def _backends_run(args, masks, res):
    import mpvae
    for backend in ("hip", "torch"):
        args.mpvae_linear = backend
        torch.manual_seed(0)
        np.random.seed(0)
        model = mpvae.VAE(args).to(DEV).train()
        inner = model._lin
        if backend == "hip":
            def lin(layer, x, relu=False, alpha=1.0):
                y = inner(layer, x, relu, alpha)
                if relu:
                    masks.append((y > 0).float())
                return y
        else:
            # hip ran the two decoders stacked (rows :B label, B: feature)
            enc, (d1, d2) = masks[:5], masks[5:]
            forced = iter(enc + [d1[:128], d2[:128], d1[128:], d2[128:]])

            def lin(layer, x, relu=False, alpha=1.0):
                y = layer(x) * alpha
                return y * next(forced) if relu else y
        model._lin = lin
        g = torch.Generator().manual_seed(3)
        feat = torch.randn(128, 1000, generator=g).to(DEV)
        label = (torch.rand(128, 38, generator=g) < 0.2).float().to(DEV)
        torch.cuda.manual_seed(9)
        out = model(label, feat)
        w = [torch.randn(o.shape, generator=g).to(DEV) for o in out]
        sum((o * wi).sum() for o, wi in zip(out, w)).backward()
        res[backend] = ([o.detach() for o in out],
                        {k: p.grad.clone() for k, p in model.named_parameters()
                         if p.grad is not None})


def test_vae_dropout_fold_bit_equal():
    """The VAE on mpv_linear with the encoders' dropout backward folded into
    the gradient GEMMs equals the same VAE with nn.Dropout's own backward, bit
    for bit (outputs and every parameter gradient, reference keep_prob 0.5)."""
    import argparse

    import mpvae
    args = argparse.Namespace(feature_dim=1000, latent_dim=50, label_dim=38, z_dim=38,
                              keep_prob=0.5, scale_coeff=1.0, residue_sigma="",
                              n_train_sample=16, n_test_sample=16, mode="train",
                              nll_coeff=0.5, c_coeff=10.0, mpvae_linear="hip")
    res = {}
    fold = mpvae.FOLD_DROPOUT
    try:
        for f in (True, False):
            mpvae.FOLD_DROPOUT = f
            torch.manual_seed(0)
            np.random.seed(0)
            model = mpvae.VAE(args).to(DEV).train()
            g = torch.Generator().manual_seed(3)
            feat = torch.randn(128, 1000, generator=g).to(DEV)
            label = (torch.rand(128, 38, generator=g) < 0.2).float().to(DEV)
            torch.cuda.manual_seed(9)
            out = model(label, feat)
            w = [torch.randn(o.shape, generator=g).to(DEV) for o in out]
            sum((o * wi).sum() for o, wi in zip(out, w)).backward()
            res[f] = [o.detach() for o in out] + [p.grad.clone() for p in model.parameters()
                                                  if p.grad is not None]
    finally:
        mpvae.FOLD_DROPOUT = fold
    assert len(res[True]) == len(res[False])
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,K,Na,Nb,alpha", [(128, 256, 50, 50, 1.3), (7, 20, 6, 3, 1.0),
                                             (512, 256, 50, 50, 0.7)])
def test_heads_match_fp64(M, K, Na, Nb, alpha):
    """mpvae_linear.heads (an encoder's mu and logvar heads in one launch)
    against fp64: outputs, d x (both heads' terms summed), dW and db of each."""
    torch.manual_seed(M + K)
    la, lb = torch.nn.Linear(K, Na).to(DEV), torch.nn.Linear(K, Nb).to(DEV)
    x = torch.randn((M, K), device=DEV, requires_grad=True)
    ya, yb = mpvae_linear.heads(x, la, lb, alpha)
    ga, gb = torch.randn_like(ya), torch.randn_like(yb)
    torch.autograd.backward((ya, yb), (ga, gb))
    with torch.no_grad():
        xd = x.detach().double()
        refs = [alpha * (xd @ l.weight.double().T + l.bias.double()) for l in (la, lb)]
        gx = alpha * (ga.double() @ la.weight.double() + gb.double() @ lb.weight.double())
    errs = {"ya": rel_err(ya.detach().cpu(), refs[0].cpu()),
            "yb": rel_err(yb.detach().cpu(), refs[1].cpu()),
            "dx": rel_err(x.grad.cpu(), gx.cpu())}
    for n, l, g in (("a", la, ga), ("b", lb, gb)):
        errs["dW" + n] = rel_err(l.weight.grad.cpu(), (alpha * g.double().T @ xd).cpu())
        errs["db" + n] = rel_err(l.bias.grad.cpu(), (alpha * g.double().sum(0)).cpu())
    record(f"linear_heads_{M}_{K}_{Na}_{Nb}", errs)
    for k, e in errs.items():
        assert e < LINEAR_RTOL, (k, e)


@pytest.mark.parametrize("M,n_a,K,Na,Nb", [(256, 128, 512, 38, 38), (7, 3, 20, 5, 4),
                                           (64, 0, 33, 6, 6), (64, 64, 33, 6, 6)])
def test_row_heads_match_fp64(M, n_a, K, Na, Nb):
    """mpvae_linear.row_heads (the stacked decoders' two last layers, one per
    row block) against fp64, empty blocks included."""
    torch.manual_seed(M + n_a + K)
    la, lb = torch.nn.Linear(K, Na).to(DEV), torch.nn.Linear(K, Nb).to(DEV)
    h = torch.randn((M, K), device=DEV, requires_grad=True)
    ya, yb = mpvae_linear.row_heads(h, la, lb, n_a)
    assert ya.shape == (n_a, Na) and yb.shape == (M - n_a, Nb)
    ga, gb = torch.randn_like(ya), torch.randn_like(yb)
    torch.autograd.backward((ya, yb), (ga, gb))
    with torch.no_grad():
        hd = h.detach().double()
        ra = hd[:n_a] @ la.weight.double().T + la.bias.double()
        rb = hd[n_a:] @ lb.weight.double().T + lb.bias.double()
        gh = torch.cat((ga.double() @ la.weight.double(), gb.double() @ lb.weight.double()), 0)
    errs = {"ya": rel_err(ya.detach().cpu(), ra.cpu()), "yb": rel_err(yb.detach().cpu(), rb.cpu()),
            "dh": rel_err(h.grad.cpu(), gh.cpu())}
    for n, l, g, rows in (("a", la, ga, hd[:n_a]), ("b", lb, gb, hd[n_a:])):
        errs["dW" + n] = rel_err(l.weight.grad.cpu(), (g.double().T @ rows).cpu())
        errs["db" + n] = rel_err(l.bias.grad.cpu(), g.double().sum(0).cpu())
    record(f"linear_row_heads_{M}_{n_a}_{K}", errs)
    for k, e in errs.items():
        assert e < LINEAR_RTOL, (k, e)


@pytest.mark.parametrize("p", [0.5, 0.1, 0.9])
@pytest.mark.parametrize("M,K,N", [(128, 1000, 256), (32, 1038, 512), (33, 17, 65)])
def test_dropout_backward_folded_bit_equal(p, M, K, N):
    """linear(..., drop_p=p) -- torch's dropout kernel in the forward, its
    backward folded into the gradient GEMMs' operand load -- equals ReLU layer
    then nn.Dropout(p) (separate masked_scale backward) bit for bit: the same
    generator draws the same masks, and (out > 0) * 1/(1-p) reproduces
    masked_scale + threshold_backward exactly."""
    layer = _layer(K, N, seed=7)
    x = torch.randn((M, K), device=DEV, requires_grad=True)
    gy = torch.randn((M, N), device=DEV)

    def run(fold):
        torch.cuda.manual_seed(123)
        if fold:
            y = mpvae_linear.linear(x, layer, True, 1.0, p)
        else:
            y = torch.nn.functional.dropout(mpvae_linear.linear(x, layer, True, 1.0), p, True)
        return (y.detach(),) + torch.autograd.grad(y, (x, layer.weight, layer.bias), gy)
    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)
