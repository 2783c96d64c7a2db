"""Where do the VAE's gradients with mpv_linear and with nn.Linear part?
Per Linear call: the kernel's own error against fp64 on the SAME inputs
(x, upstream gradient, ReLU mask), and how far the two backends' inputs to
that call already differ.  python tools/studies/vae_linear_probe.py [B]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import mpvae  # noqa: E402
import mpvae_linear  # noqa: E402
from tolerances import rel_err  # noqa: E402

DEV = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
calls = {}


def run(backend):
    args = argparse.Namespace(feature_dim=1000, latent_dim=50, label_dim=38, z_dim=38,
                              keep_prob=0.5, scale_coeff=1.0, residue_sigma="",
                              n_train_sample=16, n_test_sample=16, mode="train",
                              nll_coeff=0.5, c_coeff=10.0, mpvae_linear=backend)
    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(args).to(DEV).train()
    names = {id(m): n for n, m in model.named_modules()}
    rec = []
    orig = model._lin
    mpvae.FOLD_DROPOUT = False  # every ReLU layer through model._lin (recorded)

    def lin(layer, x, relu=False, alpha=1.0):
        xx = x.detach().clone()
        y = orig(layer, x, relu, alpha)
        ent = {"name": names[id(layer)], "x": xx, "y": y.detach().clone(), "relu": relu,
               "alpha": alpha}
        y.register_hook(lambda g: ent.__setitem__("gy", g.detach().clone()))
        rec.append(ent)
        return y
    model._lin = lin
    g = torch.Generator().manual_seed(3)
    feat = torch.randn(B, 1000, generator=g).to(DEV)
    label = (torch.rand(B, 38, generator=g) < 0.2).float().to(DEV)
    torch.cuda.manual_seed(9)
    out = model(label, feat)
    w = [torch.randn(o.shape, generator=g).to(DEV) for o in out]
    sum((o * wi).sum() for o, wi in zip(out, w)).backward()
    return model, rec


mh, rh = run("hip")
mt, rt = run("torch")
for a, b in zip(rh, rt):
    layer = dict(mh.named_modules())[a["name"]]
    W = layer.weight.detach().double()
    gy = a["gy"].double() * a["alpha"]
    if a["relu"]:
        gy = gy * (a["y"] > 0)
    dW64 = gy.T @ a["x"].double()
    flips = int(((a["y"] > 0) != (b["y"] > 0)).sum()) if a["relu"] else 0
    print(f"{a['name']:14s} x diff {rel_err(a['x'].cpu(), b['x'].cpu()):.1e}  "
          f"y diff {rel_err(a['y'].cpu(), b['y'].cpu()):.1e}  "
          f"gy diff {rel_err(a['gy'].cpu(), b['gy'].cpu()):.1e}  mask flips {flips}  "
          f"min|y>0| {a['y'][a['y'] > 0].abs().min().item() if a['relu'] else 0:.1e}", flush=True)
for n, p in mh.named_parameters():
    q = dict(mt.named_parameters())[n]
    if p.grad is not None:
        print(f"grad {n:22s} hip-vs-torch {rel_err(p.grad.cpu(), q.grad.cpu()):.1e}")
