"""The full drop-in training step at a BASELINE config:
VAE forward (12 nn.Linear + ReLU / dropout, fused reparameterisation) ->
compute_loss -> backward -> clip_grad_norm_(10) -> finite gate -> Adam
(fairsoft_train.py:47-146, mpvae.py:51-100), on synthetic mirflickr-shaped data.

Reports (one JSON line):
  eager_ms        one eager step (host gate: the reference's has_finite_grad sync)
  trainstep_ms    mpvae_step.TrainStep eager (device gate, no host sync)
  graph_ms        TrainStep captured in one HIP graph, replayed
  phases_ms       eager step cut by HIP events: forward / loss / backward / clip+gate / adam
  kernels         device time by kernel over graph replays (torch.profiler), top entries

    python tools/trainstep_profile.py [--config c2|c1] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpvae  # noqa: E402
import mpvae_step  # noqa: E402

# name: (feature_dim, label_dim, z_dim, latent_dim, batch, n_train_sample, nll, c, lr)
CONFIGS = {"c1": (1000, 38, 38, 50, 32, 10, 0.5, 10.0, 7.5e-4),
           "c2": (1000, 38, 38, 50, 128, 1000, 0.5, 10.0, 7.5e-4),
           "c3": (1000, 81, 81, 50, 256, 2000, 0.1, 200.0, 7.5e-4)}


def build(cfg, dev, fused, linear="hip"):
    F_, L, z, d, B, S, nllc, cc, lr = CONFIGS[cfg]
    args = argparse.Namespace(feature_dim=F_, latent_dim=d, label_dim=L, z_dim=z, keep_prob=0.5,
                              scale_coeff=1.0, residue_sigma="", n_train_sample=S,
                              n_test_sample=S, mode="train", nll_coeff=nllc, c_coeff=cc,
                              mpvae_noise="philox", mpvae_linear=linear,
                              mpvae_seed=torch.tensor([77], dtype=torch.int64, device=dev))
    torch.manual_seed(0)
    np.random.seed(0)
    model = mpvae.VAE(args).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=1e-5, fused=fused,
                           capturable=fused)
    g = torch.Generator().manual_seed(1)
    feat = torch.randn(B, F_, generator=g).to(dev)
    label = (torch.rand(B, L, generator=g) < 0.1).float().to(dev)
    label[:, 0], label[:, 1] = 1, 0
    return args, model, opt, label, feat


def eager_step(model, opt, args, label, feat, ev=None):
    def mark(i):
        if ev is not None:
            ev[i].record()
    mark(0)
    opt.zero_grad()
    args.mpvae_seed.add_(1)
    out = model(label, feat)
    mark(1)
    res = mpvae.compute_loss(label, *out, model.r_sqrt_sigma, args)
    mark(2)
    res[0].backward()
    mark(3)
    torch.nn.utils.clip_grad_norm_(model.parameters(), 10.0)
    ok = mpvae_step.has_finite_grad(model)   # host sync, as the reference's gate
    mark(4)
    if ok:
        opt.step()
    mark(5)
    return res


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=50)
    # torch's BLAS backend for the nn.Linear GEMMs: hipBLASLt (torch's default on
    # MI355X) or rocBLAS ("cublas" in torch's naming)
    ap.add_argument("--blas", default=None, choices=["cublaslt", "cublas"])
    # the VAE's Linear layers: mpv_linear ("hip", the default) or nn.Linear
    ap.add_argument("--linear", default="hip", choices=["hip", "torch"])
    # also list the aten ops of one eager TrainStep call (what issues the launches)
    ap.add_argument("--ops", action="store_true")
    # TrainStep's Adam: mpv_adam_step (default) or torch's fused kernel, for A/B
    ap.add_argument("--torch-adam", action="store_true")
    # nn.Dropout's own backward kernel instead of the fold into mpv_linear
    ap.add_argument("--no-fold-dropout", action="store_true")
    # autograd's adds of the encoder heads' two gradients instead of mpv_reparam_bwd's
    ap.add_argument("--no-passthrough", action="store_true")
    # the encoder heads' dx as two GEMMs and an add instead of one two-segment GEMM
    ap.add_argument("--heads-dx-two", action="store_true")
    cli = ap.parse_args()
    import mpvae_linear
    mpvae_linear.HEADS_DX_ONE_GEMM = not cli.heads_dx_two
    mpvae.FOLD_DROPOUT = not cli.no_fold_dropout
    mpvae.REPARAM_PASSTHROUGH = not cli.no_passthrough
    dev = torch.device("cuda", 0)
    if cli.blas:
        torch.backends.cuda.preferred_blas_library(cli.blas)

    args, model, opt, label, feat = build(cli.config, dev, fused=False, linear=cli.linear)
    for _ in range(3):
        eager_step(model, opt, args, label, feat)
    eager_ms = timed(lambda: eager_step(model, opt, args, label, feat), cli.steps)
    names = ["forward", "compute_loss", "backward", "clip+gate", "adam"]
    acc = np.zeros(5)
    for _ in range(cli.steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        eager_step(model, opt, args, label, feat, ev)
        torch.cuda.synchronize()
        acc += [ev[i].elapsed_time(ev[i + 1]) for i in range(5)]
    phases = {n: round(v / cli.steps, 4) for n, v in zip(names, acc)}

    args, model, opt, label, feat = build(cli.config, dev, fused=True, linear=cli.linear)
    ts = mpvae_step.TrainStep(model, opt, args, native_adam=not cli.torch_adam)
    for _ in range(3):
        ts(label, feat)
    ts_ms = timed(lambda: ts(label, feat), cli.steps)
    ts.capture(label, feat)
    for _ in range(3):
        ts(label, feat)
    graph_ms = timed(lambda: ts(label, feat), cli.steps)

    kernels = None
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(10):
                ts(label, feat)
            torch.cuda.synchronize()
        rows = []
        for e in prof.key_averages():
            t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
            if t:
                rows.append((e.key, e.count / 10, t / 10 / 1e3))
        rows.sort(key=lambda r: -r[2])
        kernels = {"per_step_ms_total": round(sum(r[2] for r in rows), 4),
                   "launches_per_step": round(sum(r[1] for r in rows), 1),
                   "top": [{"kernel": k[:120], "per_step": c, "ms": round(ms, 4)}
                           for k, c, ms in rows[:25]]}
    except Exception as e:  # profiler unavailable: report why
        kernels = {"error": repr(e)[:300]}

    ops = None
    if cli.ops:
        from torch.profiler import ProfilerActivity, profile
        _, model2, opt2, _, _ = build(cli.config, dev, fused=True, linear=cli.linear)
        ts2 = mpvae_step.TrainStep(model2, opt2, args, native_adam=not cli.torch_adam)
        ts2(label, feat)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            ts2(label, feat)
            torch.cuda.synchronize()
        rows = [(e.key, e.count) for e in prof.key_averages() if e.key.startswith("aten::")]
        rows.sort(key=lambda r: -r[1])
        ops = rows[:40]

    F_, L, z, d, B, S, nllc, cc, lr = CONFIGS[cli.config]
    print(json.dumps({"aten_ops_per_eager_step": ops,"blas": str(torch.backends.cuda.preferred_blas_library()), "linear": cli.linear,
                      "config": {"name": cli.config, "feature_dim": F_, "label_dim": L, "z_dim": z,
                                 "latent_dim": d, "batch": B, "n_train_sample": S,
                                 "nll_coeff": nllc, "c_coeff": cc, "lr": lr},
                      "steps": cli.steps, "eager_ms": round(eager_ms, 4),
                      "phases_ms": phases, "trainstep_ms": round(ts_ms, 4),
                      "graph_ms": round(graph_ms, 4), "adam": "torch" if cli.torch_adam else "mpv_adam_step",
                      "fold_dropout": mpvae.FOLD_DROPOUT,
                      "reparam_passthrough": mpvae.REPARAM_PASSTHROUGH,
                      "updates": int(ts.updates),
                      "loss_finite": bool(torch.isfinite(ts.out[0]).item()),
                      "kernels": kernels}), flush=True)


if __name__ == "__main__":
    main()
