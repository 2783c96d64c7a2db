"""Time the per-step consumers of compute_loss's indiv_prob outputs at the
north-star batch (B=512, L=1024): the device fairness regulariser (label
weights + fwd + bwd) and the train metrics, against the CPU oracle of the same
computation (oracle/fairness.py: the reference's loop structure -- a Python
dict lookup per row, group masks -- in numpy, single thread).

    python tools/studies/bench_consumers.py [--reps 20]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

import mpvae_fair as mf  # noqa: E402
import mpvae_hip as H  # noqa: E402
from oracle import fairness as of  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--L", type=int, default=1024)
    cli = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    B, L, T = cli.B, cli.L, 3
    labels = (rng.random((B, L)) < 0.02).astype(np.int64)
    labels[B // 2:] = labels[:B - B // 2]
    sens = rng.integers(0, 2, (B, 2)).astype(np.int64)
    dists = [{"".join(r.astype(str)): float(rng.uniform(0.1, 1)) for r in labels[i::5]}
             for i in range(T)]
    lz_np = rng.uniform(0.01, 0.99, (B, L)).astype(np.float32)
    fz_np = rng.uniform(0.01, 0.99, (B, L)).astype(np.float32)
    tables = [mf.LabelDistanceTable(d, L, dev) for d in dists]
    lab, sen = torch.from_numpy(labels).to(dev), torch.from_numpy(sens).to(dev)
    lz = torch.from_numpy(lz_np).to(dev).requires_grad_(True)
    fz = torch.from_numpy(fz_np).to(dev).requires_grad_(True)

    def fair_step():
        loss, cnt = mf.fairness_penalty(lz, fz, lab, sen, tables, "l1", 0.5)
        loss.backward()
        return loss

    def metric_step():
        return mf.compute_metrics(fz.detach(), lab.float(), 0.5)["maF1"]

    res = {}
    lib = H.load_library()
    for name, fn in (("fairness_fwd_bwd", fair_step), ("train_metrics", metric_step)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        lib.mpv_timing_enable(1)
        lib.mpv_timing_reset()
        t0 = time.perf_counter()
        for _ in range(cli.reps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / cli.reps * 1e3
        lib.mpv_timing_enable(0)
        kt = {k: round(v[1] / cli.reps, 4) for k, v in H.kernel_times().items()}
        res[name] = {"wall_ms": round(wall, 4), "kernel_ms": kt}
    # per-step host syncs after backward (fairsoft_train.py:141-162): the
    # reference's has_finite_grad (two host bools per parameter) and eight
    # .item() calls, against mpvae_step's one reduction + one copy each
    import argparse as _ap
    import mpvae
    import mpvae_step as ms
    vargs = _ap.Namespace(feature_dim=1000, latent_dim=50, label_dim=L, z_dim=L, keep_prob=0.5,
                          scale_coeff=1.0, residue_sigma="")
    model = mpvae.VAE(vargs).to(dev)
    for prm in model.parameters():
        prm.grad = torch.randn_like(prm)
    scal = {f"s{i}": torch.rand((), device=dev) for i in range(8)}

    def ref_syncs():
        ok = True
        for prm in model.parameters():
            if prm.grad is not None:
                ok = ok and not (torch.isnan(prm.grad).any() or torch.isinf(prm.grad).any())
        return ok, [v.item() for v in scal.values()]

    def batched_syncs():
        return ms.has_finite_grad(model), ms.step_scalars(**scal)

    for name, fn in (("step_syncs_reference", ref_syncs), ("step_syncs_batched", batched_syncs)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(cli.reps):
            fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = round((time.perf_counter() - t0) / cli.reps * 1e3, 4)
    t0 = time.perf_counter()
    of.fair_penalty(lz_np, fz_np, labels, sens, dists, "l1", 0.5)
    res["fairness_cpu_oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    t0 = time.perf_counter()
    of.train_metrics(fz_np, labels.astype(np.float32), 0.5)
    res["metrics_cpu_oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    res["config"] = {"B": B, "L": L, "targets": T, "groups": int(len(np.unique(sens, axis=0))),
                     "norm": "l1", "cpu_threads": 1}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
