"""Which host-side op launches each small device operation of one bench step
(the fixed cost that matters at n_sample 512, one rank's share at 8 GPUs):
torch.profiler over a few steps of bench.py's step function, device kernels,
memsets and memcpys grouped by the top-level op that issued them.

  python tools/studies/step_ops.py [--n-sample 512]

(The sharded path on a world-of-one RCCL group is profiled with a rocprofv3
kernel trace of MPVAE_FORCE_DIST=1 bench.py instead: under torch.profiler that
run reported no device activity.)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpvae-1_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n-sample", type=int, default=512)
ap.add_argument("--steps", type=int, default=3)
cli = ap.parse_args()
dev = torch.device("cuda:0")
L = z = 1024
y, leaves = bench.make_inputs(L, z, 512, 50, dev)
args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=cli.n_sample,
                          n_test_sample=cli.n_sample, mode="train", nll_coeff=0.1, c_coeff=200.0,
                          mpvae_noise="philox")
for it in range(3):
    bench.step(y, leaves, args, it)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts) as prof:
    for it in range(cli.steps):
        bench.step(y, leaves, args, 10 + it)
    torch.cuda.synchronize()
rows = []
for e in prof.key_averages():
    dt = getattr(e, "device_time_total", None)
    if dt is None:
        dt = getattr(e, "cuda_time_total", 0)
    if e.count and dt:
        rows.append({"op": e.key, "calls_per_step": e.count / cli.steps,
                     "device_us_per_step": dt / cli.steps})
rows.sort(key=lambda r: -r["device_us_per_step"])
print(json.dumps({"n_sample": cli.n_sample, "ops": rows[:60]}, indent=1), flush=True)
