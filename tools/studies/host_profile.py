"""Host (Python) time of one eager bench step at a small configuration, where
the eager step is host-bound (C2: ~0.3 ms eager against 0.13 ms as a HIP
graph): cProfile over N steps of bench.step, the device synchronised only at
the end, top functions by own time.

  python tools/studies/host_profile.py [--config c2] [--steps 200]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpvae-1_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--steps", type=int, default=200)
cli = ap.parse_args()
L, z, B, S, d, nll_coeff, c_coeff = bench.CONFIGS[cli.config]
dev = torch.device("cuda:0")
y, leaves = bench.make_inputs(L, z, B, d, dev)
args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S, mode="train",
                          nll_coeff=nll_coeff, c_coeff=c_coeff, mpvae_noise="philox")
for it in range(20):
    bench.step(y, leaves, args, it)
torch.cuda.synchronize()
t0 = time.perf_counter()
for it in range(cli.steps):
    bench.step(y, leaves, args, it)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / cli.steps * 1e3
prof = cProfile.Profile()
prof.enable()
for it in range(cli.steps):
    bench.step(y, leaves, args, it)
torch.cuda.synchronize()
prof.disable()
out = io.StringIO()
pstats.Stats(prof, stream=out).sort_stats("tottime").print_stats(30)
print(f"{cli.config}: eager step {wall:.4f} ms (wall, no profiler)")
print(out.getvalue())
