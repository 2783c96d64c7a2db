"""Host-side (Python) cost of one eager compute_loss forward + backward:
cProfile of N calls at a small config.  python tools/studies/eager_profile.py [c2|c3]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

import mpvae  # noqa: E402

CFG = {"c2": (38, 38, 128, 1000), "c3": (81, 81, 256, 2000)}[sys.argv[1] if len(sys.argv) > 1 else "c2"]
L, z, B, S = CFG
dev = torch.device("cuda", 0)
args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S, mode="train",
                          nll_coeff=0.5, c_coeff=10.0, mpvae_noise="philox",
                          mpvae_seed=torch.tensor([5], dtype=torch.int64, device=dev))
g = torch.Generator(device=dev).manual_seed(0)
y = (torch.rand((B, L), device=dev, generator=g) < 0.2).float()
y[:, 0], y[:, 1] = 1, 0
ins = [torch.randn((B, L), device=dev, generator=g).requires_grad_(True),
       torch.randn((B, 50), device=dev, generator=g).requires_grad_(True),
       (torch.randn((B, 50), device=dev, generator=g) * 0.1).requires_grad_(True),
       torch.randn((B, L), device=dev, generator=g).requires_grad_(True),
       torch.randn((B, 50), device=dev, generator=g).requires_grad_(True),
       (torch.randn((B, 50), device=dev, generator=g) * 0.1).requires_grad_(True)]
R = torch.nn.Parameter(torch.rand((L, z), device=dev, dtype=torch.float64) * 0.1)


def step():
    res = mpvae.compute_loss(y, *ins, R, args)
    res[0].backward()


for _ in range(5):
    step()
torch.cuda.synchronize()
N = 200
t0 = time.perf_counter()
for _ in range(N):
    step()
t_host = (time.perf_counter() - t0) / N * 1e3
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / N * 1e3
prof = cProfile.Profile()
with torch.autograd.set_multithreading_enabled(False):  # backward on this thread: profiled
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        step()
    t_single = (time.perf_counter() - t0) / N * 1e3
    prof.enable()
    for _ in range(N):
        step()
    prof.disable()
torch.cuda.synchronize()
print(f"host issue {t_host:.3f} ms/step, with device {t_all:.3f} ms/step, "
      f"single-threaded autograd {t_single:.3f} ms/step", flush=True)
pstats.Stats(prof).sort_stats("tottime").print_stats(40)
