"""Count forward launches whose row statistics differ (bitwise) from the first
launch on identical inputs: python tools/repeat_probe.py B S L z runs"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

from mpvae_ops import HipShardBackend  # noqa: E402

B, S, L, z, runs = (int(a) for a in sys.argv[1:6])
keep_T = os.environ.get("PROBE_NO_T") != "1"
DEV = "cuda:0"
g = torch.Generator(device=DEV).manual_seed(5)
y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
y[:, 0], y[:, 1] = 1, 0
fe = torch.randn((B, L), device=DEV, generator=g)
fx = torch.randn((B, L), device=DEV, generator=g)
R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * 0.03
be = HipShardBackend()
shape = be.shape(S, S, 0, B, L, z)
Rop = be.prepare_R(R)
eps = be.make_noise(shape, DEV, 42, 0)
first = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=keep_T)["rowstat"].clone()
bad_runs, bad_k = 0, set()
for _ in range(runs):
    rs = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=keep_T)["rowstat"]
    d = rs != first
    if d.any():
        bad_runs += 1
        bad_k |= set(torch.nonzero(d)[:, 0].tolist())
torch.cuda.synchronize()
print(f"{os.environ.get('MPVAE_HIP_LIB', 'default').split('/')[-2]} B={B} S={S} L={L}: "
      f"keep_T={keep_T} {bad_runs}/{runs} runs differ, stats {sorted(bad_k)}"
      + (f"; backward: {bad_g}/{runs} differ" if bwd else ""), flush=True)
