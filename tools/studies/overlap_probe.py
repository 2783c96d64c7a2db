"""Does running the next step's probit noise on a second HIP stream overlap with
the current step's GEMM kernels at C4?    The noise of
step i+1 depends only on its Philox key, so a pipeline could draw it beside
step i's forward or backward.  This times, at the headline size, each GEMM
phase alone, the noise kernel alone, both serialised on one stream, and both
issued on two streams (the noise on a side stream), with HIP events around
the pair; writes gpurun_out/overlap_probe.json.

    python tools/studies/overlap_probe.py [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

from mpvae_ops import HipShardBackend  # noqa: E402

DEV = "cuda:0"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B, S, L, z = 512, 4096, 1024, 1024
g = torch.Generator(device=DEV).manual_seed(5)
y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
y[:, 0], y[:, 1] = 1, 0
fe = torch.randn((B, L), device=DEV, generator=g)
fx = torch.randn((B, L), device=DEV, generator=g)
R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * 0.054
be = HipShardBackend()
shape = be.shape(S, S, 0, B, L, z)
Rop = be.prepare_R(R)
eps = be.make_noise(shape, DEV, 42, 0)
loc = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=True)
saved = dict(y=y, fe_out=fe, fx_out=fx, eps=eps, T=loc["T"], rowstat=loc["rowstat"],
             bstat=loc["bstat"])
gscal = torch.tensor([1.0, 0, 0, 0, 0, 0], device=DEV)
side = torch.cuda.Stream()
cur = torch.cuda.current_stream()
nxt = {}


def fwd():
    be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=True)


def bwd():
    be.backward_local(shape, saved, gscal, 0b000001, None, None, 0.1, 200.0, True)


def noise():
    nxt["eps"] = be.make_noise(shape, DEV, 43, 0)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(reps):
        a.record(cur)
        fn()
        b.record(cur)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    ms.sort()
    return ms[len(ms) // 2]


def serial(phase):
    def f():
        phase()
        noise()
    return f


def concurrent(phase):
    def f():
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            noise()
        phase()
        cur.wait_stream(side)
    return f


res = {"config": f"B={B} S={S} L=z={L}", "reps": reps, "median_ms": {}}
t0 = time.time()
for name, fn in (("noise", noise), ("forward", fwd), ("backward", bwd),
                 ("forward+noise serial", serial(fwd)), ("forward+noise two streams", concurrent(fwd)),
                 ("backward+noise serial", serial(bwd)),
                 ("backward+noise two streams", concurrent(bwd))):
    res["median_ms"][name] = round(timed(fn), 3)
    print(name, res["median_ms"][name], flush=True)
m = res["median_ms"]
res["saved_ms"] = {"forward": round(m["forward+noise serial"] - m["forward+noise two streams"], 3),
                   "backward": round(m["backward+noise serial"] - m["backward+noise two streams"], 3)}
print(json.dumps(res["saved_ms"]), f"({time.time() - t0:.1f} s)")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "overlap_probe.json"), "w"), indent=1)
