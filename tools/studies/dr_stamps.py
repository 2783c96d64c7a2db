"""Where a dR16s slot goes: s_memtime stamps at the slot
boundaries of workgroup 0's 8 waves over its first 64 stages, from a study
build of the library (MPV_DR_STAMPS=1):

  cd mpvae-1_amd && hipcc ... -DMPV_DR_STAMPS=1 -c csrc/probit_bwd.hip -o ../scratch/drS/probit_bwd.o
  (link with the other objects into scratch/drS/libmpvae_hip.so)
  MPVAE_HIP_LIB=scratch/drS/libmpvae_hip.so python tools/studies/dr_stamps.py [B S L z] > out.json

Stamp points per stage i (dR16s_kernel, DR_G0_STAGE / DR_G1_STAGE):
  0 slot start, 1 group 0 after its LDS-DMA issue, 2 after the fragment reads
  and lds_barrier, 3 after the MFMA issue, 4 group 0 after wait_vmcnt(0) (its
  DMA of stage i+1 landed), 5 after the closing barrier.
Reports, per group, the median length (s_memtime ticks: shader-clock cycles)
of each phase and of the slot pair (one stage).  Group 0's mem slot is
points 0-2, its MFMA slot 2-5; group 1's mem slot 0-2, MFMA slot 2-5, one
slot later."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpvae_hip  # noqa: E402
from mpvae_ops import HipShardBackend  # noqa: E402

B, S, L, z = (int(a) for a in sys.argv[1:5]) if len(sys.argv) >= 5 else (512, 4096, 1024, 1024)
DEV = "cuda:0"
g = torch.Generator(device=DEV).manual_seed(5)
y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
y[:, 0], y[:, 1] = 1, 0
fe = torch.randn((B, L), device=DEV, generator=g)
fx = torch.randn((B, L), device=DEV, generator=g)
R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * 0.03
be = HipShardBackend()
shape = be.shape(S, S, 0, B, L, z)
eps = be.make_noise(shape, DEV, 42, 0)
loc = be.forward_local(shape, y, fe, fx, be.prepare_R(R), eps, keep_T=True)
saved = dict(y=y, fe_out=fe, fx_out=fx, eps=eps, T=loc["T"], rowstat=loc["rowstat"],
             bstat=loc["bstat"])
gscal = torch.tensor([1.0, 0.0, 0.0, 0.0, 0.0, 0.0], device=DEV)
for _ in range(2):  # the second launch is the one read back
    be.backward_local(shape, saved, gscal, 0b000001, None, None, 0.1, 200.0, True)
torch.cuda.synchronize()
lib = mpvae_hip.load_library()
buf = (ctypes.c_ulonglong * (8 * 64 * 6))()
if lib.mpv_study_dr_stamps(buf) != 0:
    raise SystemExit("mpv_study_dr_stamps failed")
st = np.frombuffer(buf, dtype=np.uint64).reshape(8, 64, 6).astype(np.int64)


def med(x):
    return float(np.median(x))


out = {"shape": [B, S, L, z], "unit": "s_memtime ticks", "stages": 64}
n = 62  # skip the last stages of the window (the next stage's stamps bound them)
for grp, waves in (("group0", range(0, 4)), ("group1", range(4, 8))):
    w = st[list(waves)]
    r = {"slot_pair": med(w[:, 1:n + 1, 0] - w[:, 0:n, 0])}
    if grp == "group0":
        r.update(dma_issue=med(w[:, :n, 1] - w[:, :n, 0]), reads=med(w[:, :n, 2] - w[:, :n, 1]),
                 mfma_issue=med(w[:, :n, 3] - w[:, :n, 2]), dma_wait=med(w[:, :n, 4] - w[:, :n, 3]),
                 barrier=med(w[:, :n, 5] - w[:, :n, 4]))
    else:
        r.update(reads=med(w[:, :n, 2] - w[:, :n, 0]), mfma_issue=med(w[:, :n, 3] - w[:, :n, 2]),
                 barrier=med(w[:, :n, 5] - w[:, :n, 3]))
    out[grp] = r
print(json.dumps(out, indent=1))
