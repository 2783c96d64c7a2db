"""Drift between the forward's eps sharers (timing study MPV_ABL & 524288:
csrc/probit_fwd.hip writes per-workgroup tile start times to
gpurun_out/fwd_study_<n>.bin).  python tools/fwd_drift.py <file> [nNt]"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 40).astype(np.int64)
nNt = int(sys.argv[2]) if len(sys.argv) > 2 else 4
nblk = a.shape[0]
t0 = a[:, 0][a[:, 0] > 0].min()
start, end = a[:, :32] - t0, a[:, 32] - t0
xcc = a[:, 34] & 15
ids = np.arange(nblk)
q, r = ids // (8 * nNt), ids % (8 * nNt)
nt, g = r // 8, q * 8 + r % 8
tile = np.median((end - start[:, 0]) / 32)  # ticks per tile (100 MHz)
stage = tile / 32
print(f"blocks {nblk}, launch {(end.max()) / 100:.0f} us, tile {tile / 100:.2f} us, "
      f"stage {stage / 100:.3f} us")
G = g.max() + 1
sp_start, sp_mid, sp_end, same_xcc = [], [], [], 0
for gg in range(G):
    m = np.where(g == gg)[0]
    if len(m) != nNt:
        continue
    same_xcc += len(set(xcc[m])) == 1
    sp_start.append(np.ptp(start[m, 0]))
    sp_mid.append(np.ptp(start[m, 16]))
    sp_end.append(np.ptp(end[m]))
for name, v in (("start", sp_start), ("tile 16", sp_mid), ("end", sp_end)):
    v = np.array(v) / stage
    print(f"sharer spread at {name:8s} (stages): median {np.median(v):6.1f}  p90 "
          f"{np.percentile(v, 90):6.1f}  max {v.max():6.1f}")
print(f"groups with all sharers on one XCC: {same_xcc} / {G}")
# dispatch waves: start times of block 0's successors
order = np.argsort(start[:, 0])
print("first-tile start (us) by dispatch rank 0/255/256/511/2047:",
      [round(start[order[i], 0] / 100, 1) for i in (0, 255, 256, 511, nblk - 1)])
