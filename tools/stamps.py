"""Read the dR16 in-kernel phase stamps of an MPV_ABL&1024 build (timing study).

    MPVAE_HIP_LIB=abl/<variant>/libmpvae_hip.so python tools/stamps.py
Runs two C4 steps through bench.py's step(), then prints per-phase cycle
counts (median over iterations 256..287 of blocks 0-1) for every wave.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import mpvae_hip as H  # noqa: E402

dev = torch.device("cuda", 0)
L, z, B, S, d, nllc, cc, _ = bench.CONFIGS["c4"]
args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S, mode="train",
                          nll_coeff=nllc, c_coeff=cc, mpvae_noise="philox", mpvae_shard=False,
                          mpvae_gemm="f16x3")
y, leaves = bench.make_inputs(L, z, B, d, dev)
print("stepping", flush=True)
for it in range(2):
    bench.step(y, leaves, args, it)
torch.cuda.synchronize()
lib = H.load_library()
buf = np.zeros((2, 8, 32, 4), np.uint64)
fn = lib.mpv_dbg_dr_stamps
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
st = buf.astype(np.int64)
KIND = int(os.environ.get("STAMP_KIND", "0"))
names = (["wait(vmcnt)", "barrier", "dma issue", "reads+mfma issue"] if KIND == 0 else
         ["A:issue|B:reads", "A:reads+bar|B:bar", "A:mfma+wait|B:mfma", "bar->next"])
for blk in range(2):
    for w in range(8):
        t = st[blk, w]
        ph = [t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[1:, 0] - t[:-1, 3]]
        print(f"block {blk} wave {w}: " + "  ".join(f"{n} {int(np.median(p))}" for n, p in zip(names, ph))
              + f"  iter {int(np.median(t[1:, 0] - t[:-1, 0]))}")

fn = getattr(lib, "mpv_dbg_fwd_stamps", None)
if fn is not None:
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    fb = np.zeros((2, 8, 32, 4), np.uint64)
    eb = np.zeros((2, 8, 8, 6), np.uint64)
    assert fn(fb.ctypes.data, eb.ctypes.data) == 0
    st, ep = fb.astype(np.int64), eb.astype(np.int64)
    np.savez(os.path.join(ROOT, "gpurun_out", "stamps_raw.npz"), fwd=st, epi=ep)
    names = ["wait(vmcnt)", "barrier", "dma issue", "reads+mfma issue"]
    enames = ["T store", "label loop", "row sums", "rowpart", "tail"]
    for blk in range(2):
        for w in range(8):
            t = st[blk, w]
            ph = [t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[1:, 0] - t[:-1, 3]]
            e = ep[blk, w]
            print(f"fwd block {blk} wave {w}: " +
                  "  ".join(f"{n} {int(np.median(p))}" for n, p in zip(names, ph)) +
                  f"  iter {int(np.median(t[1:, 0] - t[:-1, 0]))}  epilogue {int(np.median(e[:, 5] - e[:, 0]))}"
                  f" [" + " ".join(f"{n} {int(np.median(e[:, k + 1] - e[:, k]))}" for k, n in enumerate(enames)) +
                  f"]  tile {int(np.median(e[1:, 0] - e[:-1, 0]))}")
