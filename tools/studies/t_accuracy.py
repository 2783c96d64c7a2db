"""Accuracy of the noise product t = eps R^T that the forward kernels keep in
T, against the fp64 product rounded once: the 3xf16 split GEMM, the exact-fp32
MFMA mode and torch's fp32 matmul (the reference's own tensordot arithmetic),
at a C4/C5-like K.  Reports, per mode, max and rms |t - t64| in units of
ulp(t64) and the mean signed error (a bias would add up over the labels of the
per-sample log-likelihood).  Writes gpurun_out/t_accuracy.json.

    python tools/studies/t_accuracy.py [z] [B] [S]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

from mpvae_ops import HipShardBackend  # noqa: E402

DEV = "cuda:0"
z = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
S = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
L = z
g = torch.Generator(device=DEV).manual_seed(3)
y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
fe = torch.randn((B, L), device=DEV, generator=g)
fx = torch.randn((B, L), device=DEV, generator=g)
R = ((torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1)
     * (6.0 / (L + z)) ** 0.5)
Rt32 = R.float()
res = {"z": z, "B": B, "S": S, "modes": {}}


def stats(t, t64):
    d = t.double() - t64
    mag = torch.floor(torch.log2(t64.abs().clamp_min(1e-30)))
    ulp = torch.finfo(torch.float32).eps * torch.exp2(mag)
    u = d / ulp
    return {"max_ulp": float(u.abs().max()), "rms_ulp": float(u.pow(2).mean().sqrt()),
            "mean_ulp": float(u.mean()), "mean_abs_err": float(d.abs().mean()),
            "mean_signed_err": float(d.mean()), "rms_t": float(t64.pow(2).mean().sqrt())}


# the fp32 noise (what the reference would hold) and the fp64 product of the
# fp32 operands, rounded once: the target every mode approximates
shape = HipShardBackend("f32").shape(S, S, 0, B, L, z)
e32 = HipShardBackend("f32").make_noise(shape, DEV, 77, 0)      # (S, B, z)
t64 = (e32.double().reshape(-1, z) @ Rt32.double().t()).view(S, B, L).permute(1, 0, 2)
t32 = (e32.reshape(-1, z) @ Rt32.t()).view(S, B, L).permute(1, 0, 2)
res["modes"]["torch_fp32_matmul"] = stats(t32, t64)
del t32
for gemm in ("f16x3", "f32"):
    be = HipShardBackend(gemm)
    Rop = be.prepare_R(R)
    eps = be.make_noise(shape, DEV, 77, 0)
    loc = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=True)
    res["modes"][gemm] = stats(loc["T"][:, :, :L], t64)
    if gemm == "f16x3":  # the GEMM alone: against the product of the split values
        ev = eps.value()[:B * S, :z].view(B, S, z).double()
        rv = Rop.value()[:L, :z].double()
        tp = ev @ rv.t()
        res["modes"]["f16x3_vs_split_operands"] = stats(loc["T"][:, :, :L], tp)
        del ev, rv, tp
    del loc, eps
    torch.cuda.empty_cache()
for k, v in res["modes"].items():
    print(k, {a: f"{b:.3g}" for a, b in v.items()}, flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "t_accuracy.json"), "w"), indent=1)
