"""Run each stage of the HIP path twice on identical inputs and report which
buffers differ (bitwise), and where: noise planes, forward rowstat / bstat /
colsum / T, finalize outputs, backward buffers.

    python tools/studies/determinism_probe.py B S L z [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

from mpvae_ops import HipShardBackend  # noqa: E402

B, S, L, z = (int(a) for a in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 4
DEV = "cuda:0"
g = torch.Generator(device=DEV).manual_seed(5)
y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
y[:, 0], y[:, 1] = 1, 0
fe = torch.randn((B, L), device=DEV, generator=g)
fx = torch.randn((B, L), device=DEV, generator=g)
R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * 0.03
be = HipShardBackend()
shape = be.shape(S, S, 0, B, L, z)


def diff(name, a, b):
    if torch.equal(a, b):
        return f"{name}: same"
    d = (a.double() - b.double()).abs()
    idx = torch.nonzero(d.reshape(-1) > 0)
    return (f"{name}: DIFFER at {idx.numel()} of {d.numel()} (max {float(d.max()):.3g}, "
            f"first flat idx {idx[:6].reshape(-1).tolist()}, shape {tuple(a.shape)})")


runs = []
for r in range(reps):
    Rop = be.prepare_R(R)
    eps = be.make_noise(shape, DEV, 42, 0)
    loc = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=True)
    torch.cuda.synchronize()
    runs.append(dict(R=Rop.data.clone(), eps=eps.data.clone(), rowstat=loc["rowstat"].clone(),
                     bstat=loc["bstat"].clone(), colsum=loc["colsum"].clone(), T=loc["T"].clone()))
    gscal = torch.tensor([1.0, 0.0, 0.0, 0.0, 0.0, 0.0], device=DEV)
    saved = dict(y=y, fe_out=fe, fx_out=fx, eps=eps, T=loc["T"], rowstat=loc["rowstat"],
                 bstat=loc["bstat"])
    flat, _, _ = be.backward_local(shape, saved, gscal, 0b000001, None, None, 0.1, 200.0, True)
    torch.cuda.synchronize()
    runs[-1]["grads"] = flat.clone()
for r in range(1, reps):
    print(f"--- run {r} vs run 0")
    for k in runs[0]:
        print(" ", diff(k, runs[r][k], runs[0][k]))

# where rowstat differs: (k, b, s), each run's value, and N / P recomputed in
# fp64 from the run's own T (identical across runs) for the suspicious rows
rs = [r["rowstat"] for r in runs]
bad = torch.zeros_like(rs[0], dtype=torch.bool)
for r in rs[1:]:
    bad |= r != rs[0]
idx = torch.nonzero(bad)
print("differing (k, b, s):", idx.shape[0])
T = runs[0]["T"][..., :L].double()                                # (B, S, L)
u_e = T + fe.double()[:, None, :]
E = 0.5 * (1 + torch.erf(u_e / 2 ** 0.5)) * (1 - 1e-6) + 0.5e-6
neg = (y == 0).double()[:, None, :]
pos = (y == 1).double()[:, None, :]
Nref = (torch.exp(5 * E) * neg).sum(-1)                           # (B, S)
Pref = (torch.exp(-5 * E) * pos).sum(-1)
LPref = (torch.log(E) * pos + torch.log(1 - E) * neg).sum(-1)
for k, b, s in idx[:60].tolist():
    ref = {0: LPref, 2: Pref, 3: Nref}.get(k)
    print(f"  k={k} b={b} s={s}: runs {[round(float(r[k, b, s]), 4) for r in rs]}"
          + (f" ref {float(ref[b, s]):.4f}" if ref is not None else ""))
# which lanes / rows: s mod 128 (position in the tile) histogram
if idx.shape[0]:
    pos_in_tile = (idx[:, 2] % 128).tolist()
    print("sample rows (s):", sorted(set(idx[:, 2].tolist()))[:80])
    print("positions in 128-tile:", sorted(set(pos_in_tile))[:64])
    print("batch rows:", sorted(set(idx[:, 1].tolist()))[:64])
    print("stats k:", sorted(set(idx[:, 0].tolist())))
