"""Count forward launches whose row statistics differ (bitwise) from the first
launch on identical inputs: python tools/repeat_probe.py B S L z runs

Every output and workspace buffer is NaN-poisoned before each launch
(HipShardBackend(poison=True); PROBE_NO_POISON=1 turns it off), so a store
that is skipped or lost shows as a NaN (counted separately) instead of
hiding behind the bytes an identical earlier launch left behind."""
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
if os.environ.get("PROBE_SWAP") == "1":  # the two branches' means exchanged
    fe, fx = fx, fe
R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * 0.03
be = HipShardBackend(poison=os.environ.get("PROBE_NO_POISON") != "1")
shape = be.shape(S, S, 0, B, L, z)
Rop = be.prepare_R(R)
eps = be.make_noise(shape, DEV, 42, 0)
gscal = torch.tensor([1.0, 0.0, 0.0, 0.0, 0.0, 0.0], device=DEV)
bwd = os.environ.get("PROBE_BWD") == "1"


def one(keep):
    loc = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=keep or bwd)
    if os.environ.get("PROBE_T") == "1" and keep:  # compare the T stash too
        return loc["rowstat"].clone(), loc["T"][..., :L].clone()  # pad columns: unwritten
    if not bwd:
        return loc["rowstat"].clone(), None
    saved = dict(y=y, fe_out=fe, fx_out=fx, eps=eps, T=loc["T"], rowstat=loc["rowstat"],
                 bstat=loc["bstat"])
    flat, _, _ = be.backward_local(shape, saved, gscal, 0b000001, None, None, 0.1, 200.0, True)
    return loc["rowstat"].clone(), flat.clone()


first, gfirst = one(True)
bad_runs, bad_k, bad_g, nan_runs = 0, set(), 0, 0
detail = os.environ.get("PROBE_DETAIL") == "1"
shown = 0
for _ in range(runs):
    rs, gr = one(keep_T)
    if not torch.isfinite(rs).all() or (gr is not None and not torch.isfinite(gr).all()):
        nan_runs += 1  # an unwritten (still poisoned) output element
    d = rs != first
    if d.any():
        bad_runs += 1
        bad_k |= set(torch.nonzero(d)[:, 0].tolist())
        if detail and shown < 4:
            # which (stat, b, s) differ, by how much, and in how many
            # (b, 16-sample block) groups; the first launch as the reference
            shown += 1
            idx = torch.nonzero(d)
            blocks = sorted({(int(b), int(s) // 16) for _, b, s in idx.tolist()})
            print(f"  run differs in {idx.shape[0]} entries, {len(blocks)} (b, s//16) blocks "
                  f"{blocks[:6]}", flush=True)
            for k, b, s_ in idx[:6].tolist():
                a, c = float(first[k, b, s_]), float(rs[k, b, s_])
                print(f"    k={k} b={b} s={s_}: {a:.9g} -> {c:.9g} (diff {c - a:.6g})", flush=True)
    if (bwd or gr is not None) and not torch.equal(gr, gfirst):
        bad_g += 1
        if detail and not bwd:
            dt = torch.nonzero(gr != gfirst)
            print(f"  T differs in {dt.shape[0]} elements, first {dt[:4].tolist()}", flush=True)
torch.cuda.synchronize()
print(f"{os.environ.get('MPVAE_HIP_LIB', 'x/default/x').split('/')[-2]} B={B} S={S} L={L}: "
      f"keep_T={keep_T} {bad_runs}/{runs} runs differ, stats {sorted(bad_k)}, "
      f"{nan_runs}/{runs} with unwritten (NaN) outputs"
      + (f"; backward/T: {bad_g}/{runs} differ" if (bwd or gfirst is not None) else ""),
      flush=True)
