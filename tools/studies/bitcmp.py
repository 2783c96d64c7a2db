"""Bit-for-bit comparison of two library builds' backward outputs.

  MPVAE_HIP_LIB=<lib A> python tools/studies/bitcmp.py dump A.pt
  MPVAE_HIP_LIB=<lib B> python tools/studies/bitcmp.py dump B.pt
  python tools/studies/bitcmp.py cmp A.pt B.pt

Cases: binary labels at L = 1024 (every wave full), L = 1100 (masked
columns), soft labels, and a degenerate row (all labels 1: NaN row
coefficients) on the LDS-ring element pass; L = 500 and 200 (soft) on the
register one.  A change meant to keep every bit (an instruction-count trim)
must print "identical" for all of them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))
import torch  # noqa: E402

CASES = {"binary_L1024": (16, 512, 1024, 256, "binary"), "binary_L1100": (16, 512, 1100, 256, "binary"),
         "soft_L1024": (8, 512, 1024, 256, "soft"), "dead_row_L1024": (8, 512, 1024, 256, "dead"),
         "binary_L500": (16, 512, 500, 256, "binary"), "soft_L200": (16, 256, 200, 64, "soft")}


def dump(path):
    from mpvae_ops import HipShardBackend
    dev = "cuda:0"
    be = HipShardBackend()
    out = {}
    for name, (B, S, L, z, kind) in CASES.items():
        g = torch.Generator(device=dev).manual_seed(7)
        y = (torch.rand((B, L), device=dev, generator=g) < 0.15).float()
        y[:, 0], y[:, 1] = 1, 0
        if kind == "soft":
            y[1:3, 5:40] = 0.3
        if kind == "dead":
            y[3, :] = 1.0
        fe = torch.randn((B, L), device=dev, generator=g)
        fx = torch.randn((B, L), device=dev, generator=g)
        R = (torch.rand((L, z), device=dev, generator=g, dtype=torch.float64) * 2 - 1) * 0.03
        shape = be.shape(S, S, 0, B, L, z)
        Rop = be.prepare_R(R)
        eps = be.make_noise(shape, dev, 42, 0)
        gscal = torch.tensor([1.0, 0.0, 0.0, 0.0, 0.0, 0.0], device=dev)
        loc = be.forward_local(shape, y, fe, fx, Rop, eps, keep_T=True)
        saved = dict(y=y, fe_out=fe, fx_out=fx, eps=eps, T=loc["T"], rowstat=loc["rowstat"],
                     bstat=loc["bstat"])
        flat, _, _ = be.backward_local(shape, saved, gscal, 0b000001, None, None, 0.1, 200.0, True)
        torch.cuda.synchronize()
        out[name] = flat.detach().cpu().clone()
    torch.save(out, path)
    print("dumped", path, {k: tuple(v.shape) for k, v in out.items()})


def cmp(pa, pb):
    a, b = torch.load(pa, weights_only=True), torch.load(pb, weights_only=True)
    bad = 0
    for k in a:
        x, y = a[k].contiguous(), b[k].contiguous()
        same = x.shape == y.shape and torch.equal(x.view(torch.int32), y.view(torch.int32))
        nd = int((x.view(torch.int32) != y.view(torch.int32)).sum()) if x.shape == y.shape else -1
        nan = int(torch.isnan(x).sum())
        print(f"{k}: {'identical' if same else 'DIFFERENT'} ({nd} of {x.numel()} differ, {nan} NaN)")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
