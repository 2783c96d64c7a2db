"""Where the full-C4 gradient error comes from: the product (f16x3, f32) and the
reference's own fp32 arithmetic (t from an fp32 GEMM) against the fp64-t
restatement (tests/torch64_ref.py), per seed, plus the elements where the
largest differences sit.  Writes gpurun_out/c4_spread.json."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mpvae-1_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import mpvae  # noqa: E402
from torch64_ref import ChunkedElbo  # noqa: E402

DEV = "cuda:0"
OUTS = ["total", "nll", "nll_x", "c", "c_x", "kl", "indiv_prob", "indiv_prob_label"]


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max())


def case(seed, B=512, S=4096, L=1024, z=1024, d=50):
    g = torch.Generator(device=DEV).manual_seed(1000 + seed)
    y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
    y[:, 0], y[:, 1] = 1, 0
    fe = torch.randn((B, L), device=DEV, generator=g)
    fx = torch.randn((B, L), device=DEV, generator=g)
    mus = [torch.randn((B, d), device=DEV, generator=g) * s for s in (1.0, 0.1, 1.0, 0.1)]
    R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * \
        (6.0 / (L + z)) ** 0.5
    noise = torch.randn((S, B, z), device=DEV, generator=g)
    return y, fe, fx, mus, R, noise


def product(y, fe, fx, mus, R, noise, gemm):
    S, B, z = noise.shape
    L = y.shape[1]
    leaves = [x.clone().requires_grad_(True) for x in (fe, mus[0], mus[1], fx, mus[2], mus[3], R)]
    args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S,
                              mode="train", nll_coeff=0.1, c_coeff=200.0, mpvae_noise=noise,
                              mpvae_gemm=gemm)
    out = mpvae.compute_loss(y, *leaves, args)
    out[0].backward()
    res = {"fe_out": leaves[0].grad.detach().clone(), "fx_out": leaves[3].grad.detach().clone(),
           "r_sqrt_sigma": leaves[6].grad.detach().clone()}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[1, 2, 3])
    cli = ap.parse_args()
    rows = []
    for seed in cli.seeds:
        y, fe, fx, mus, R, noise = case(seed)
        S = noise.shape[0]
        grads = {}
        for gemm in ("f16x3", "f32"):
            grads[gemm] = product(y, fe, fx, mus, R, noise, gemm)
            torch.cuda.empty_cache()
        refs = {}
        for name, t32 in (("fp64_t", False), ("fp32_t", True)):
            ce = ChunkedElbo(y, fe, fx, R, lambda a, b: noise[a:b], S, 256, t_fp32=t32)
            ce.forward(*mus, 0.1, 200.0)
            refs[name] = ce.backward(0.1, 200.0, 1.0)
            del ce
        row = {"seed": seed}
        for k in ("fe_out", "fx_out", "r_sqrt_sigma"):
            r64 = refs["fp64_t"][k]
            row[k] = {"f16x3": rel(grads["f16x3"][k], r64), "f32": rel(grads["f32"][k], r64),
                      "ref_fp32_t": rel(refs["fp32_t"][k], r64),
                      "f16x3_vs_ref_fp32_t": rel(grads["f16x3"][k], refs["fp32_t"][k])}
            if k != "r_sqrt_sigma":
                d = (grads["f16x3"][k].double() - r64).abs()
                i = int(d.argmax())
                b, l = divmod(i, y.shape[1])
                row[k]["worst"] = {"b": b, "l": l, "y": float(y[b, l]),
                                   "ref": float(r64[b, l]), "got": float(grads["f16x3"][k][b, l]),
                                   "ref_fp32_t": float(refs["fp32_t"][k][b, l]),
                                   "max_abs_ref": float(r64.abs().max())}
        print(json.dumps(row), flush=True)
        rows.append(row)
        del grads, refs, noise
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "c4_spread.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
