"""Golden record of compute_loss on empty inputs (reference mpvae.py:145-210).

Runs ONLY in the build container (the reference checkout at /root/reference
never travels to the GPU box); imports the reference's own ``mpvae.py`` the
way make_golden.py does and records, as JSON data:

  * a batch of 0 rows (n_sample 4, L = z = 6, d = 4), modes train and test:
    the dtype and shape of each of the 8 outputs, which scalars are NaN, and
    for each output used alone as the objective which inputs receive a
    gradient, with its shape and whether it is all zeros;
  * n_sample = 0 with a batch of 3: the exception type the reference raises.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_edge.py
Writes: tests/golden/edge_cases.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import load_reference  # noqa: E402

NAMES = ["fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar", "r_sqrt_sigma"]
L, Z, D = 6, 6, 4


def _inputs(B, seed):
    g = torch.Generator().manual_seed(seed)
    y = torch.zeros(B, L)
    if B:
        y[:, 0] = 1
    t = [torch.randn(B, n, generator=g).requires_grad_() for n in (L, D, D, L, D, D)]
    R = torch.from_numpy(np.random.default_rng(seed).uniform(-0.5, 0.5, (L, Z))).requires_grad_()
    return y, t + [R]


def _args(S, mode):
    return argparse.Namespace(label_dim=L, z_dim=Z, n_train_sample=S, n_test_sample=S, mode=mode,
                              nll_coeff=0.5, c_coeff=10.0)


def main():
    ref = load_reference()
    rec = {"L": L, "z": Z, "d": D, "nll_coeff": 0.5, "c_coeff": 10.0, "empty_batch": {}}
    for mode in ("train", "test"):
        y, leaves = _inputs(0, 1)
        out = ref.compute_loss(y, *leaves, _args(4, mode))
        case = {"outputs": [{"dtype": str(o.dtype).replace("torch.", ""), "shape": list(o.shape),
                             "nan": bool(o.dim() == 0 and torch.isnan(o).item())}
                            for o in out]}
        if mode == "train":
            grads = []
            for i in range(8):
                y, leaves = _inputs(0, 1)
                o = ref.compute_loss(y, *leaves, _args(4, mode))[i]
                o.sum().backward()
                grads.append({n: None if v.grad is None else
                              {"shape": list(v.grad.shape), "dtype": str(v.grad.dtype).replace(
                                  "torch.", ""), "zero": bool((v.grad == 0).all().item())}
                              for n, v in zip(NAMES, leaves)})
            case["grads_per_output"] = grads
        rec["empty_batch"][mode] = case
    y, leaves = _inputs(3, 2)
    try:
        ref.compute_loss(y, *leaves, _args(0, "train"))
        rec["zero_samples_raises"] = None
    except Exception as e:  # noqa: BLE001 -- recording which one the reference raises
        rec["zero_samples_raises"] = type(e).__name__
    path = os.path.join(HERE, "edge_cases.json")
    json.dump(rec, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
