"""Golden vectors for the fairness regulariser and the per-step train metrics.

Runs ONLY in the build container, where the reference is mounted at
/root/reference (it never travels to the GPU box).  The outputs come from the
reference's own code:

  * evals.compute_metrics (reference evals.py:178-238), imported by file path
    (it needs numpy + scikit-learn, both present), with all_metrics=False as
    the training loop calls it (fairsoft_train.py:149-153);
  * the fairness block of train_mpvae_softfair_one_epoch (fairsoft_train.py,
    from ``if penalize_unfair:`` through ``smooth_reg_fair +=
    fairloss.item()``), executed from the file's source text in a namespace
    that provides the loop's variables.  The module itself cannot be imported
    here (fairsoft_train -> main -> train -> tensorboard, absent), and the
    block is inline in the training function.  Recorded: fairloss (None when
    the reference leaves it a Python float), contributed_reg_fair_sample, and
    the gradients of fairloss w.r.t. indiv_prob_label and indiv_prob.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fair.py
Writes: tests/golden/fair_*.npz, tests/golden/metrics_*.npz
"""
import argparse
import importlib.util
import json
import os
import textwrap

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def load_evals():
    spec = importlib.util.spec_from_file_location("_ref_evals", os.path.join(REF, "evals.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def fairness_block():
    """The reference's fairness block (fairsoft_train.py, first training loop), dedented."""
    lines = open(os.path.join(REF, "fairsoft_train.py")).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.strip() == "if penalize_unfair:")
    end = next(i for i in range(start, len(lines))
               if "smooth_reg_fair += fairloss.item()" in lines[i])
    return textwrap.dedent("\n".join(lines[start:end + 1])), (start + 1, end + 1)


class _Data:
    pass


def run_fair_case(block, labels, sens, dists, targets, norm, coeff, seed, pyfloat=False):
    rng = np.random.default_rng(seed)
    B, L = labels.shape
    lz = torch.tensor(rng.uniform(0.01, 0.99, (B, L)), dtype=torch.float32, requires_grad=True)
    fz = torch.tensor(rng.uniform(0.01, 0.99, (B, L)), dtype=torch.float32, requires_grad=True)
    base = torch.tensor(1.25, dtype=torch.float32, requires_grad=True)
    data = _Data()
    data.labels, data.sensitive_feat = labels, sens
    ns = dict(torch=torch, np=np, penalize_unfair=True, indiv_prob_label=lz, indiv_prob=fz,
              data=data, idx=np.arange(B), args=argparse.Namespace(
                  device="cpu", fairness_loss_norm=norm, fair_coeff=coeff),
              target_fair_labels=targets, label_distances=dists, contributed_reg_fair_sample=0,
              total_loss=base * 1.0, smooth_reg_fair=0.0)
    exec(block, ns)
    fl = ns["fairloss"]
    rec = dict(label_z=lz.detach().numpy(), feat_z=fz.detach().numpy(), labels=labels,
               sensitive=sens, norm=np.array(norm), coeff=np.array(coeff),
               contributed=np.array(ns["contributed_reg_fair_sample"]),
               dists=np.array(json.dumps([{k: float(v) for k, v in dists[t].items()}
                                          for t in targets])),
               pyfloat=np.array(int(pyfloat)))
    if isinstance(fl, float):
        rec["active"] = np.array(0)
        rec["fairloss"] = np.array(fl)
    else:
        fl.backward()
        rec["active"] = np.array(1)
        rec["fairloss"] = np.array(fl.item())
        rec["ref_dtype"] = np.array(str(fl.dtype).replace("torch.", ""))
        rec["g_label_z"] = lz.grad.numpy()
        rec["g_feat_z"] = fz.grad.numpy()
        rec["total"] = np.array(ns["total_loss"].item())
    return rec


def make_dists(rng, labels, n_targets, n_extra, miss_rows=0, pyfloat=False):
    B, L = labels.shape
    keys = ["".join(r.astype(str)) for r in labels[miss_rows:]]
    extra = ["".join(rng.integers(0, 2, L).astype(str)) for _ in range(n_extra)]
    dists, targets = {}, []
    for t in range(n_targets):
        tk = "".join(rng.integers(0, 2, L).astype(str))
        # np.float64 values, as label_distance.py's np.clip(np.exp(...)) produces:
        # the reference's torch.tensor(weights) is then float64
        # pyfloat: Python floats, as label_distance_obs.py's indication (1.0 / 0.),
        # constant (1.0), and un-gamma'd Jaccard / Hamming (int / int) produce:
        # torch.tensor(weights) is then float32 and the whole penalty runs in fp32
        if pyfloat:
            d = {k: int(rng.integers(0, 4)) / 3 for k in keys + extra if rng.random() < 0.7}
        else:
            d = {k: np.float64(rng.uniform(0.05, 1.0)) for k in keys + extra
                 if rng.random() < 0.7}
        dists[tk] = d
        targets.append(tk)
    return dists, targets


def main():
    block, (a, b) = fairness_block()
    print(f"fairness block: fairsoft_train.py:{a}-{b}")
    cases = [  # name, B, L, n_sens_cols, n_targets, norm, coeff, seed, miss_rows, pyfloat
        ("f1_l1", 16, 12, 2, 2, "l1", 1.5, 1, 0, False),
        ("f2_l2", 16, 12, 2, 2, "l2", 0.7, 2, 0, False),
        ("f3_zero_group", 24, 20, 1, 3, "l1", 2.0, 3, 8, False),
        ("f4_l100", 32, 100, 2, 2, "l2", 1.0, 4, 0, False),
        ("f5_inactive", 8, 10, 1, 1, "l1", 1.0, 5, 8, False),
        ("f6_pyfloat_l1", 64, 24, 2, 2, "l1", 1.5, 6, 4, True),
        ("f7_pyfloat_l2", 64, 90, 2, 3, "l2", 0.8, 7, 0, True),
    ]
    for name, B, L, ns_, T, norm, coeff, seed, miss, pyf in cases:
        rng = np.random.default_rng(100 + seed)
        labels = (rng.random((B, L)) < 0.3).astype(np.int64)
        labels[B // 2:, :] = labels[:B - B // 2, :]  # repeated patterns
        sens = rng.integers(0, 2, (B, ns_)).astype(np.int64)
        if name == "f3_zero_group":
            sens[:8, 0] = 5  # a group whose rows (the first 8) are all absent from the dicts
        dists, targets = make_dists(rng, labels, T, 4, miss_rows=miss if name != "f5_inactive"
                                    else B, pyfloat=pyf)
        rec = run_fair_case(block, labels, sens, dists, targets, norm, coeff, seed, pyfloat=pyf)
        np.savez(os.path.join(HERE, f"fair_{name}.npz"), **rec)
        print(name, "active", int(rec["active"]), "fairloss", float(rec["fairloss"]),
              str(rec.get("ref_dtype", "-")),
              "contributed", int(rec["contributed"]))

    ev = load_evals()
    keys = ["ACC", "HA", "ebF1", "miF1", "maF1", "p_at_1", "p_at_3", "p_at_5"]
    for name, B, L, seed, zero_rows in [("m1", 64, 20, 1, 0), ("m2_zero_rows", 48, 30, 2, 6),
                                        ("m3_l300", 16, 300, 3, 0)]:
        rng = np.random.default_rng(200 + seed)
        tgt = (rng.random((B, L)) < 0.25).astype(np.float32)
        tgt[0, 0], tgt[0, 1] = 1, 0
        pred = rng.random((B, L)).astype(np.float32)
        if zero_rows:
            tgt[1:1 + zero_rows] = 0
            pred[1:1 + zero_rows] = rng.random((zero_rows, L)).astype(np.float32) * 0.4
        m = ev.compute_metrics(pred.copy(), tgt.copy(), 0.5, all_metrics=False)
        vals = np.array([float(m[k]) for k in keys], np.float64)
        np.savez(os.path.join(HERE, f"metrics_{name}.npz"), pred=pred, target=tgt, values=vals)
        print(name, dict(zip(keys, np.round(vals, 6))))


if __name__ == "__main__":
    main()
