"""numpy restatement of the fairness regulariser and the per-step train
metrics -- TEST INFRASTRUCTURE ONLY (the checker of csrc/fairness.hip).

fair_penalty      reference fairsoft_train.py:75-131: row weights from the
                  label-string dict (:85-93), weighted batch mean (:97-101) and
                  per-sensitive-group means (:103-128) of indiv_prob_label
                  (label_z) and indiv_prob (feat_z), l1 / l2 distances,
                  fairloss = fair_coeff * (reg_label + reg_feat) (:130-131);
                  fp64 as in the reference (its weights tensor is float64).
                  Also the analytic gradient w.r.t. label_z and feat_z.
train_metrics     reference evals.py:178-238 with all_metrics=False, built
                  from the helpers at evals.py:13-117.

Pinning: tests/test_oracle_fair.py checks both against golden vectors that
tests/golden/make_golden_fair.py records by running the reference's own
code (evals.py imported by path; the fairsoft_train.py:75-136 block executed
from its source text -- the module itself needs tensorboard, absent here).
"""
import numpy as np


def row_weights(labels, dist):
    """fairsoft_train.py:89-93: dict lookup of ''.join(label.astype(int).astype(str))."""
    out = np.zeros(labels.shape[0], np.float64)
    for b, row in enumerate(labels):
        out[b] = float(dist.get("".join(row.astype(int).astype(str)), 0.0))
    return out


def fair_penalty(label_z, feat_z, labels, sensitive, dists, norm, coeff):
    """-> (fairloss or None when no term is active, contributed count,
    d fairloss / d label_z, d fairloss / d feat_z)."""
    lz, fz = np.asarray(label_z, np.float64), np.asarray(feat_z, np.float64)
    B, L = lz.shape
    groups = np.unique(sensitive, axis=0)
    gid = np.array([np.flatnonzero((groups == s).all(1))[0] for s in sensitive])
    reg, gl, gf, contributed, active = 0.0, np.zeros((B, L)), np.zeros((B, L)), 0, False
    for dist in dists:
        w = row_weights(labels, dist)
        contributed += int((w > 0).sum())
        W = w.sum()
        if not W > 0:
            continue
        for z, g in ((lz, gl), (fz, gf)):
            m = (z * w[:, None]).sum(0) / W
            esum = np.zeros(L)
            for k in range(len(groups)):
                mask = gid == k
                Wk = w[mask].sum()
                if not Wk > 0:
                    continue
                mk = (z[mask] * w[mask, None]).sum(0) / Wk
                d = mk - m
                if norm == "l1":
                    reg += np.abs(d).sum()
                    fp = np.sign(d)
                elif norm == "l2":
                    reg += (d ** 2).sum()
                    fp = 2.0 * d
                else:
                    continue
                active = True
                g[mask] += coeff * w[mask, None] * fp[None, :] / Wk
                esum += fp
            g -= coeff * w[:, None] * esum[None, :] / W
    loss = coeff * reg if active else None
    return loss, contributed, gl, gf


def train_metrics(pred, target, thr):
    """evals.compute_metrics(pred, target, thr, all_metrics=False) values
    [ACC, HA, ebF1, miF1, maF1, p@1, p@3, p@5]; p@k ties to the larger index."""
    pred, t = np.asarray(pred, np.float32), np.asarray(target, np.float32)
    B, L = pred.shape
    prec = []
    for k in (1, 3, 5):
        hits = []
        for b in range(B):
            order = sorted(range(L), key=lambda l: (pred[b, l], l), reverse=True)[:k]
            hits.append(sum(t[b, l] == 1.0 for l in order) / k)
        prec.append(np.mean(hits))
    p = np.where(pred < thr, 0.0, 1.0).astype(np.float32)
    acc = np.mean(np.all(t == p, axis=1))
    ha = 1.0 - np.mean(np.mean(np.logical_xor(t, p), axis=1))
    tp_r = np.sum(t * p, axis=1).astype(np.float32)
    den = np.sum(t, axis=1).astype(np.float32) + np.sum(p, axis=1).astype(np.float32)
    keep = den != 0
    ebf1 = np.mean((2 * tp_r[keep]) / den[keep]) if keep.any() else np.nan
    tp = np.sum(t * p, axis=0).astype(np.float32)
    fp = np.sum(np.logical_not(t) * p, axis=0).astype(np.float32)
    fn = np.sum(t * np.logical_not(p), axis=0).astype(np.float32)
    mi = 2 * np.sum(tp) / float(2 * np.sum(tp) + np.sum(fp) + np.sum(fn))
    f = (2 * tp) / (2 * tp + fp + fn + np.float32(1e-6))
    ma = np.mean(f[np.isfinite(f)])
    return np.array([acc, ha, ebf1, mi, ma] + prec, np.float64)
