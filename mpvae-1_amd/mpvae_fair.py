"""Device versions of the two per-step consumers of compute_loss's
``indiv_prob`` / ``indiv_prob_label`` in the reference training loop
(SURVEY.md section 8(f), ranks 2 and 3):

* the fairness regulariser, fairsoft_train.py:75-138 -- per target fair label,
  row weights from ``label_distances[target]`` keyed by the row's label
  string (:85-93), the weighted batch mean and per-sensitive-group means of
  indiv_prob_label (label_z) and indiv_prob (feat_z), l1 or l2 distance,
  ``fairloss = fair_coeff * (reg_label_z_unfair + reg_feat_z_unfair)``;
* the per-step train metrics, ``evals.compute_metrics(indiv_prob, labels,
  0.5, all_metrics=False)`` (evals.py:178-238, used at fairsoft_train.py:149-153).

Both run in libmpvae_hip.so (csrc/fairness.hip) behind the C ABI; there is no
host fallback.  Differences from the reference, none of them numeric:
* the reference returns the Python float 0. when no target/group term is
  active (and then does not add it); ``fairness_penalty`` returns a zero
  fp64 tensor instead, which adds nothing -- deciding "float or tensor" would
  need a host sync every step;
* the penalty is computed in fp64 whatever the distance values are.  The
  reference's ``torch.tensor(weights)`` is float64 when the dict values are
  numpy float64 (label_distance*.py's ``np.clip(np.exp(...))``) and float32
  when they are Python floats (indication / constant / un-gamma'd Jaccard and
  Hamming), and the penalty then runs in fp32.  The returned loss takes the
  reference's dtype (fp32 when every table holds Python floats), its value
  differs from the reference's fp32 one by fp32 rounding only
  (tests/golden fair_f6/f7, tests/test_gpu_fair.py);
* the metrics come back as 0-d fp64 device tensors (``.item()`` works as on
  the reference's numpy scalars); p@k ties go to the larger label index
  (numpy's default argsort is not stable, so the reference's tie order is
  implementation-defined).
"""
import ctypes

import numpy as np
import torch

import mpvae_hip as H

_MIX = (0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB)
_M64 = (1 << 64) - 1


def _mix64(z):
    z = (z + _MIX[0]) & _M64
    z = ((z ^ (z >> 30)) * _MIX[1]) & _M64
    z = ((z ^ (z >> 27)) * _MIX[2]) & _M64
    return z ^ (z >> 31)


def pack_pattern(key, L):
    """The reference's key string (``''.join(label.astype(str))``) -> W words,
    bit j of word w = label 64w + j.  None if the string is not a 0/1 pattern
    of length L (such a key can never match a binary label row)."""
    if len(key) != L or any(c not in "01" for c in key):
        return None
    W = (L + 63) // 64
    words = [0] * W
    for i, c in enumerate(key):
        if c == "1":
            words[i // 64] |= 1 << (i % 64)
    return words


def pattern_hash(words):
    h = 0x6A09E667F3BCC909 ^ len(words)
    for x in words:
        h = _mix64(h ^ x)
    return h


class LabelDistanceTable:
    """One target label's ``label_distances[target]`` dict (label string ->
    distance) as a device open-addressing table (mpv_label_table).

    ``ref_dtype`` is decided once per table: float64 if any value is a numpy
    float64, else float32.  The reference decides per batch, from the values
    actually looked up (``torch.tensor(weights)``) and promoted over the
    targets that were active in that batch -- a data-dependent host decision.
    The two agree whenever a table's values share one type (every
    label_distance*.py table does); for a table mixing Python floats and numpy
    float64, or an fp64 table inactive in a batch beside an active fp32 one,
    the returned loss is fp64 where the reference's is fp32, a difference of
    fp32 rounding only (the arithmetic is fp64 here either way)."""

    def __init__(self, distances, label_dim, device):
        self.L, self.W = label_dim, (label_dim + 63) // 64
        # torch.tensor() of the looked-up values is float64 iff they are numpy
        # float64 (fairsoft_train.py:91-97); Python floats give float32
        self.ref_dtype = torch.float64 if any(isinstance(v, np.float64)
                                              for v in distances.values()) else torch.float32
        items = [(pack_pattern(k, label_dim), float(v)) for k, v in distances.items()]
        items = [(w, v) for w, v in items if w is not None]
        n = 1
        while n < 2 * max(1, len(items)):
            n *= 2
        keys = np.zeros((n, self.W), np.uint64)
        vals = np.zeros(n, np.float64)
        used = np.zeros(n, np.int32)
        for words, v in items:
            slot = pattern_hash(words) & (n - 1)
            while used[slot] and list(keys[slot]) != words:
                slot = (slot + 1) & (n - 1)
            keys[slot] = np.array(words, np.uint64)
            vals[slot] = v
            used[slot] = 1
        self.nslots = n if items else 0
        self.keys = torch.from_numpy(keys.view(np.int64).copy()).to(device)
        self.vals = torch.from_numpy(vals).to(device)
        self.used = torch.from_numpy(used).to(device)

    def c_struct(self):
        return H.LabelTable(H.ptr(self.keys), H.ptr(self.vals), H.ptr(self.used), self.nslots,
                            self.W)


def label_weights(labels, tables):
    """(T, B) fp64 row weights, one row per target table, and the int32 count
    of (target, row) pairs with a positive weight (fairsoft_train.py:85-93)."""
    H.require_gpu(labels)
    y = labels.contiguous().float()
    B, L = y.shape
    w = torch.empty((len(tables), B), dtype=torch.float64, device=y.device)
    count = torch.zeros((), dtype=torch.int32, device=y.device)
    lib, st = H.load_library(), H.stream_of(y.device)
    for t, tab in enumerate(tables):
        if tab.L != L:
            raise ValueError(f"table built for label_dim {tab.L}, labels have {L}")
        s = tab.c_struct()
        H.check(lib.mpv_label_weights(H.ptr(y), B, L, ctypes.byref(s), H.ptr(w[t]), H.ptr(count),
                                      st), "mpv_label_weights")
    return w, count


def group_ids(sensitive_feat):
    """Row b's index in ``torch.unique(sensitive_feat, dim=0)`` (the reference's
    group order, fairsoft_train.py:80, :103-104), from fixed-size tensor ops:
    the number of distinct rows that sort before row b (lexicographically).
    No data-dependent shape and no host sync, so it can be captured in a HIP
    graph; O(B^2 n_sensitive) compares, a few microseconds at B = 512."""
    X = sensitive_feat.reshape(sensitive_feat.shape[0], -1)
    B = X.shape[0]
    if B == 0:
        return torch.zeros(0, dtype=torch.int32, device=X.device)
    ne = X[:, None, :] != X[None, :, :]                         # [c, b, j]
    differ = ne.any(-1)                                         # rows c, b differ
    first = ne.to(torch.uint8).argmax(-1, keepdim=True)         # first differing column
    less = differ & (torch.gather(X[:, None, :].expand(B, B, X.shape[1]), 2, first) <
                     torch.gather(X[None, :, :].expand(B, B, X.shape[1]), 2, first)).squeeze(-1)
    # row c is the first occurrence of its pattern: no earlier identical row
    earlier = torch.ones(B, B, dtype=torch.bool, device=X.device).triu(1)  # [c', c]: c' < c
    firsts = ~((~differ) & earlier).any(0)
    return (less & firsts[:, None]).sum(0).to(torch.int32)


def sensitive_groups(sensitive_feat, max_groups=None):
    """(gid, order, goff, G, overflow): group id per row (``group_ids``), the
    rows listed group by group, and the group offsets, for G group slots.  G is
    ``max_groups`` (an upper bound on the distinct sensitive patterns of a
    batch, e.g. of the whole dataset, known on the host once) or the batch
    size: the slots past the batch's own groups stay empty, and an empty group
    adds nothing (its weight sum is 0, the reference's
    ``weight_sensitive.sum() > 0`` gate).  A batch with more distinct patterns
    than ``max_groups`` sets the 0-d bool device tensor ``overflow`` (its ids
    are clamped into range, so no kernel reads out of bounds; the penalty
    turns NaN).  Nothing here waits for the device."""
    gid = group_ids(sensitive_feat)
    B = gid.numel()
    G = int(max_groups) if max_groups is not None else max(B, 1)
    if G < 1:
        raise ValueError(f"max_groups must be >= 1 (got {max_groups})")
    overflow = (gid >= G).any()
    gid = gid.clamp(max=G - 1)
    order = torch.argsort(gid, stable=True).to(torch.int32)
    counts = torch.zeros(G, dtype=torch.int32, device=gid.device)
    counts.index_add_(0, gid.long(), torch.ones_like(gid))
    goff = torch.zeros(G + 1, dtype=torch.int32, device=gid.device)
    goff[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return gid.contiguous(), order.contiguous(), goff, G, overflow


class _FairPenalty(torch.autograd.Function):
    @staticmethod
    def forward(ctx, label_z, feat_z, w, gid, order, goff, G, norm, fair_coeff):
        lz, fz = label_z.detach().contiguous().float(), feat_z.detach().contiguous().float()
        B, L = lz.shape
        T = w.shape[0]
        lib, st = H.load_library(), H.stream_of(lz.device)
        nbytes = lib.mpv_fair_workspace_bytes(L, T, G)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=lz.device)
        out = torch.empty((), dtype=torch.float64, device=lz.device)
        a = H.FairArgs(H.ptr(lz), H.ptr(fz), H.ptr(w), H.ptr(order), H.ptr(goff), H.ptr(gid), B, L,
                       T, G, norm, float(fair_coeff), H.ptr(out))
        H.check(lib.mpv_fair_fwd(ctypes.byref(a), H.ptr(ws), nbytes, st), "mpv_fair_fwd")
        ctx.keep = (lz, fz, w, gid, order, goff, ws, a, nbytes)
        ctx.dtypes = (label_z.dtype, feat_z.dtype)
        return out

    @staticmethod
    def backward(ctx, gout):
        lz, fz, w, gid, order, goff, ws, a, nbytes = ctx.keep
        g = gout.detach().to(torch.float64).contiguous()
        gl, gf = torch.empty_like(lz), torch.empty_like(fz)
        lib = H.load_library()
        H.check(lib.mpv_fair_bwd(ctypes.byref(a), H.ptr(g), H.ptr(gl), H.ptr(gf), H.ptr(ws), nbytes,
                                 H.stream_of(lz.device)), "mpv_fair_bwd")
        return (gl.to(ctx.dtypes[0]), gf.to(ctx.dtypes[1])) + (None,) * 7


NORMS = {"l1": H.FAIR_L1, "l2": H.FAIR_L2}


def fairness_penalty(indiv_prob_label, indiv_prob, input_label, sensitive_feat, tables,
                     fairness_loss_norm, fair_coeff, max_groups=None):
    """fairsoft_train.py:75-131 on the device.

    indiv_prob_label, indiv_prob -- compute_loss outputs 8 and 7 (label_z, feat_z)
    input_label                   -- (B, L) batch labels (data.labels[idx])
    sensitive_feat                -- (B, n_sensitive) (data.sensitive_feat[idx])
    tables                        -- [LabelDistanceTable(label_distances[t], L, dev)
                                      for t in target_fair_labels]
    max_groups                    -- optional upper bound on the distinct sensitive
                                     patterns in a batch (default: the batch size;
                                     a batch with more distinct patterns than the
                                     bound makes the penalty NaN)
    No host sync: the call (forward and backward) can be captured in a HIP
    graph (tests/test_gpu_fair.py).
    Returns ``(fairloss, contributed)``: fairloss is a differentiable 0-d
    tensor to add to total_loss (zero when no term is active), computed in fp64
    and returned in the reference's dtype (fp64 if any table holds numpy
    float64 distances, else fp32), contributed the
    int32 count that the reference adds to contributed_reg_fair_sample."""
    H.require_gpu(indiv_prob_label, indiv_prob, input_label, sensitive_feat)
    w, count = label_weights(input_label, tables)
    gid, order, goff, G, overflow = sensitive_groups(sensitive_feat, max_groups)
    norm = NORMS.get(fairness_loss_norm, 0)
    loss = _FairPenalty.apply(indiv_prob_label, indiv_prob, w, gid, order, goff, G, norm,
                              fair_coeff)
    if max_groups is not None:  # G < B: a batch may hold more patterns than the bound
        loss = torch.where(overflow, torch.full_like(loss, float("nan")), loss)
    if tables and all(t.ref_dtype == torch.float32 for t in tables):
        loss = loss.float()
    return loss, count


METRIC_KEYS = ["ACC", "HA", "ebF1", "miF1", "maF1", "p_at_1", "p_at_3", "p_at_5"]


def compute_metrics(predictions, targets, threshold, all_metrics=False):
    """evals.compute_metrics (evals.py:178-238) for the per-step call
    (all_metrics=False): the same keys, the AUC/AUPR/FDR entries 0 as in the
    reference; values are 0-d fp64 device tensors."""
    if all_metrics:
        raise NotImplementedError("all_metrics=True (per-label AUC/AUPR/FDR curves, evaluation "
                                  "only) is not on the device path; use the reference's "
                                  "evals.compute_metrics on host arrays")
    H.require_gpu(predictions, targets)
    p = predictions.detach().contiguous().float()
    t = targets.detach().contiguous().float()
    B, L = p.shape
    lib = H.load_library()
    nbytes = lib.mpv_metrics_workspace_bytes(B, L)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=p.device)
    out = torch.empty(8, dtype=torch.float64, device=p.device)
    H.check(lib.mpv_train_metrics(H.ptr(p), H.ptr(t), B, L, float(threshold), H.ptr(out), H.ptr(ws),
                                  nbytes, H.stream_of(p.device)), "mpv_train_metrics")
    res = {k: out[i] for i, k in enumerate(METRIC_KEYS)}
    for k in ["meanAUC", "medianAUC", "varAUC", "allAUC", "meanAUPR", "medianAUPR", "varAUPR",
              "allAUPR", "meanFDR", "medianFDR", "varFDR", "allFDR"]:
        res[k] = 0
    return res
