"""CPU: the fairness / metrics oracle (oracle/fairness.py) against the golden
vectors recorded from the reference's own code, and the host side of the
device label-pattern table (mpvae_fair.py)."""
import numpy as np
import pytest

from fair_io import fair_fixtures, metric_fixtures
from oracle import fairness as of

FAIR = fair_fixtures()
MET = metric_fixtures()


@pytest.mark.parametrize("f", FAIR, ids=[f["name"] for f in FAIR])
def test_fair_oracle_matches_reference(f):
    loss, contributed, gl, gf = of.fair_penalty(f["label_z"], f["feat_z"], f["labels"],
                                                f["sensitive"], f["dists"], f["norm"], f["coeff"])
    assert contributed == int(f["contributed"])
    if not int(f["active"]):
        assert loss is None
        return
    # Python-float distances: the reference computes in fp32 (fair_f6/f7), the
    # oracle in fp64 -- they differ by fp32 rounding (measured: loss 8e-9, grads 2.5e-7)
    ltol, gtol = (1e-7, 1e-6) if f["pyfloat"] else (1e-12, 1e-6)
    assert str(f["ref_dtype"]) == ("float32" if f["pyfloat"] else "float64")
    assert abs(loss - float(f["fairloss"])) <= ltol * abs(float(f["fairloss"]))
    for g, ref in ((gl, f["g_label_z"]), (gf, f["g_feat_z"])):
        assert np.abs(g - ref).max() <= gtol * np.abs(ref).max()


@pytest.mark.parametrize("m", MET, ids=[m["name"] for m in MET])
def test_metrics_oracle_matches_reference(m):
    v = of.train_metrics(m["pred"], m["target"], 0.5)
    assert np.allclose(v, m["values"], rtol=1e-6, atol=1e-7), (v, m["values"])


def test_pattern_table_reference_dtype():
    """torch.tensor(weights) in the reference is float64 iff the dict values are
    numpy float64; the table records which (mpvae_fair.fairness_penalty casts
    the loss to it)."""
    import torch
    import mpvae_fair as mf
    k = "0110"
    assert mf.LabelDistanceTable({k: 1.0}, 4, "cpu").ref_dtype == torch.float32
    assert mf.LabelDistanceTable({k: 2 / 3}, 4, "cpu").ref_dtype == torch.float32
    assert mf.LabelDistanceTable({k: np.float64(0.5)}, 4, "cpu").ref_dtype == torch.float64
    assert torch.tensor([np.float64(0.5), 0.]).dtype == torch.float64
    assert torch.tensor([1.0, 0.]).dtype == torch.float32


def test_pattern_table_host_build():
    import torch
    import mpvae_fair as mf
    rng = np.random.default_rng(0)
    L = 130
    keys = {"".join(rng.integers(0, 2, L).astype(str)): float(i + 1) for i in range(50)}
    keys["2" + "0" * (L - 1)] = 9.0          # not a 0/1 pattern: never matchable
    tab = mf.LabelDistanceTable(keys, L, "cpu")
    assert tab.nslots == 128 and tab.W == 3
    kk = tab.keys.numpy().view(np.uint64)
    used, vals = tab.used.numpy(), tab.vals.numpy()
    for k, v in keys.items():
        words = mf.pack_pattern(k, L)
        if words is None:
            continue
        slot = mf.pattern_hash(words) & (tab.nslots - 1)
        while used[slot] and list(kk[slot]) != words:
            slot = (slot + 1) & (tab.nslots - 1)
        assert used[slot] and vals[slot] == v
    assert int(used.sum()) == 50
