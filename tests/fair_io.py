"""Load the fairness / metrics golden fixtures (tests/golden/make_golden_fair.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fair_fixtures():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "fair_*.npz"))):
        z = np.load(p)
        d = {k: z[k] for k in z.files}
        d["name"] = os.path.basename(p)[5:-4]
        d["dists"] = json.loads(str(d["dists"]))
        # the value types decide the reference's weights dtype (make_golden_fair.py):
        # np.float64 -> float64, Python float -> float32
        d["pyfloat"] = bool(int(d["pyfloat"])) if "pyfloat" in d else False
        if not d["pyfloat"]:
            d["dists"] = [{k: np.float64(v) for k, v in t.items()} for t in d["dists"]]
        d["norm"] = str(d["norm"])
        d["coeff"] = float(d["coeff"])
        out.append(d)
    return out


def metric_fixtures():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "metrics_*.npz"))):
        z = np.load(p)
        d = {k: z[k] for k in z.files}
        d["name"] = os.path.basename(p)[8:-4]
        out.append(d)
    return out
