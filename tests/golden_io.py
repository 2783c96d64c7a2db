"""Load the golden fixtures of tests/golden (made by tests/golden/make_golden.py)."""
import argparse
import glob
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
OUTS = ["total", "nll", "nll_x", "c", "c_x", "kl", "indiv_prob", "indiv_prob_label"]
INPUTS = ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar", "r_sqrt_sigma"]
DIFF = ["fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar"]
PART_KEYS = ["g_nll", "g_nll_x", "g_c", "g_c_x", "g_kl"]


class Fixture:
    def __init__(self, path):
        z = np.load(path)
        self.name = os.path.basename(path)[5:-4]
        self.data = {k: z[k] for k in z.files}
        self.L, self.z, self.B, self.S, self.d = (int(v) for v in self.data["meta"])
        self.mode = str(self.data["mode"])
        self.nll_coeff, self.c_coeff = (float(v) for v in self.data["coeffs"])
        self.r_kind = str(self.data["r_kind"])
        self.extreme = "extreme" in self.name

    def __getitem__(self, k):
        return self.data[k]

    def args(self, **extra):
        a = argparse.Namespace(label_dim=self.L, z_dim=self.z, n_train_sample=self.S,
                               n_test_sample=self.S, mode=self.mode, nll_coeff=self.nll_coeff,
                               c_coeff=self.c_coeff)
        for k, v in extra.items():
            setattr(a, k, v)
        return a

    def outputs(self):
        return {k: self.data["out_" + k] for k in OUTS}

    def grads(self, kind):
        pre = kind + "_"
        return {k[len(pre):]: v for k, v in self.data.items() if k.startswith(pre)}

    @property
    def trainable_r(self):
        return self.r_kind == "train64"


def fixtures():
    return [Fixture(p) for p in sorted(glob.glob(os.path.join(GOLDEN, "elbo_*.npz")))]


def fixture_ids():
    return [f.name for f in fixtures()]
