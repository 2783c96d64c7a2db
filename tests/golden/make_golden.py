"""Generate the golden vectors for the probit-ELBO hot path.

Runs ONLY in the build container, where the reference checkout is mounted at
/root/reference (it never travels to the GPU box).  It imports the reference's
own ``mpvae.py`` (by file path, under the private module name ``_ref_mpvae``)
and records, on small synthetic inputs:

  * ``compute_loss`` (reference mpvae.py:145-210) -- all 8 outputs, and the
    gradients of two scalar objectives w.r.t. every differentiable input:
      obj_total = total + <g_I, indiv_prob> + <g_IL, indiv_prob_label>
      obj_parts = a . (nll, nll_x, c, c_x, kl)       (random weights a)
    ``obj_parts`` pins each loss component's gradient separately; the NaN
    pattern of degenerate label rows (mpvae.py:117-121 + autograd) is kept.
  * ``VAE`` (reference mpvae.py:10-100) -- the state_dict layout (names,
    shapes, dtypes) with per-tensor fingerprints of the seeded init, and the
    eval-mode forward outputs on CPU together with the reparameterisation
    noise the reference draws (label eps first, then feat eps).

The noise of compute_loss is drawn by the reference itself from torch's CPU
default generator (mpvae.py:162).  We seed that generator, draw
``torch.normal(0, 1, size=(S, B, z))`` to record the exact noise tensor, then
re-seed and call ``compute_loss``: the reference's internal draw is the same
tensor bit for bit (checked below by re-running with the recorded noise
monkey-patched in).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
Writes: tests/golden/elbo_*.npz, tests/golden/vae_small.npz
"""
import argparse
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/mpvae.py"


def load_reference():
    spec = importlib.util.spec_from_file_location("_ref_mpvae", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# name, L, z, B, S, d, mode, nll_coeff, c_coeff, r_kind, label_kind, logit_scale, seed
CASES = [
    ("f1_l38", 38, 38, 8, 16, 50, "train", 0.5, 10.0, "train64", "normal", 1.0, 11),
    ("f2_degenerate", 38, 38, 8, 16, 50, "train", 0.5, 10.0, "train64", "degenerate", 1.0, 12),
    ("f3_adult_like", 25, 10, 16, 12, 8, "train", 0.1, 200.0, "train64", "normal", 1.0, 13),
    ("f4_extreme", 38, 38, 6, 8, 50, "train", 0.5, 10.0, "train64", "normal", 6.0, 14),
    ("f5_testmode", 38, 38, 8, 24, 50, "test", 0.5, 10.0, "train64", "normal", 1.0, 15),
    ("f6_l81", 81, 81, 4, 8, 50, "train", 0.1, 200.0, "train64", "normal", 1.0, 16),
    ("f7_l256", 256, 96, 2, 4, 50, "train", 0.1, 200.0, "train64", "normal", 1.0, 17),
    ("f8_rzero", 38, 38, 8, 16, 50, "train", 0.5, 10.0, "zero32", "normal", 1.0, 18),
    ("f9_rrandom", 38, 38, 8, 16, 50, "train", 0.5, 10.0, "nograd64", "normal", 1.0, 19),
    ("f10_softlabels", 20, 12, 8, 16, 8, "train", 0.5, 10.0, "train64", "soft", 1.0, 20),
]


def make_inputs(L, z, B, d, r_kind, label_kind, logit_scale, rng):
    if label_kind == "soft":
        # non-binary labels: they take part in the BCE term but count as
        # neither positive nor negative in the ranking term (mpvae.py:107-108)
        y = rng.choice([0.0, 1.0, 0.5, 0.25], size=(B, L), p=[0.5, 0.3, 0.1, 0.1])
        y[:, 0], y[:, 1] = 1.0, 0.0
    else:
        y = (rng.random((B, L)) < 0.3).astype(np.float64)
        y[:, 0], y[:, 1] = 1.0, 0.0
        if label_kind == "degenerate":
            y[1, :] = 0.0          # no positives  -> normaliser 0
            y[4, :] = 1.0          # no negatives  -> normaliser 0
    fe = rng.standard_normal((B, L)) * logit_scale
    fx = rng.standard_normal((B, L)) * logit_scale
    mu_e, mu_x = rng.standard_normal((B, d)), rng.standard_normal((B, d))
    lv_e, lv_x = 0.3 * rng.standard_normal((B, d)), 0.3 * rng.standard_normal((B, d))
    bound = np.sqrt(6.0 / (L + z))
    if r_kind == "zero32":
        R = np.zeros((L, z), np.float32)
    else:
        R = rng.uniform(-bound, bound, (L, z))          # float64, as mpvae.py:41/47
    f32 = lambda a: np.ascontiguousarray(a, np.float32)
    return dict(y=f32(y), fe_out=f32(fe), fx_out=f32(fx), fe_mu=f32(mu_e), fe_logvar=f32(lv_e),
                fx_mu=f32(mu_x), fx_logvar=f32(lv_x), r_sqrt_sigma=R)


DIFF = ["fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar"]
OUTS = ["total", "nll", "nll_x", "c", "c_x", "kl", "indiv_prob", "indiv_prob_label"]


def run_case(ref, case):
    name, L, z, B, S, d, mode, nllc, cc, r_kind, label_kind, scale, seed = case
    rng = np.random.default_rng(seed)
    inp = make_inputs(L, z, B, d, r_kind, label_kind, scale, rng)
    args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S,
                              mode=mode, nll_coeff=nllc, c_coeff=cc)
    torch.manual_seed(1000 + seed)
    noise = torch.normal(0, 1, size=(S, B, z))
    g_I = rng.standard_normal((B, L)).astype(np.float32)
    g_IL = rng.standard_normal((B, L)).astype(np.float32)
    a_parts = rng.uniform(0.5, 2.0, 5)

    def call(obj_kind):
        t = {k: torch.from_numpy(v.copy()) for k, v in inp.items()}
        grad_names = []
        if mode == "train":
            for k in DIFF:
                t[k].requires_grad_(True)
                grad_names.append(k)
            if r_kind == "train64":
                t["r_sqrt_sigma"].requires_grad_(True)
                grad_names.append("r_sqrt_sigma")
        torch.manual_seed(1000 + seed)
        out = ref.compute_loss(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"], t["fx_out"],
                               t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"], args)
        grads = {}
        if mode == "train":
            if obj_kind == "total":
                obj = out[0] + (out[6] * torch.from_numpy(g_I)).sum() + \
                    (out[7] * torch.from_numpy(g_IL)).sum()
            else:
                obj = sum(float(a) * o for a, o in zip(a_parts, out[1:6]))
            obj.backward()
            grads = {k: t[k].grad.detach().numpy().copy() for k in grad_names}
        return [o.detach().numpy().copy() for o in out], grads

    outs, grads_total = call("total")
    _, grads_parts = call("parts")

    # check: the reference's internal draw is exactly `noise`
    orig_normal = torch.normal
    torch.normal = lambda *a, **k: noise.clone()
    try:
        t = {k: torch.from_numpy(v.copy()) for k, v in inp.items()}
        chk = ref.compute_loss(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"], t["fx_out"],
                               t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"], args)
    finally:
        torch.normal = orig_normal
    for a, b in zip(chk, outs):
        assert np.array_equal(a.detach().numpy(), b, equal_nan=True), name

    rec = dict(inp)
    rec["noise"] = noise.numpy()
    rec["g_I"], rec["g_IL"], rec["a_parts"] = g_I, g_IL, a_parts
    rec["meta"] = np.array([L, z, B, S, d], np.int64)
    rec["mode"] = np.array(mode)
    rec["coeffs"] = np.array([nllc, cc], np.float64)
    rec["r_kind"] = np.array(r_kind)
    for k, v in zip(OUTS, outs):
        rec["out_" + k] = v
    for k, v in grads_total.items():
        rec["gtot_" + k] = v
    for k, v in grads_parts.items():
        rec["gpart_" + k] = v
    path = os.path.join(HERE, f"elbo_{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: total={outs[0]:.6f} nan_grads="
          f"{sum(int(np.isnan(v).any()) for v in grads_total.values())} -> {path}")


def run_vae(ref):
    args = argparse.Namespace(feature_dim=20, latent_dim=8, label_dim=6, z_dim=4, keep_prob=0.5,
                              scale_coeff=1.0, residue_sigma="")
    torch.manual_seed(0)
    np.random.seed(0)
    model = ref.VAE(args)
    sd = model.state_dict()
    rng = np.random.default_rng(5)
    label = (rng.random((5, 6)) < 0.4).astype(np.float32)
    feat = rng.standard_normal((5, 20)).astype(np.float32)
    rec = {"label": label, "feat": feat}
    # the weights themselves are reproduced from the seeds (construction order
    # and init draws are part of the contract); store only fingerprints
    rec["sd_names"] = np.array(list(sd.keys()))
    rec["sd_shapes"] = np.array([list(v.shape) + [0] * (2 - v.dim()) for v in sd.values()])
    rec["sd_dtypes"] = np.array([str(v.dtype) for v in sd.values()])
    rec["sd_sums"] = np.array([v.double().sum().item() for v in sd.values()])
    rec["sd_sumsq"] = np.array([(v.double() ** 2).sum().item() for v in sd.values()])
    rec["sd_head"] = np.stack([v.reshape(-1)[:4].double().numpy() for v in sd.values()])
    # eval mode: the only RNG draws are label eps then feat eps (mpvae.py:68,73)
    model.eval()
    torch.manual_seed(1)
    eps_label = torch.randn(5, 8)
    eps_feat = torch.randn(5, 8)
    torch.manual_seed(1)
    with torch.no_grad():
        out = model(torch.from_numpy(label), torch.from_numpy(feat))
    for k, v in zip(["label_out", "label_mu", "label_logvar", "feat_out", "feat_mu",
                     "feat_logvar"], out):
        rec["eval_" + k] = v.numpy()
    rec["eps_label"], rec["eps_feat"] = eps_label.numpy(), eps_feat.numpy()
    path = os.path.join(HERE, "vae_small.npz")
    np.savez_compressed(path, **rec)
    print(f"vae: {len(sd)} state_dict keys -> {path}")


def main():
    ref = load_reference()
    torch.set_num_threads(1)
    for case in CASES:
        run_case(ref, case)
    run_vae(ref)


if __name__ == "__main__":
    main()
