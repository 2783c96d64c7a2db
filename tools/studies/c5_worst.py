"""Where the f16x3 gradient error of the full C5 problem comes from (VERDICT r04
item 2): BASELINE configs[4] (B 512, n_sample 8192, L = z = 4096) on one GPU,
one seed, philox noise, total_loss as the objective.

Decomposes the kernels' error against the fp64-t restatement
(tests/torch64_ref.py) into
  * t: the kernels' own t (their T stash) against the fp64 product of the same
    fp32 operands, beside an fp32 GEMM's t (the reference's tensordot);
  * conditioning: the reference's formulas evaluated on the kernels' t
    (ChunkedElbo(t_src=...)) against the fp64-t values -- what the
    reference's own arithmetic gives from this t;
  * the kernels' arithmetic after t: kernels against that restatement;
and records the worst elements of d fe_out / d fx_out with the sample terms
that dominate them (t under each arithmetic, E and 1 - E in fp32).

  python tools/studies/c5_worst.py --seed 11 [--config c5|c4] > out.json
  python tools/studies/c5_worst.py --c4test 3 > out.json   (the inputs of
      tests/test_gpu_parity.py::test_c4_full_size_against_fp64_reference, explicit
      noise; adds the forward row statistics of the worst rows: the kernels'
      rowstat against the reference's formulas on the kernels' own t)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mpvae-1_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpvae  # noqa: E402
from mpvae_ops import HipShardBackend  # noqa: E402
from tolerances import rel_err  # noqa: E402
from torch64_ref import F32, F64, ChunkedElbo, INV_SQRT_2PI, probit_prob, _C1  # noqa: E402

DEV = "cuda:0"
CFG = {"c5": (512, 8192, 4096, 4096, 50), "c4": (512, 4096, 1024, 1024, 50)}


def inputs(cfg, seed):
    B, S, L, z, d = CFG[cfg]
    g = torch.Generator(device=DEV).manual_seed(seed)
    y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
    y[:, 0], y[:, 1] = 1, 0
    fe = torch.randn((B, L), device=DEV, generator=g)
    fx = torch.randn((B, L), device=DEV, generator=g)
    mus = [torch.randn((B, d), device=DEV, generator=g) for _ in range(4)]
    R = ((torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1)
         * (6.0 / (L + z)) ** 0.5)
    return (B, S, L, z, d), y, fe, fx, mus, R


def c4test_inputs(seed):
    """tests/test_gpu_parity.py::test_c4_full_size_against_fp64_reference's inputs."""
    B, S, L, z, d = 512, 4096, 1024, 1024, 50
    g = torch.Generator(device=DEV).manual_seed(1000 + seed)
    y = (torch.rand((B, L), device=DEV, generator=g) < 0.15).float()
    y[:, 0], y[:, 1] = 1, 0
    fe = torch.randn((B, L), device=DEV, generator=g)
    fx = torch.randn((B, L), device=DEV, generator=g)
    mus = [torch.randn((B, d), device=DEV, generator=g) * s for s in (1.0, 0.1, 1.0, 0.1)]
    R = (torch.rand((L, z), device=DEV, generator=g, dtype=torch.float64) * 2 - 1) * \
        (6.0 / (L + z)) ** 0.5
    noise = torch.randn((S, B, z), device=DEV, generator=g)
    return (B, S, L, z, d), y, fe, fx, mus, R, noise


def plane_noise(pl, B, S, z):
    rows = pl.data[:B * S].view(B, S, pl.ld)
    cols = pl.cols

    def noise(a, b):
        v = rows[:, a:b].contiguous().view(torch.float16).float().view(B, b - a, cols // 32, 2, 32)
        e = (v[:, :, :, 0, :] + v[:, :, :, 1, :]).reshape(B, b - a, cols)[:, :, :z] / pl.scale
        return e.permute(1, 0, 2).contiguous()
    return noise


def per_sample_terms(ce, br, b, l, t_col):
    """gu[s] of element (b, l) of branch br (0: label / d fe_out, 1: feature)
    from the restatement's row statistics, for a given t column t_col (S,)."""
    base = (ce.fe if br == 0 else ce.fx)[b, l]
    u32 = (t_col.to(F32) + base)
    E = probit_prob(u32, ce.erf_fp64).to(F64)
    S = ce.S
    B = ce.y.shape[0]
    w = torch.exp(ce.rowstat[br, b] - ce.m[br, b]) / ce.Z[br, b]
    a = -0.1 * w / B
    scale = 200.0 / (ce.n[b] * S * B)
    yv = float(ce.y[b, l])
    gE = a * (yv / E - (1.0 - yv) / (1.0 - E))
    if yv == 1.0:
        gE = gE - scale * ce.rowstat[3 + 2 * br, b] * torch.exp(-5.0 * E)
    elif yv == 0.0:
        gE = gE + scale * ce.rowstat[2 + 2 * br, b] * torch.exp(5.0 * E)
    u = u32.to(F64)
    return gE * float(_C1) * INV_SQRT_2PI * torch.exp(-0.5 * u * u), E


def flip_scan(y, base, t_row, d_obs, top=4):
    """One sample row (b, s) of one branch: which labels' log q would move by
    the observed logp difference d_obs if fl(erf(x)) -- the reference's first
    rounding of E (x = u / sqrt 2 in fp32) -- were its fp32 neighbour instead,
    and how close erf(x) lies to the midpoint between the two (|pos| = 0.5: a
    tie; pos = erf(x) in fp64 minus torch's fp32 erf, in fp32 ulps of erf)."""
    sq2 = torch.tensor(2.0 ** 0.5, dtype=F32, device=t_row.device)
    u32 = t_row.to(F32) + base.to(F32)
    x = u32 / sq2
    e32 = torch.erf(x)
    e64 = torch.erf(x.to(F64))
    up = torch.nextafter(e32, torch.full_like(e32, 2.0))
    dn = torch.nextafter(e32, torch.full_like(e32, -2.0))
    yv = y.to(F64)

    def logq(ev):
        E = ((0.5 * (1.0 + ev)) * _C1.to(ev.device) + float(0.5e-6)).to(F64)
        return yv * torch.log(E) + (1.0 - yv) * torch.log(1.0 - E)
    l0 = logq(e32)
    d_up, d_dn = logq(up) - l0, logq(dn) - l0
    pos = (e64 - e32.to(F64)) / (up.to(F64) - e32.to(F64))
    # the neighbour that reproduces d_obs best
    d_best = torch.where((d_up - d_obs).abs() < (d_dn - d_obs).abs(), d_up, d_dn)
    order = torch.topk(-(d_best - d_obs).abs(), top).indices.tolist()
    return [{"l": l, "y": float(y[l]), "u": float(u32[l]), "E_ref": float(torch.exp(l0[l])) if y[l] == 1
             else 1.0 - float(torch.exp(l0[l])), "dlogq_flip": float(d_best[l]),
             "pos_ulps": float(pos[l])} for l in order]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--config", default="c5", choices=sorted(CFG))
    ap.add_argument("--top", type=int, default=3)
    ap.add_argument("--c4test", type=int, default=None)
    cli = ap.parse_args()
    explicit = None
    if cli.c4test is not None:
        (B, S, L, z, d), y, fe, fx, mus, R, explicit = c4test_inputs(cli.c4test)
        cli.config, cli.seed = "c4", cli.c4test
    else:
        (B, S, L, z, d), y, fe, fx, mus, R = inputs(cli.config, cli.seed)
    key = 55490 + cli.seed
    chunk = 64 if cli.config == "c5" else 256
    leaves = [x.clone().requires_grad_(True) for x in (fe, mus[0], mus[1], fx, mus[2], mus[3], R)]
    args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S,
                              mode="train", nll_coeff=0.1, c_coeff=200.0,
                              mpvae_noise="philox" if explicit is None else explicit,
                              mpvae_seed=key)
    out = mpvae.compute_loss(y, *leaves, args)
    out[0].backward()
    got = {"fe_out": leaves[0].grad.detach().double(), "fx_out": leaves[3].grad.detach().double(),
           "r_sqrt_sigma": leaves[6].grad.detach().double()}
    del out, leaves, args
    torch.cuda.empty_cache()
    be = HipShardBackend("f16x3")
    shape = be.shape(S, S, 0, B, L, z)
    if explicit is None:
        pl = be.make_noise(shape, DEV, key, 0)
        noise = plane_noise(pl, B, S, z)
    else:
        pl = be.prepare_noise(explicit, shape)
        noise = lambda a, b: explicit[a:b]
    # the kernels' own t (the forward's T stash, (B, S, L) b-major) and row statistics
    loc = be.forward_local(shape, y, fe, fx, be.prepare_R(R), pl, keep_T=True)
    T = loc["T"]
    k_rowstat, k_bstat = loc["rowstat"].double(), loc["bstat"].double()
    del loc
    t_kern = lambda a, b: T[:, a:b, :L].permute(1, 0, 2)
    res = {"config": cli.config, "seed": cli.seed, "B": B, "S": S, "L": L, "z": z}
    # t accuracy over the first 256 samples: kernels and an fp32 GEMM against
    # the fp64 product of the same fp32 operands
    ref64 = ChunkedElbo(y, fe, fx, R, noise, S, chunk=chunk)
    ref32 = ChunkedElbo(y, fe, fx, R, noise, S, chunk=chunk, t_fp32=True)
    t64, _ = ref64._t(0, 256)
    t32, _ = ref32._t(0, 256)
    tk = t_kern(0, 256)
    e64 = lambda t: (t.double() - t64.double()).abs()
    scale = float(t64.abs().max())
    res["t_err"] = {"kernels_max": float(e64(tk).max()) / scale,
                    "fp32_gemm_max": float(e64(t32).max()) / scale,
                    "kernels_mean": float(e64(tk).mean()) / scale,
                    "fp32_gemm_mean": float(e64(t32).mean()) / scale,
                    "kernels_bias": float((tk.double() - t64.double()).mean()) / scale,
                    "note": "normwise over samples [0, 256): |t - t_fp64| / max|t_fp64|"}
    del t64, t32, tk
    rf = ref64.forward(*mus, 0.1, 200.0)
    rg = ref64.backward(0.1, 200.0, 1.0, None, None)
    ref32.forward(*mus, 0.1, 200.0)
    rg32 = ref32.backward(0.1, 200.0, 1.0, None, None)
    del ref32
    refk = ChunkedElbo(y, fe, fx, R, noise, S, chunk=chunk, t_src=t_kern)
    refk.forward(*mus, 0.1, 200.0)
    rgk = refk.backward(0.1, 200.0, 1.0, None, None)
    # the forward's row statistics (logp, P, N per branch) and per-row
    # log-sum-exp terms: kernels against the reference on the same t
    rs_diff = (k_rowstat - refk.rowstat).abs()
    res["rowstat_max_abs_diff"] = {n: float(rs_diff[k].max()) for k, n in enumerate(
        ("logp_e", "logp_x", "P_e", "N_e", "P_x", "N_x"))}
    res["bstat_rel_diff"] = {n: float(((k_bstat[k] - (refk.m if k in (0, 2) else refk.Z)[k // 2]) /
                                       (refk.m if k in (0, 2) else refk.Z)[k // 2]).abs().max())
                             for k, n in ((0, "m_e"), (1, "Z_e"), (2, "m_x"), (3, "Z_x"))}
    refk_rowstat, refk_m, refk_Z = refk.rowstat, refk.m, refk.Z
    del refk
    np_ = lambda t: t.detach().cpu().numpy()
    res["grad_err"] = {}
    for k in got:
        res["grad_err"][k] = {
            "kernels_vs_fp64t": rel_err(np_(got[k]), np_(rg[k])),
            "ref_fp32_vs_fp64t": rel_err(np_(rg32[k]), np_(rg[k])),
            "ref_on_kernel_t_vs_fp64t": rel_err(np_(rgk[k]), np_(rg[k])),
            "kernels_vs_ref_on_kernel_t": rel_err(np_(got[k]), np_(rgk[k]))}
    # worst elements of d fe_out / d fx_out, with their dominant sample terms
    res["worst"] = []
    Rt = R.to(F32).to(F64).t()
    for br, k in ((0, "fe_out"), (1, "fx_out")):
        diff = (got[k] - rg[k]).abs()
        scale_k = float(rg[k].abs().max())
        flat = torch.topk(diff.reshape(-1), cli.top).indices
        for idx in flat.tolist():
            b, l = divmod(idx, L)
            # t of column (b, l) over all samples: fp64, fp32 GEMM, kernels
            eps_b = torch.cat([noise(a, min(S, a + 1024))[:, b, :] for a in range(0, S, 1024)])
            t64c = (eps_b.double() @ Rt[:, l]).to(F32)
            t32c = eps_b.to(F32) @ Rt[:, l].to(F32)
            tkc = T[b, :, l]
            g64, E64 = per_sample_terms(ref64, br, b, l, t64c)
            gk, Ek = per_sample_terms(ref64, br, b, l, tkc)
            g32, E32 = per_sample_terms(ref64, br, b, l, t32c)
            dom = torch.topk((gk - g64).abs(), 3).indices.tolist()
            # this row's softmax weights over s: kernels' statistics vs the
            # reference's on the kernels' t (the forward's share of the error)
            lp_k = k_rowstat[br, b]
            w_k = torch.exp(lp_k - lp_k.max()) / torch.exp(lp_k - lp_k.max()).sum()
            lp_r = refk_rowstat[br, b]
            w_r = torch.exp(lp_r - refk_m[br, b]) / refk_Z[br, b]
            top = torch.topk(w_r, 3).indices.tolist()
            base_row = (fe if br == 0 else fx)[b, :L]
            res.setdefault("rows", []).append({
                "grad": "d" + k, "b": b, "max_abs_logp_diff": float((lp_k - lp_r).abs().max()),
                "top_samples": [{"s": s_, "w_ref_on_kernel_t": float(w_r[s_]), "w_kernels": float(w_k[s_]),
                                 "logp_ref_on_kernel_t": float(lp_r[s_]), "logp_kernels": float(lp_k[s_]),
                                 "flip_candidates": flip_scan(y[b, :L], base_row, T[b, s_, :L],
                                                              float(lp_k[s_] - lp_r[s_]))}
                                for s_ in top]})
            res["worst"].append({
                "grad": "d" + k, "b": b, "l": l, "y": float(y[b, l]),
                "rel_to_max": float(diff[b, l]) / scale_k,
                "got": float(got[k][b, l]), "ref_fp64t": float(rg[k][b, l]),
                "ref_fp32": float(rg32[k][b, l]), "ref_on_kernel_t": float(rgk[k][b, l]),
                "terms": [{"s": s, "t_fp64": float(t64c[s]), "t_kernels": float(tkc[s]),
                           "t_fp32_gemm": float(t32c[s]), "E_fp64t": float(E64[s]),
                           "one_minus_E_fp64t": float(1.0 - E64[s]),
                           "one_minus_E_kernel_t": float(1.0 - Ek[s]),
                           "one_minus_E_fp32_t": float(1.0 - E32[s]),
                           "gu_fp64t": float(g64[s]), "gu_kernel_t": float(gk[s]),
                           "gu_fp32_t": float(g32[s])} for s in dom]})
            del eps_b
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
