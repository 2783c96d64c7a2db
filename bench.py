"""Benchmark of the MPVAE probit-ELBO hot path on MI355X.

One step = one ``compute_loss`` forward + backward (reference mpvae.py:145-210
and its autograd) over one synthetic batch, with the probit noise generated on
the device (philox mode), inputs resident in HBM.  Metric (BASELINE.json):
probit MC label-samples/s = n_sample x B x L per step, whole job.

Default workload (north star): C4 -- B=512, n_sample=4096, L=z=1024.  With
--gpus N the n_sample axis of that one estimate is split over the N ranks
(strong scaling, the default: 4096/N samples per GPU, the north star's "scaling
at 8 GPUs" of the (512, 4096, 1024) problem), exchanging only the exact
log-sum-exp statistics and gradient sums (mpvae_dist.py).  --scaling weak
gives every rank its own 4096 samples of an n_sample = 4096*N estimate.
--n-sample overrides the config's n_sample (e.g. 512: one rank's share at N=8,
timed on one GPU with MPVAE_FORCE_DIST=1 to see the fixed costs).

    python bench.py [--gpus N --steps K --warmup W --config c4|c2|c3|c5 --scaling strong|weak]
    torchrun --nproc-per-node N bench.py --gpus N ...

``python bench.py --gpus N`` (N > 1, no WORLD_SIZE in the environment) starts
its own N rank processes (mpvae_launch.py) before any GPU call and prints rank
0's line.  MPVAE_DIST_BACKEND=gloo runs the exchange over gloo instead of RCCL
and maps ranks onto the visible GPUs round robin: a rehearsal of the N-rank
path on a one-GPU box (tests/test_gpu_dist.py), not a scaling measurement.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpvae-1_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mpvae  # noqa: E402
import mpvae_dist  # noqa: E402
import mpvae_hip as H  # noqa: E402
import mpvae_launch  # noqa: E402

METRIC = "probit MC label-samples/sec (B×n_sample×L) at 1/2/4/8 GPU; ELBO rel-err"
FP32_MFMA_PEAK = 157.3e12   # MI355X_MICROARCH.md: dense f32-input MFMA (= f32 vector peak)
F16_MFMA_PEAK = 2.5e15      # MI355X_MICROARCH.md: dense BF16/F16 MFMA
# The f16x3 GEMMs evaluate one fp32-accurate multiply-add as three f16 MFMA
# products (hi*hi + hi*lo + lo*hi), so their fp32-equivalent ceiling is a third
# of the dense f16 peak.
PEAKS = {"f16x3": (F16_MFMA_PEAK / 3.0, "f16x3 MFMA: dense f16 peak / 3"),
         "f32": (FP32_MFMA_PEAK, "f32 MFMA")}
HBM_PEAK = 8.0e12           # MI355X_MICROARCH.md: HBM3E spec
# VALU ceiling (MI355X_MICROARCH.md: 157.3 TFLOPS fp32 vector = 256 CUs x 4
# SIMD-32 x 32 lanes x 2.4 GHz x 2 flop per FMA): one lane-instruction per lane
# per cycle, 78.6e12 lane-instructions/s.  A packed fp32 op (v_pk_*) counts as
# one lane-instruction, like the counter (SQ_INSTS_VALU) it is measured with.
VALU_PEAK = FP32_MFMA_PEAK / 2.0

# name: (L, z, B, n_sample (total under strong scaling, per GPU under weak), d,
#        nll_coeff, c_coeff)
CONFIGS = {
    "c2": (38, 38, 128, 1000, 50, 0.5, 10.0),
    "c3": (81, 81, 256, 2000, 50, 0.1, 200.0),
    "c4": (1024, 1024, 512, 4096, 50, 0.1, 200.0),
    "c5": (4096, 4096, 512, 8192, 50, 0.1, 200.0),
}
# default (timed steps, warm-up steps) per config: 200 steps keep the C2-C4
# runs several seconds of GPU work; C5 (~0.7 s per step on one GPU) takes 10
DEFAULT_STEPS = {"c2": (200, 5), "c3": (200, 5), "c4": (200, 5), "c5": (10, 2)}
# the probit kernels of the small configurations (L, z <= 128) are VALU-bound
# (SURVEY.md section 8(d)): their roofline is the VALU ceiling
SMALL_LZ = 128
# The algorithmic VALU floor of the two element-wise kernels, in lane-
# instructions per label-sample (both branches; a packed fp32 op serving two
# elements counts 1/2 per element), counted from the formulation the kernels
# evaluate (csrc/mpv_common.h probit_w2xN_zq / probit_dw2xN_zq and their
# callers), so that frac_algorithmic prices algorithmic work, not whatever a
# kernel executes:
#   forward, per element and branch: argument 0.5, t = rcp(fma) 2, degree-6 P
#   3, exponent 0.5, exp 1, erfc 0.5, 1 - erfc 0.5, copysign 1, w 0.5, E in
#   the reference's order 1, BCE operand 0.5, ranking exponent 0.5, exp 1, the
#   log of a 4-label product 0.625, row sum 0.125, P / N sums 1, column sum
#   0.5 = 14.75; x 2 branches = 29.5 (C4 executes 43.6);
#   element pass, per element and branch: argument 0.5, t 2, degree-6 Q 3,
#   -z^2 0.5, exp 1, erfc 1.5, copysign 1, w 0.5, E 1, d 0.5, rcp 1, dE 0.5,
#   ranking select 1, exponent 0.5, exp 1, fma 0.5, x exp(-z^2) 0.5 = 16.5,
#   plus the column sum, G = dE + dE_x and its 3xf16 split 3.5 = 20; x 2 = 40
#   (C4 executes 42.5).
VALU_FLOOR_PER_LS = {"probit_fwd": 29.5, "bwd_elem": 40.0}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_dist():
    """(world, rank, cuda device index) from the launcher's environment."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MPVAE_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if backend == "gloo":
        local = local % max(1, n_dev)   # rehearsal: several ranks may share a GPU
    elif local >= n_dev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {n_dev} GPUs visible")
    torch.cuda.set_device(local)
    # MPVAE_FORCE_DIST=1: a process group (and the sample-shard exchange) even
    # on one rank -- rehearses the RCCL path on a single-GPU box
    if world > 1 or os.environ.get("MPVAE_FORCE_DIST") == "1":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def make_inputs(L, z, B, d, device, seed=1234):
    g = torch.Generator(device=device).manual_seed(seed)
    y = (torch.rand((B, L), device=device, generator=g) < 0.15).float()
    y[:, 0], y[:, 1] = 1.0, 0.0      # no degenerate rows
    leaves = dict(
        fe_out=torch.randn((B, L), device=device, generator=g),
        fe_mu=torch.randn((B, d), device=device, generator=g),
        fe_logvar=0.1 * torch.randn((B, d), device=device, generator=g),
        fx_out=torch.randn((B, L), device=device, generator=g),
        fx_mu=torch.randn((B, d), device=device, generator=g),
        fx_logvar=0.1 * torch.randn((B, d), device=device, generator=g),
        r_sqrt_sigma=(torch.rand((L, z), device=device, generator=g, dtype=torch.float64) * 2 - 1)
        * (6.0 / (L + z)) ** 0.5,
    )
    for v in leaves.values():
        v.requires_grad_(True)
    return y, leaves


ORDER = ["fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar", "r_sqrt_sigma"]


def step(y, leaves, args, it):
    for v in leaves.values():
        v.grad = None
    args.mpvae_seed = 0x5EED0000 + it
    if args.mode != "train":  # evaluation: forward only, no autograd state
        with torch.no_grad():
            return mpvae.compute_loss(y, *[leaves[k] for k in ORDER], args)
    out = mpvae.compute_loss(y, *[leaves[k] for k in ORDER], args)
    out[0].backward()
    return out


def graph_steps(y, leaves, args, warmup, steps):
    """Capture one fwd+bwd step in a HIP graph and time `steps` replays.  The
    Philox key is a device tensor that the step's own finalize launch advances
    after the noise has read it (args.mpvae_seed_advance), so every replay
    draws fresh noise (tests/test_gpu_parity.py checks replays against eager)."""
    seed = torch.tensor([0x5EED0000], dtype=torch.int64, device=y.device)
    args.mpvae_seed = seed
    args.mpvae_seed_advance = True
    # fresh leaves: their AccumulateGrad nodes are created on the capture's
    # side stream, not on the default stream of the eager pass
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in leaves.items()}

    def one():
        for v in leaves.values():
            v.grad = None
        if args.mode != "train":
            with torch.no_grad():
                return mpvae.compute_loss(y, *[leaves[k] for k in ORDER], args)
        out = mpvae.compute_loss(y, *[leaves[k] for k in ORDER], args)
        out[0].backward()
        return out

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(max(2, warmup)):
            one()
    torch.cuda.current_stream().wait_stream(side)
    for v in leaves.values():
        v.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = one()
    for _ in range(max(1, warmup)):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        graph.replay()
    torch.cuda.synchronize()
    return out, time.perf_counter() - t0


def roofline(times, S_local, B, L, z, steps, gemm, valu=None):
    """Dominant kernel's achieved rate vs its bound, from in-library HIP events.
    GEMM work is the algorithmic fp32 GEMM (2*S*B*L*z flops per launch).  With
    L, z <= SMALL_LZ the kernels are VALU-bound: `valu` ({kernel tag: VALU
    lane-instructions per launch}, from a committed PMC profile of the same
    config) prices the dominant kernel against VALU_PEAK instead."""
    mfma_peak, peak_note = PEAKS[gemm]
    work = {  # algorithmic work per launch
        "probit_fwd": ("mfma", 2.0 * S_local * B * L * z, mfma_peak, "TFLOP/s"),
        "dR_gemm": ("mfma", 2.0 * S_local * B * L * z, mfma_peak, "TFLOP/s"),
        "bwd_elem": ("hbm", 8.0 * S_local * B * L, HBM_PEAK, "GB/s"),
        "noise_philox": ("hbm", 4.0 * S_local * B * z, HBM_PEAK, "GB/s"),
    }
    dom = max(times, key=lambda k: times[k][1])
    n, ms = times[dom]
    avg_s = ms / n / 1e3
    small = L <= SMALL_LZ and z <= SMALL_LZ
    if small:
        # VALU-bound: achieved lane-instructions/s of the dominant kernel
        per = (valu or {}).get(dom)
        pk = VALU_PEAK / 1e12
        achieved = per / avg_s / 1e12 if per else None
        ls = S_local * B * L
        res = {"kernel": dom, "bound": "valu", "achieved": achieved, "peak": pk,
               "unit": "Tlane-instr/s", "frac": achieved / pk if achieved else None,
               "traffic": None, "avg_ms": round(avg_s * 1e3, 4),
               "peak_basis": "VALU: 157.3 TFLOPS fp32 vector / 2 = one lane-instruction per "
                             "lane per cycle at 2.4 GHz (packed ops count once, as in "
                             "SQ_INSTS_VALU)",
               "valu_executed_per_ls": per / ls if per else None}
        # the same kernel priced on its ALGORITHMIC instruction floor
        # (VALU_FLOOR_PER_LS): executed-count fractions reward extra work
        if dom in VALU_FLOOR_PER_LS:
            res["frac_algorithmic"] = VALU_FLOOR_PER_LS[dom] * ls / avg_s / VALU_PEAK
            res["valu_floor_per_ls"] = VALU_FLOOR_PER_LS[dom]
        alg = sum(VALU_FLOOR_PER_LS[k] * ls * times[k][0] for k in VALU_FLOOR_PER_LS
                  if k in times) / steps
        res["step_frac_algorithmic"] = alg / (sum(v[1] for v in times.values()) / steps / 1e3) \
            / VALU_PEAK
        if valu:  # the whole step: every profiled kernel's lane-instructions
            tot = sum(valu.get(k, 0.0) * times[k][0] for k in times) / steps
            step_s = sum(v[1] for v in times.values()) / steps / 1e3
            res["step_valu_frac"] = tot / step_s / VALU_PEAK
        res["ms_per_step_by_op"] = {k: round(v[1] / steps, 4) for k, v in
                                    sorted(times.items(), key=lambda kv: -kv[1][1])}
        return res
    if dom in work:
        bound, per_launch, peak, unit = work[dom]
        scale = 1e12 if unit == "TFLOP/s" else 1e9
        achieved = per_launch / avg_s / scale
        pk = peak / scale
        frac = achieved / pk
    else:
        bound, achieved, pk, unit, frac = "unknown", None, None, None, None
    # milliseconds per step of every timed op (an op may be several launches)
    breakdown = {k: round(v[1] / steps, 4) for k, v in sorted(times.items(),
                                                              key=lambda kv: -kv[1][1])}
    return {"kernel": dom, "bound": bound, "achieved": achieved, "peak": pk, "unit": unit,
            "frac": frac, "traffic": None, "peak_basis": peak_note if bound == "mfma" else
            "HBM3E spec", "avg_ms": round(avg_s * 1e3, 4),
            "ms_per_step_by_op": breakdown}


def pmc_valu(config):
    """{kernel tag: VALU lane-instructions per launch} from the newest committed
    PMC summary of this config that holds them (tools/valu_summary.py:
    (SQ_INSTS_VALU - SQ_INSTS_MFMA) x 64 per launch), with its path."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc.json")))[::-1]:
        ks = json.load(open(f)).get("kernels", {})
        v = {k: d["valu_lane_insts_per_launch"] for k, d in ks.items()
             if d.get("valu_lane_insts_per_launch")}
        if v:
            return v, os.path.relpath(f, ROOT)
    return None, None


def pmc_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC
    summary for this config (profiles/r*_<config>_pmc.json, tools/profile.sh +
    tools/pmc_summary.py); None when no profile of this kernel exists."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc.json")))
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    k = data.get("kernels", {}).get(kernel)
    if not k or k.get("hbm_bytes_per_launch") is None:
        return None, None
    return k["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def trace_avg_ms(config, kernel):
    """The committed rocprofv3 trace's average duration of `kernel` over the
    bench's timed steps (cross-check of the in-library HIP-event timing)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config}_pmc.json")))
    if not files:
        return None
    k = json.load(open(files[-1])).get("kernels", {}).get(kernel) or {}
    return k.get("avg_ms_trace_timed_steps", k.get("avg_ms_trace"))


def cpu_baseline(L, z, B, d, S_cpu, reps, device):
    """Reference algorithm restated in torch (oracle/torch_ref.py) on the host
    cores, fwd+bwd on a bounded slice of the workload; also the ELBO rel-err of
    the GPU path on the same slice."""
    sys.path.insert(0, ROOT)
    from oracle import torch_ref
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(99)
    y = (torch.rand((B, L), generator=g) < 0.15).float()
    y[:, 0], y[:, 1] = 1.0, 0.0
    mk = lambda *s: torch.randn(*s, generator=g)
    base = dict(fe_out=mk(B, L), fe_mu=mk(B, d), fe_logvar=0.1 * mk(B, d), fx_out=mk(B, L),
                fx_mu=mk(B, d), fx_logvar=0.1 * mk(B, d),
                r_sqrt_sigma=(torch.rand((L, z), generator=g, dtype=torch.float64) * 2 - 1)
                * (6.0 / (L + z)) ** 0.5)
    noise = mk(S_cpu, B, z)
    best = float("inf")
    cpu_out = None
    for _ in range(reps):
        leaves = {k: v.clone().requires_grad_(True) for k, v in base.items()}
        t0 = time.perf_counter()
        out = torch_ref.elbo_naive(y, *[leaves[k] for k in ORDER], noise, 0.1, 200.0)
        out[0].backward()
        best = min(best, time.perf_counter() - t0)
        cpu_out = (out[0].detach(), leaves["fe_out"].grad, leaves["r_sqrt_sigma"].grad)
    # same slice on the GPU path (explicit noise) -> ELBO rel-err
    gl = {k: v.to(device).requires_grad_(True) for k, v in base.items()}
    a = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S_cpu, n_test_sample=S_cpu,
                           mode="train", nll_coeff=0.1, c_coeff=200.0, mpvae_noise=noise)
    out = mpvae.compute_loss(y.to(device), *[gl[k] for k in ORDER], a)
    out[0].backward()
    rel = lambda p, q: float((p.detach().cpu().double() - torch.as_tensor(q).double()).abs().max()
                             / torch.as_tensor(q).double().abs().max())
    # against the fp64-reduction oracle (the parity checker, oracle/probit_elbo.py)
    # and against the torch-CPU port, whose fp32 1 - E near E -> 1 alone moves
    # d fe_out by ~2e-3 (tests/test_oracle_golden.py::test_torch_port_spread_...)
    from oracle import probit_elbo as pe
    npb = {k: v.numpy() for k, v in base.items()}
    ins = [y.numpy()] + [npb[k] for k in ORDER[:6]]
    ref = pe.elbo_forward(*ins, npb["r_sqrt_sigma"], noise.numpy(), 0.1, 200.0)
    rg = pe.elbo_backward(ref, *ins, noise.numpy(), 0.1, 200.0, g_total=1.0)
    errs = {"vs_oracle": {"total": rel(out[0], ref["total"]),
                          "d_fe_out": rel(gl["fe_out"].grad, rg["fe_out"]),
                          "d_fx_out": rel(gl["fx_out"].grad, rg["fx_out"]),
                          "d_r_sqrt_sigma": rel(gl["r_sqrt_sigma"].grad, rg["r_sqrt_sigma"])},
            "vs_torch_port": {"total": rel(out[0], cpu_out[0]),
                              "d_fe_out": rel(gl["fe_out"].grad, cpu_out[1]),
                              "d_r_sqrt_sigma": rel(gl["r_sqrt_sigma"].grad, cpu_out[2])}}
    return {"value": S_cpu * B * L / best, "unit": "label-samples/s", "cores": threads,
            "kind": "port",
            "sample": f"B={B} L=z={L} n_sample={S_cpu} fwd+bwd, oracle/torch_ref.elbo_naive "
                      f"(reference algorithm, O(S*B*L^2) ranking tensor), best of {reps}, "
                      f"{best:.2f} s/rep"}, errs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: DEFAULT_STEPS[config]")
    ap.add_argument("--warmup", type=int, default=None, help="default: DEFAULT_STEPS[config]")
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-s", type=int, default=2)
    ap.add_argument("--cpu-reps", type=int, default=2)
    ap.add_argument("--gemm", default="f16x3", choices=sorted(PEAKS))
    # eval: the forward-only evaluation call (fairsoft_evaluate.py:40,72-74 with
    # fairsoft_trial.py:70: mode 'test', n_sample = n_test_sample = 10000 unless
    # --eval-samples); not the headline metric
    ap.add_argument("--mode", default="train", choices=["train", "eval"])
    ap.add_argument("--eval-samples", type=int, default=10000)
    # graph: the step captured once in a HIP graph (torch.cuda.graph) and replayed,
    # its Philox key a device tensor the step advances (mpv_noise_philox*_dev);
    # per-kernel times (roofline) come from an eager pass of the same step
    ap.add_argument("--graph", action="store_true")
    # strong (default): the config's n_sample split over the ranks; weak: n_sample
    # per rank (n_sample * N in total)
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--n-sample", type=int, default=None,
                    help="override the config's n_sample (train mode)")
    cli = ap.parse_args()
    if cli.steps is None:
        cli.steps = DEFAULT_STEPS[cli.config][0]
    if cli.warmup is None:
        cli.warmup = DEFAULT_STEPS[cli.config][1]

    if mpvae_launch.needs_spawn(cli.gpus):
        # plain `python bench.py --gpus N`: N rank processes, started before
        # this process makes any GPU call; rank 0's JSON line is relayed
        sys.exit(mpvae_launch.launch_ranks(cli.gpus, [sys.executable, os.path.abspath(__file__)]
                                           + sys.argv[1:]))
    world, rank, local = setup_dist()
    forced = dist.is_initialized() and world == 1
    if world != cli.gpus:
        log(f"warning: --gpus {cli.gpus} but WORLD_SIZE {world}; using {world}")
    device = torch.device("cuda", local)
    L, z, B, S, d, nllc, cc = CONFIGS[cli.config]
    scaling = cli.scaling
    if cli.n_sample is not None:
        S = cli.n_sample
    if cli.mode == "eval":
        S = cli.eval_samples
    S_total = S * world if scaling == "weak" else S
    # this rank's share (mpvae_dist.split_samples: the first S % world ranks
    # take one more; the roofline uses rank 0's)
    S_local = S if scaling == "weak" else S // world + (1 if S % world else 0)
    args = argparse.Namespace(label_dim=L, z_dim=z, n_train_sample=S_total,
                              n_test_sample=S_total, mode="train" if cli.mode == "train" else "test",
                              nll_coeff=nllc, c_coeff=cc,
                              mpvae_noise="philox", mpvae_shard=world > 1 or forced,
                              mpvae_force_exchange=forced, mpvae_gemm=cli.gemm)
    y, leaves = make_inputs(L, z, B, d, device)
    lib = H.load_library()

    for it in range(cli.warmup):
        step(y, leaves, args, it)
    torch.cuda.synchronize()
    lib.mpv_timing_enable(1)
    lib.mpv_timing_reset()
    comm = mpvae_dist.COMM_TIMER
    comm.reset()
    comm.enabled = dist.is_initialized()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(cli.steps):
        out = step(y, leaves, args, 1000 + it)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lib.mpv_timing_enable(0)
    comm.enabled = False
    times = H.kernel_times()
    comm_by_op = comm.summary() if dist.is_initialized() else None
    graph_note = None
    if cli.graph:
        if world > 1 or forced:
            raise SystemExit("--graph runs one process (no collectives in the captured step)")
        del out  # the eager pass's autograd graph
        out, elapsed = graph_steps(y, leaves, args, cli.warmup, cli.steps)
        graph_note = "HIP graph replay of the captured step (ms_per_step, value); roofline " \
                     "kernel times from the eager pass of the same step"
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    finite = bool(torch.isfinite(out[0]).item())
    value = S_total * B * L * cli.steps / elapsed
    prof_key = cli.config if cli.mode == "train" else cli.config + "eval"
    valu, valu_src = pmc_valu(prof_key)
    rl = roofline(times, S_local, B, L, z, cli.steps, cli.gemm, valu)
    if rl["bound"] == "valu":
        rl["valu_source"] = valu_src
    rl["traffic"], rl["traffic_source"] = pmc_traffic(prof_key, rl["kernel"])
    rl["rocprof_avg_ms"] = trace_avg_ms(prof_key, rl["kernel"])
    # collectives of the sample-shard exchange (ms per step) and every rank's
    # per-op kernel times: a multi-GPU line explains its own scaling loss
    comm_ms, ranks = None, None
    if comm_by_op is not None:
        per_step = {op: {k: (round(v / cli.steps, 4) if isinstance(v, float) else v)
                         for k, v in d.items()} for op, d in comm_by_op.items()}
        dev_ms = sum(d["device_ms"] or 0.0 for d in comm_by_op.values()) / cli.steps
        host_ms = sum(d["host_ms"] for d in comm_by_op.values()) / cli.steps
        mine = {"rank": rank, "ms_per_step_by_op": rl["ms_per_step_by_op"],
                "comm_device_ms": round(dev_ms, 4), "comm_host_ms": round(host_ms, 4),
                "comm_by_op": per_step}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        comm_ms = {"device_max": max(r["comm_device_ms"] for r in ranks),
                   "host_max": max(r["comm_host_ms"] for r in ranks),
                   "note": "per step; device: CUDA events around each collective on the "
                           "issuing stream (RCCL), host: wall clock around the call (gloo "
                           "blocks the host)"}

    cpu, errs = None, None
    if rank == 0 and world == 1 and not cli.no_cpu_baseline and cli.mode == "train":
        S_cpu = max(1, min(cli.cpu_sample_s, S))
        cpu, errs = cpu_baseline(L, z, B, d, S_cpu, cli.cpu_reps, device)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "label-samples/s", "n_gpus": world,
            "steps": cli.steps, "warmup": cli.warmup, "ms_per_step": elapsed / cli.steps * 1e3,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{cli.config}: compute_loss "
                                   f"{'fwd+bwd' if cli.mode == 'train' else 'forward only (eval)'}, "
                                   f"B={B}, L={L}, z={z}, "
                                   f"n_sample={S_total} ({S_local}/GPU), philox noise on device",
                       "global_batch": B, "n_sample": S_total, "label_dim": L, "z_dim": z,
                       "parallelism": f"n_sample-sharded x{world}", "gemm": cli.gemm,
                       "dist_backend": (os.environ.get("MPVAE_DIST_BACKEND", "nccl")
                                        if dist.is_initialized() else None)},
            "roofline": rl, "cpu_baseline": cpu, "elbo_rel_err": errs, "loss_finite": finite,
        }
        if comm_ms is not None:
            line["comm_ms"] = comm_ms
            line["ranks"] = ranks
        if graph_note:
            line["graph"] = graph_note
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
