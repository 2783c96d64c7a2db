"""The multi-GPU exchange over RCCL, rehearsed on one GPU: a world-of-one
"nccl" process group with the sample-shard exchange forced on
(args.mpvae_force_exchange) must give the single-device results.  The
collectives (all_gather of bstat, all_reduce of colsum and of the packed
gradient buffer) then run through RCCL on device tensors exactly as on the
8-GPU node, where the driver runs bench.py --gpus 8."""
import argparse
import os
import socket

import pytest
import torch
import torch.distributed as dist

import mpvae

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _step(args, y, leaves):
    for v in leaves.values():
        v.grad = None
    out = mpvae.compute_loss(y, *[leaves[k] for k in ("fe_out", "fe_mu", "fe_logvar", "fx_out",
                                                       "fx_mu", "fx_logvar", "r_sqrt_sigma")],
                             args)
    (out[0] + out[6].sum() * 0.25 + out[7].sum() * 0.5).backward()
    return [o.detach().clone() for o in out], {k: v.grad.clone() for k, v in leaves.items()}


def test_rccl_exchange_world_one_matches_local():
    torch.manual_seed(3)
    B, L, z, d, S = 4, 256, 256, 8, 256
    y = (torch.rand(B, L) < 0.2).float()
    y[:, 0], y[:, 1] = 1, 0
    mk = lambda *s: torch.randn(*s, device=DEV)
    leaves = dict(fe_out=mk(B, L), fe_mu=mk(B, d), fe_logvar=0.1 * mk(B, d), fx_out=mk(B, L),
                  fx_mu=mk(B, d), fx_logvar=0.1 * mk(B, d),
                  r_sqrt_sigma=(torch.rand(L, z, device=DEV, dtype=torch.float64) * 2 - 1) * 0.05)
    for v in leaves.values():
        v.requires_grad_(True)
    y = y.to(DEV)
    base = dict(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S, mode="train",
                nll_coeff=0.1, c_coeff=200.0, mpvae_noise="philox", mpvae_seed=77)
    ref_out, ref_grad = _step(argparse.Namespace(**base), y, leaves)

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=torch.device(DEV))
    runs = []
    try:
        # int seed (agree_seed: broadcast + .item()) and a device-tensor seed
        # (broadcast into a device copy, no host sync); replica check on every
        # call (fp64 checksum bits, MIN / MAX all_reduce) -- all through RCCL
        for seed in (77, torch.tensor([77], dtype=torch.int64, device=DEV)):
            args = argparse.Namespace(**dict(base, mpvae_seed=seed), mpvae_shard=True,
                                      mpvae_force_exchange=True, mpvae_check_replicas=True)
            runs.append(_step(args, y, leaves))
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    # a world of one combines exactly (M = m, Z = Z e^0, sums of one term)
    for out, grad in runs:
        for a, b in zip(out, ref_out):
            assert torch.allclose(a, b, rtol=1e-6, atol=0.0), (a, b)
        for k in grad:
            assert torch.allclose(grad[k], ref_grad[k], rtol=1e-6, atol=1e-12), k


def _gloo_worker(rank, world, port, q):
    """One rank of an N-rank job sharing cuda:0, exchange over gloo on device
    tensors: the HIP shard backend + SampleShardExchange + a real N-rank
    all_gather of bstat, against the unsharded call on the same inputs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        g = torch.Generator(device=DEV).manual_seed(11)
        B, L, z, d, S = 64, 100, 90, 8, 777           # ragged: 389 + 388, or 98 x 1 + 97 x 7
        y = (torch.rand((B, L), device=DEV, generator=g) < 0.2).float()
        y[:, 0], y[:, 1] = 1, 0
        mk = lambda *s: torch.randn(*s, device=DEV, generator=g)
        leaves = dict(fe_out=mk(B, L), fe_mu=mk(B, d), fe_logvar=0.1 * mk(B, d), fx_out=mk(B, L),
                      fx_mu=mk(B, d), fx_logvar=0.1 * mk(B, d),
                      r_sqrt_sigma=(torch.rand((L, z), device=DEV, generator=g,
                                               dtype=torch.float64) * 2 - 1) * 0.1)
        for v in leaves.values():
            v.requires_grad_(True)
        base = dict(label_dim=L, z_dim=z, n_train_sample=S, n_test_sample=S, mode="train",
                    nll_coeff=0.5, c_coeff=10.0, mpvae_noise="philox",
                    mpvae_seed=1000 + 17 * rank)  # rank 0's seed must win
        ref_out, ref_grad = _step(argparse.Namespace(**dict(base, mpvae_seed=1000)), y, leaves)
        out, grad = _step(argparse.Namespace(**base, mpvae_shard=True, mpvae_check_replicas=True),
                          y, leaves)
        torch.cuda.synchronize()
        from tolerances import rel_err
        errs = [rel_err(a.cpu().double().numpy(), b.cpu().double().numpy())
                for a, b in zip(out, ref_out)]
        errs += [rel_err(grad[k].cpu().double().numpy(), ref_grad[k].cpu().double().numpy())
                 for k in grad]
        q.put((rank, errs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_ranks_on_one_gpu_match_unsharded(world):
    """2 ranks, and the driver's 8 (each with its own HIP context on cuda:0;
    an RCCL group cannot hold two ranks of one device, so gloo carries the
    collectives): loss, indiv_prob and gradients equal the unsharded call."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert sorted(r for r, _ in res) == list(range(world))
    for rank, errs in res:
        assert max(errs) <= 1e-5, (rank, errs)


@pytest.mark.parametrize("scaling,n_total", [("strong", 1000), ("weak", 2000)])
def test_bench_spawns_two_ranks_itself(scaling, n_total):
    """`python bench.py --gpus 2` with no torchrun: the bench's own launcher
    starts both ranks (gloo, both on cuda:0 here) and reports n_gpus 2.  The
    default is strong scaling (C2's n_sample = 1000 split 500 + 500); --scaling
    weak gives each rank its own 1000."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    env["MPVAE_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps",
                        "2", "--warmup", "1", "--config", "c2", "--no-cpu-baseline"]
                       + ([] if scaling == "strong" else ["--scaling", "weak"]),
                       env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "n_sample-sharded x2"
    assert line["config"]["n_sample"] == n_total and line["loss_finite"]
    assert line["scaling"] == scaling
