"""Multi-rank S-sharding on CPU (gloo, world_size 2, 3 and 8): the product's
autograd Function + cross-rank exchange (mpvae_dist) with an oracle shard
backend must reproduce the unsharded golden values and gradients."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpvae_dist import SampleShardExchange, split_samples
from mpvae_ops import ElboConfig, ProbitELBO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, names, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golden_io import DIFF, OUTS, fixtures
        from oracle_backend import OracleShardBackend
        from tolerances import FWD_RTOL, GRAD_RTOL, rel_err
        res = []
        for f in [f for f in fixtures() if f.name in names]:
            S_local, s_off = split_samples(f.S, world, rank)
            t = {k: torch.from_numpy(f[k].copy()) for k in
                 ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar",
                  "r_sqrt_sigma"]}
            for k in DIFF + (["r_sqrt_sigma"] if f.trainable_r else []):
                t[k].requires_grad_(True)
            noise = torch.from_numpy(f["noise"][s_off:s_off + S_local].copy())
            cfg = ElboConfig(f.S, S_local, s_off, f.nll_coeff, f.c_coeff,
                             backend=OracleShardBackend(), exchange=SampleShardExchange())
            out = ProbitELBO.apply(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"], t["fx_out"],
                                   t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"], noise, cfg)
            errs = {k: rel_err(o.detach().numpy(), f["out_" + k]) for k, o in zip(OUTS, out)}
            obj = out[0] + (out[6] * torch.from_numpy(f["g_I"])).sum() + \
                (out[7] * torch.from_numpy(f["g_IL"])).sum()
            obj.backward()
            for k, v in f.grads("gtot").items():
                errs["d" + k] = rel_err(t[k].grad.numpy(), v)
            ok = all(v <= (FWD_RTOL if not k.startswith("d") else GRAD_RTOL)
                     for k, v in errs.items())
            res.append((f.name, ok, errs))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_elbo_matches_unsharded_reference(world):
    """world 8 rehearses the driver's 8-GPU node on the CPU (ragged shards:
    16 samples as 2 each, 12 as 2,2,2,2,1,1,1,1)."""
    names = ["f1_l38", "f2_degenerate", "f3_adult_like"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, names, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in results:
        assert len(res) == len(names)
        for name, ok, errs in res:
            assert ok, (rank, name, errs)


def test_check_replicas_schedule(monkeypatch):
    """mpvae_check_replicas: None -> first sharded call only, True -> every
    call, k > 1 -> every k-th call, False -> never."""
    import argparse
    import mpvae_dist as D
    monkeypatch.setattr(D.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(D.dist, "get_world_size", lambda group=None: 2)
    monkeypatch.setattr(D.dist, "get_rank", lambda group=None: 0)
    for check, want in ((None, [1, 0, 0, 0, 0]), (True, [1] * 5), (False, [0] * 5),
                        (3, [1, 0, 0, 1, 0])):
        monkeypatch.setattr(D, "_SHARDED_CALLS", 0)
        a = argparse.Namespace(mpvae_shard=True, mpvae_check_replicas=check)
        got = [int(D.shard_for(a, 10).exchange.verify) for _ in range(5)]
        assert got == want, (check, got)


def test_split_samples_covers_axis():
    for n, w in [(10, 3), (4096, 8), (7, 7), (1000, 6)]:
        parts = [split_samples(n, w, r) for r in range(w)]
        assert sum(p[0] for p in parts) == n
        assert [p[1] for p in parts] == list(np.cumsum([0] + [p[0] for p in parts])[:-1])


def _replica_worker(rank, world, port, q):
    """Rank-dependent fe_out must raise ReplicaMismatch on every rank; the
    Philox seed is rank 0's whatever each rank proposes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golden_io import fixtures
        from mpvae_dist import ReplicaMismatch
        from oracle_backend import OracleShardBackend
        f = next(f for f in fixtures() if f.name == "f1_l38")
        ex = SampleShardExchange(verify=True)
        dev_seed = ex.agree_seed(torch.tensor([7000 + rank], dtype=torch.int64), "cpu")
        seeds = (ex.agree_seed(1000 + rank, "cpu"), ex.agree_seed(2 ** 64 - 1 - rank, "cpu"),
                 int(dev_seed[0]), tuple(dev_seed.shape), str(dev_seed.dtype))
        S_local, s_off = split_samples(f.S, world, rank)
        t = {k: torch.from_numpy(f[k].copy()) for k in
             ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar",
              "r_sqrt_sigma"]}
        noise = torch.from_numpy(f["noise"][s_off:s_off + S_local].copy())
        outcome = []
        for perturb in (False, True, "nan"):
            fe = t["fe_out"].clone()
            if perturb is True and rank == world - 1:
                fe[0, 0] += 1e-3   # one element on one rank
            if perturb == "nan":   # identical NaN / opposite infinities on every rank
                fe[0, 0], fe[1, 1], fe[2, 2] = float("nan"), float("inf"), float("-inf")
            cfg = ElboConfig(f.S, S_local, s_off, f.nll_coeff, f.c_coeff,
                             backend=OracleShardBackend(), exchange=ex)
            try:
                ProbitELBO.apply(t["y"], fe, t["fe_mu"], t["fe_logvar"], t["fx_out"], t["fx_mu"],
                                 t["fx_logvar"], t["r_sqrt_sigma"], noise, cfg)
                outcome.append("ok")
            except ReplicaMismatch as e:
                outcome.append("mismatch" if "fe_out" in str(e) else str(e))
        q.put((rank, seeds, outcome))
    finally:
        dist.destroy_process_group()


def test_replica_contract_is_enforced():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seeds, outcome in results:
        assert seeds == (1000, 2 ** 64 - 1, 7000, (1,), "torch.int64"), (rank, seeds)
        assert outcome == ["ok", "mismatch", "ok"], (rank, outcome)


def _comm_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mpvae_dist
        from golden_io import fixtures
        from oracle_backend import OracleShardBackend
        f = next(f for f in fixtures() if f.name == "f1_l38")
        S_local, s_off = split_samples(f.S, world, rank)
        t = {k: torch.from_numpy(f[k].copy()).requires_grad_(k != "y") for k in
             ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar",
              "r_sqrt_sigma"]}
        noise = torch.from_numpy(f["noise"][s_off:s_off + S_local].copy())
        timer = mpvae_dist.COMM_TIMER
        timer.reset()
        timer.enabled = True
        for _ in range(2):
            cfg = ElboConfig(f.S, S_local, s_off, f.nll_coeff, f.c_coeff,
                             backend=OracleShardBackend(), exchange=SampleShardExchange())
            out = ProbitELBO.apply(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"], t["fx_out"],
                                   t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"], noise, cfg)
            out[0].backward()
        timer.enabled = False
        q.put((rank, timer.summary()))
    finally:
        dist.destroy_process_group()


def test_comm_timer_records_every_collective():
    """bench.py --gpus N reports comm_ms from mpvae_dist.COMM_TIMER: with the
    timer on, each collective of the exchange is recorded once per call (host
    clock; CPU tensors have no device events), and nothing when it is off."""
    import mpvae_dist
    assert not mpvae_dist.COMM_TIMER.enabled
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, summ in results:
        # the forward's statistics travel in one packed all_reduce
        assert set(summ) == {"combine_all_reduce", "reduce_grads"}, summ
        assert all(d["calls"] in (None, 2) for d in summ.values()), summ
        for op, d in summ.items():
            assert d["device_ms"] is None and d["host_ms"] > 0.0, (rank, op, d)


def _host_worker(rank, world, port, q):
    """compute_loss itself on CPU tensors with args.mpvae_shard: the product's
    host backend (libmpvae_host.so) on every rank, the exchange over gloo."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mpvae
        from golden_io import DIFF, OUTS, fixtures
        from tolerances import FWD_RTOL, GRAD_RTOL, rel_err
        res = []
        for f in [f for f in fixtures() if f.name in ("f1_l38", "f2_degenerate", "f6_l81")]:
            t = {k: torch.from_numpy(f[k].copy()) for k in
                 ["y", "fe_out", "fe_mu", "fe_logvar", "fx_out", "fx_mu", "fx_logvar",
                  "r_sqrt_sigma"]}
            for k in DIFF + (["r_sqrt_sigma"] if f.trainable_r else []):
                t[k].requires_grad_(True)
            args = f.args(mpvae_noise=torch.from_numpy(f["noise"]), mpvae_shard=True,
                          mpvae_check_replicas=True)
            out = mpvae.compute_loss(t["y"], t["fe_out"], t["fe_mu"], t["fe_logvar"],
                                     t["fx_out"], t["fx_mu"], t["fx_logvar"], t["r_sqrt_sigma"],
                                     args)
            errs = {k: rel_err(o.detach().numpy(), f["out_" + k]) for k, o in zip(OUTS, out)}
            obj = out[0] + (out[6] * torch.from_numpy(f["g_I"])).sum() + \
                (out[7] * torch.from_numpy(f["g_IL"])).sum()
            obj.backward()
            for k, v in f.grads("gtot").items():
                g = t[k].grad.double().numpy()
                errs["d" + k] = rel_err(g, v) if np.array_equal(np.isnan(g), np.isnan(v)) \
                    else float("inf")
            ok = all(v <= (FWD_RTOL if not k.startswith("d") else GRAD_RTOL)
                     for k, v in errs.items())
            res.append((f.name, ok, errs))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_compute_loss_on_the_host_backend(world):
    """The drop-in compute_loss with args.mpvae_shard on CPU tensors: every rank
    runs the host C++ backend on its sample shard, the statistics and gradients
    cross ranks over gloo, and the result is the reference's golden record."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in results:
        for name, ok, errs in res:
            assert ok, (rank, name, errs)
