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
    try:
        args = argparse.Namespace(**base, mpvae_shard=True, mpvae_force_exchange=True)
        out, grad = _step(args, y, leaves)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    # a world of one combines exactly (M = m, Z = Z e^0, sums of one term)
    for a, b in zip(out, ref_out):
        assert torch.allclose(a, b, rtol=1e-6, atol=0.0), (a, b)
    for k in grad:
        assert torch.allclose(grad[k], ref_grad[k], rtol=1e-6, atol=1e-12), k
