"""Sharding of the Monte-Carlo sample axis over ranks.

One process per GPU; every rank holds the same batch, MLP replica and
r_sqrt_sigma, and evaluates samples s in [s_offset, s_offset + S_local) of the
n_sample Monte-Carlo draws.  The reference has no distributed code; what has
to cross ranks for results identical to a single device (up to summation
order) is:

  forward   all_gather of the per-row log-sum-exp statistics bstat (6 x B floats:
            local max m and sum Z of exp(logp - m) per branch + ranking sums),
            combined exactly as M = max m_r, Z = sum Z_r exp(m_r - M)
            (kernel mpv_bstat_combine); all_reduce(SUM) of the (2,B,L) sums of
            E over s behind indiv_prob / indiv_prob_label.
  backward  one all_reduce(SUM) of the packed [d fe_out | d fx_out | d r_sqrt_sigma]
            buffer (the local backward kernels write straight into it).

The MLP parameter gradients are then identical on every rank (they depend
only on the reduced d fe_out / d fx_out / KL terms), so no DDP all-reduce is
needed.  With philox noise, element ((s*B+b)*z+k) of the noise is a function
of its global index only, so the sharded run draws exactly the single-device
noise.  The collectives go through torch.distributed: RCCL ("nccl") over xGMI
on the GPU node, gloo for the CPU tests.
"""
import torch
import torch.distributed as dist


class SampleShardExchange:
    """Exact cross-rank combine of the per-shard statistics and gradients."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)

    def combine(self, bstat, colsum, backend):
        parts = [torch.empty_like(bstat) for _ in range(self.world)]
        dist.all_gather(parts, bstat.contiguous(), group=self.group)
        bstat_global = backend.combine_bstats(torch.stack(parts))
        dist.all_reduce(colsum, group=self.group)
        return bstat_global, colsum

    def reduce_grads(self, flat):
        dist.all_reduce(flat, group=self.group)
        return flat


class Shard:
    def __init__(self, S_local, s_offset, exchange):
        self.S_local, self.s_offset, self.exchange = S_local, s_offset, exchange


def split_samples(n_sample, world, rank):
    """Contiguous split; the first n_sample % world ranks take one extra sample."""
    base, extra = divmod(n_sample, world)
    S_local = base + (1 if rank < extra else 0)
    s_offset = rank * base + min(rank, extra)
    return S_local, s_offset


def shard_for(args, n_sample, group=None):
    """This rank's slice of the sample axis (the whole axis unless args.mpvae_shard).
    args.mpvae_force_exchange runs the collectives even on a world of one (a
    rehearsal of the multi-GPU path on a single GPU)."""
    if not getattr(args, "mpvae_shard", False) or not dist.is_available() \
            or not dist.is_initialized():
        return Shard(n_sample, 0, None)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if world == 1 and not getattr(args, "mpvae_force_exchange", False):
        return Shard(n_sample, 0, None)
    if n_sample < world:
        raise ValueError(f"n_sample={n_sample} cannot be sharded over {world} ranks")
    S_local, s_offset = split_samples(n_sample, world, rank)
    return Shard(S_local, s_offset, SampleShardExchange(group))
