"""Sharding of the Monte-Carlo sample axis over ranks.

One process per GPU; every rank holds the same batch, MLP replica and
r_sqrt_sigma, and evaluates samples s in [s_offset, s_offset + S_local) of the
n_sample Monte-Carlo draws.  The reference has no distributed code; what has
to cross ranks for results identical to a single device (up to summation
order) is:

  forward   one all_reduce(SUM) of a packed buffer [the (2,B,L) sums of E over
            s behind indiv_prob / indiv_prob_label | world slots of the per-row
            log-sum-exp statistics bstat (6 x B floats: local max m and sum Z
            of exp(logp - m) per branch + ranking sums)], each rank's bstat in
            its own slot and zeros elsewhere, so the sum is also the exact
            all_gather of bstat; combined as M = max m_r, Z = sum Z_r
            exp(m_r - M) (kernel mpv_bstat_combine).
  backward  one all_reduce(SUM) of the packed [d fe_out | d fx_out | d r_sqrt_sigma]
            buffer (the local backward kernels write straight into it).

The MLP parameter gradients are then identical on every rank (they depend
only on the reduced d fe_out / d fx_out / KL terms), so no DDP all-reduce is
needed.  With philox noise, element ((s*B+b)*z+k) of the noise is a function
of its global index only, so the sharded run draws exactly the single-device
noise.  The collectives go through torch.distributed: RCCL ("nccl") over xGMI
on the GPU node, gloo for the CPU tests.

Replica contract.  Every rank must hold the same y / fe_out / fx_out /
r_sqrt_sigma (same batch, same dropout masks, same reparameterisation draws:
seed torch and numpy identically on every rank) -- otherwise the combined
statistics mix different forward graphs and the MLP replicas drift apart
silently.  Two guards:
  * the Philox seed is broadcast from the group's rank 0 (agree_seed), so a
    per-rank seed (the common seed + rank pattern) cannot split the noise;
  * verify_replicas compares an order-sensitive fp64 checksum of those four
    tensors across ranks (all_reduce MIN and MAX of its bit pattern, so NaNs
    and infinities in identical replicas compare equal) and raises
    ReplicaMismatch on every rank when they differ.  It costs one host sync, so
    by default it runs on the first sharded compute_loss of the process only;
    args.mpvae_check_replicas = True checks every call, an int k > 1 every k-th
    call (catches later drift, e.g. from nondeterministic MLP backward kernels),
    False never.
"""
import time

import torch
import torch.distributed as dist


class CommTimer:
    """Optional timing of the exchange's collectives (bench.py --gpus N).

    While enabled, every collective of SampleShardExchange.combine /
    reduce_grads is bracketed by CUDA events on the current stream (RCCL makes
    that stream wait for the collective, so the pair spans it; for device
    tensors these events are the device-side cost) and by a host clock (gloo
    blocks the host until its collective is done).  Off by default: nothing
    is recorded and no event is created on the product path."""

    def __init__(self):
        self.enabled = False
        self.reset()

    def reset(self):
        self._events = {}  # op -> [(start, end), ...]
        self._host = {}    # op -> seconds

    def run(self, op, device, fn):
        if not self.enabled:
            return fn()
        cuda = isinstance(device, torch.device) and device.type == "cuda"
        if cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
        t0 = time.perf_counter()
        out = fn()
        self._host[op] = self._host.get(op, 0.0) + time.perf_counter() - t0
        if cuda:
            b.record()
            self._events.setdefault(op, []).append((a, b))
        return out

    def summary(self):
        """{op: {"calls", "device_ms", "host_ms"}} (synchronizes the device)."""
        out = {}
        for op in sorted(set(self._events) | set(self._host)):
            ev = self._events.get(op, [])
            if ev:
                ev[-1][1].synchronize()
            out[op] = {"calls": len(ev) or None,
                       "device_ms": sum(a.elapsed_time(b) for a, b in ev) if ev else None,
                       "host_ms": 1e3 * self._host.get(op, 0.0)}
        return out


COMM_TIMER = CommTimer()


class ReplicaMismatch(RuntimeError):
    """Ranks of a sample-sharded compute_loss hold different inputs."""


_SHARDED_CALLS = 0


def replica_checksum(tensors):
    """(2 * len(tensors),) fp64 checksum: plain sum and a position-weighted sum
    of each tensor (identical tensors give bitwise identical checksums on
    identical devices; a permutation or a single changed element does not)."""
    out = []
    for t in tensors:
        x = t.detach().reshape(-1).to(torch.float64)
        w = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.float64)
        w = torch.remainder(w * 0.6180339887498949, 1.0) + 0.5
        out += [x.sum(), (x * w).sum()]
    return torch.stack(out)


class SampleShardExchange:
    """Exact cross-rank combine of the per-shard statistics and gradients."""

    def __init__(self, group=None, verify=False):
        self.group = group
        self.world = dist.get_world_size(group)
        self.verify = verify

    def _src(self):
        return 0 if self.group is None else dist.get_global_rank(self.group, 0)

    def agree_seed(self, seed, device):
        """The Philox seed of the group's rank 0, on every rank.  A device
        tensor seed is broadcast into a copy and stays on the device (no host
        sync); an int comes back as an int."""
        if isinstance(seed, torch.Tensor):
            t = seed.detach().to(device=device, dtype=torch.int64).reshape(1).clone()
            COMM_TIMER.run("seed_broadcast", t.device,
                           lambda: dist.broadcast(t, src=self._src(), group=self.group))
            return t
        u = int(seed) & (2 ** 64 - 1)  # the 64-bit Philox key, carried as int64
        t = torch.tensor([u - 2 ** 64 if u >= 2 ** 63 else u], dtype=torch.int64, device=device)
        dist.broadcast(t, src=self._src(), group=self.group)
        return int(t.item()) & (2 ** 64 - 1)

    def verify_replicas(self, tensors):
        """Raise ReplicaMismatch (on every rank) unless all ranks hold the same
        tensors.  No-op unless this exchange was built with verify=True."""
        if not self.verify:
            return
        # compare bit patterns: a NaN checksum (NaN in a replica) or one of
        # opposite infinities must not make identical replicas differ
        ck = replica_checksum(tensors).view(torch.int64)
        lo, hi = ck.clone(), ck.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
        if not torch.equal(lo, hi):
            bad = [i // 2 for i in range(ck.numel()) if int(lo[i]) != int(hi[i])]
            names = ["input_label", "fe_out", "fx_out", "r_sqrt_sigma"]
            raise ReplicaMismatch(
                "sample-sharded compute_loss: ranks hold different "
                + ", ".join(sorted({names[i] if i < len(names) else str(i) for i in bad}))
                + " -- seed torch and numpy identically on every rank (same batch, "
                  "dropout masks and reparameterisation draws)")

    def stat_slots(self):
        """(world, this rank's slot) of the packed forward statistics
        (HipShardBackend.forward_local)."""
        return self.world, dist.get_rank(self.group)

    def combine(self, loc, backend):
        """Global bstat and colsum from a shard's forward_local output: one
        all_reduce of the packed [colsum | bstat slots] buffer (two collectives,
        all_gather + all_reduce, for a backend that does not pack)."""
        bstat, colsum, packed = loc["bstat"], loc["colsum"], loc.get("packed")
        if packed is not None:
            COMM_TIMER.run("combine_all_reduce", packed.device,
                           lambda: dist.all_reduce(packed, group=self.group))
            B = bstat.shape[1]
            slots = packed[colsum.numel():].view(self.world, 6, B)
            return backend.combine_bstats(slots), colsum
        parts = [torch.empty_like(bstat) for _ in range(self.world)]
        COMM_TIMER.run("combine_all_gather", bstat.device,
                       lambda: dist.all_gather(parts, bstat.contiguous(), group=self.group))
        bstat_global = backend.combine_bstats(torch.stack(parts))
        COMM_TIMER.run("combine_all_reduce", colsum.device,
                       lambda: dist.all_reduce(colsum, group=self.group))
        return bstat_global, colsum

    def gather_slots(self, loc):
        """The all-reduced packed buffer as (world, 6, B) bstat slots and the
        summed colsum, for a backend that combines the slots inside its
        finalize launch (HipShardBackend.finalize_slots); None without a
        packed buffer (then combine() is used)."""
        bstat, colsum, packed = loc["bstat"], loc["colsum"], loc.get("packed")
        if packed is None:
            return None
        COMM_TIMER.run("combine_all_reduce", packed.device,
                       lambda: dist.all_reduce(packed, group=self.group))
        B = bstat.shape[1]
        return packed[colsum.numel():].view(self.world, 6, B), colsum

    def reduce_grads(self, flat):
        COMM_TIMER.run("reduce_grads", flat.device, lambda: dist.all_reduce(flat, group=self.group))
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
    rehearsal of the multi-GPU path on a single GPU).  args.mpvae_check_replicas:
    None (default) verifies the replica contract on the first sharded call of
    the process, True on every call, an int k > 1 on every k-th call, False
    never."""
    global _SHARDED_CALLS
    if not getattr(args, "mpvae_shard", False) or not dist.is_available() \
            or not dist.is_initialized():
        return Shard(n_sample, 0, None)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if world == 1 and not getattr(args, "mpvae_force_exchange", False):
        return Shard(n_sample, 0, None)
    if n_sample < world:
        raise ValueError(f"n_sample={n_sample} cannot be sharded over {world} ranks")
    S_local, s_offset = split_samples(n_sample, world, rank)
    check = getattr(args, "mpvae_check_replicas", None)
    if check is None:
        verify = _SHARDED_CALLS == 0
    elif isinstance(check, bool) or int(check) <= 1:
        verify = bool(check)
    else:
        verify = _SHARDED_CALLS % int(check) == 0
    _SHARDED_CALLS += 1
    return Shard(S_local, s_offset, SampleShardExchange(group, verify=verify))
