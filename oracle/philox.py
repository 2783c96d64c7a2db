"""numpy Philox4x32-10 + Box-Muller -- TEST INFRASTRUCTURE ONLY.

Restates the counter-based generator the build uses for its perf-mode probit
noise (the reference draws that noise from torch's CPU generator,
mpvae.py:162; the build's ``noise='philox'`` mode replaces it by design, see
DESIGN.md).  Philox4x32-10 follows Salmon et al., "Parallel random numbers: as
easy as 1, 2, 3" (SC'11) / Random123; pinned by its published known-answer
vectors in tests/test_oracle_golden.py.

Noise element e = ((s_global * B + b) * z + k) of the (S,B,z) tensor is output
word (e mod 4) of philox(counter = (e div 4) as (lo, hi, 0, 0), key = seed,
offset) with words (0,1) and (2,3) Box-Muller pairs:
    u = ((w_even >> 8) + 0.5) * 2^-24,   v = (w_odd >> 8) * 2^-24
    n_even = sqrt(-2 ln u) cos(2 pi v),  n_odd = sqrt(-2 ln u) sin(2 pi v)
The key is (seed_lo, seed_hi); the 64-bit ``offset`` is added to the counter so
successive calls draw disjoint streams.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 on uint32 arrays; returns 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(a, np.uint32).copy() for a in (c0, c1, c2, c3))
    k0 = np.asarray(k0, np.uint32).copy()
    k1 = np.asarray(k1, np.uint32).copy()
    for _ in range(10):
        p0 = c0.astype(np.uint64) * M0
        p1 = c2.astype(np.uint64) * M1
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = ((k0.astype(np.uint64) + np.uint64(W0)) & MASK).astype(np.uint32)
        k1 = ((k1.astype(np.uint64) + np.uint64(W1)) & MASK).astype(np.uint32)
    return c0, c1, c2, c3


def normal_noise(S_local, B, z, seed, offset=0, s_offset=0):
    """(S_local,B,z) float64 noise of the shard starting at global sample s_offset."""
    e0 = s_offset * B * z
    e = np.arange(e0, e0 + S_local * B * z, dtype=np.uint64)
    ctr = e // np.uint64(4) + np.uint64(offset)
    lane = (e % np.uint64(4)).astype(np.int64)
    seed = np.uint64(seed)
    w = philox4x32_10((ctr & MASK).astype(np.uint32), (ctr >> np.uint64(32)).astype(np.uint32),
                      np.zeros_like(ctr, np.uint32), np.zeros_like(ctr, np.uint32),
                      np.full(ctr.shape, seed & MASK, np.uint32),
                      np.full(ctr.shape, seed >> np.uint64(32), np.uint32))
    w = np.stack(w, -1)                                    # (n, 4)
    pair = lane // 2
    we = w[np.arange(len(e)), 2 * pair].astype(np.float64)
    wo = w[np.arange(len(e)), 2 * pair + 1].astype(np.float64)
    u = (np.floor(we / 256.0) + 0.5) * 2.0 ** -24
    v = np.floor(wo / 256.0) * 2.0 ** -24
    r = np.sqrt(-2.0 * np.log(u))
    n = np.where(lane % 2 == 0, r * np.cos(2 * np.pi * v), r * np.sin(2 * np.pi * v))
    return n.reshape(S_local, B, z)
