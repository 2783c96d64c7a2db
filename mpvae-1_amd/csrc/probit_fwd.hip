// Forward of the MPVAE probit ELBO for one S-shard (reference mpvae.py:145-210).
//
//   probit_fwd16_kernel  t = eps . R^T with 3xf16 split operands on the f16
//                        matrix cores (v_mfma_f32_16x16x32_f16, fp32 accumulate,
//                        ~fp32 accuracy, see mpv_common.h), operand tiles
//                        streamed global->LDS by LDS-DMA (global_load_lds_dwordx4)
//                        into a double-buffered, XOR-swizzled image.
//   probit_fwd_kernel    the same with exact fp32 MFMA (v_mfma_f32_16x16x4_f32)
//                        on fp32 operands (MPV_GEMM_F32, the bit-faithful mode).
//   Both share the fused epilogue: u = t + fe_out / fx_out,
//   E = Phi(u)(1-1e-6)+0.5e-6 for both branches, per-row BCE log-prob and
//   ranking factors P, N (partial over this label tile), column sums of E over
//   s, optional T stash for the backward.
//   fwd_combine_kernel   one block per batch row b: sums the label-tile
//                        partials, writes rowstat, the shard's log-sum-exp
//                        statistics (m, Z) and ranking sums.
//   finalize_kernel      the 8 outputs of compute_loss (+ KL, mpvae.py:147-148).
//
// Tiling: a workgroup owns one batch row b, one label tile [n0, n0+BN) and a
// chunk of s-tiles of BM samples; the GEMM's M axis is s (eps rows for fixed
// b), so fe/fx/y of the epilogue are per-lane constants and the column sums
// over s stay in registers until the workgroup ends.  Workgroups sharing eps
// rows (same b and s-chunk, other label tiles) get ids equal mod 8: one XCD.
#include <cstdlib>
#include <cstring>

#include "abi_util.h"
#include "mpv_common.h"

namespace mpv {

int launch_sum_slabs(const float* in, int64_t nslab, int64_t n, void* out, int out_dtype,
                     hipStream_t s);

struct FwdParams {
  const float* y;
  const float* fe;
  const float* fx;
  const float* R;    // fp32 mode
  const float* eps;  // fp32 mode
  mpv_split16 R16;   // 3xf16 mode
  mpv_split16 eps16;
  float* T;        // (B, S, ldT)
  float* rowpart;  // [6][nNt][B][S]
  float* colpart;  // [nSc][2][B][L]
  int S, B, L, z;
  int ldT;  // t_cols(L)
  int nNt, nSc, tps, nSt;
};

// Tuning constants of the product kernels (each measured; DESIGN.md section 3
// lists the variants that lost and were removed):
// fwd_combine: one block per batch row (512 / 256 threads: C4 0.076 -> 0.115 /
// 0.188 ms, C3 0.023 -> 0.027 / 0.038 ms; round 3; 512 at C2 / C3 +-0, round 6)
#ifndef MPV_COMBINE_THREADS
#define MPV_COMBINE_THREADS 1024
#endif
constexpr int kCombineThreads = MPV_COMBINE_THREADS;
constexpr int kCombineFoldSlabs = 64;  // s-chunk partials fwd_combine sums itself, at most
constexpr int kCombineKeep = 4;        // fwd_combine: samples per thread kept in registers
constexpr int kFwdWant = 2048;         // fp32 mode: target workgroup count of the forward grid
constexpr int kEpiSampleBlocks = 5;    // epilogue: sample blocks between scheduling barriers
// samples per tile of the 48-label tile (L <= 48): 256 (C2 forward 25.1 us;
// 128: 26.8; round 5's MFMA-layout 48 x 128 tile, two workgroups per CU
// without packed fp32: 33.4; same box, eager)
constexpr int kFwd48BM = 256;
// The 256 x 256 tile (probit_fwd16b, L > 128 and S >= 256; round 6, same-box
// A/Bs in profiles/r06_fwd16b_ab.json), C4 forward ms against 13.60 for the
// 256 x 128 tile:
//   kFwdBA    sample blocks of waves 0-3 (of 16): 8 -> 13.07, 9 and 10 -> 12.79;
//             11 and 12 spill
//   kFwdBPart sample blocks per epilogue part: 1 -> 13.44, 2 -> 12.79
//   kFwdBCQ   column-sum slots per 16-lane row: 4 (lane quads) -> 12.58
//   kFwdBEpi, kFwdBUnroll: the label loop's scheduling knobs (fwd_tile_epilogue_t)
#ifndef MPV_FWD_B
#define MPV_FWD_B 1
#endif
#ifndef MPV_FWD_BA
#define MPV_FWD_BA 10
#endif
#ifndef MPV_FWD_BPART
#define MPV_FWD_BPART 2
#endif
#ifndef MPV_FWD_BCQ
#define MPV_FWD_BCQ 4
#endif
#ifndef MPV_FWD_BEPI
#define MPV_FWD_BEPI 2
#endif
#ifndef MPV_FWD_BUNROLL
#define MPV_FWD_BUNROLL 0
#endif
constexpr bool kFwdB = MPV_FWD_B;
constexpr int kFwdBA = MPV_FWD_BA;
constexpr int kFwdBPart = MPV_FWD_BPART;
constexpr int kFwdBCQ = MPV_FWD_BCQ;
constexpr int kFwdBEpi = MPV_FWD_BEPI;
constexpr bool kFwdBUnroll = MPV_FWD_BUNROLL;

constexpr int kBK = 32;   // fp32 mode: K (= z) chunk staged in LDS
constexpr int kLDK = 40;  // fp32 mode: LDS row stride in floats (conflict-free ds_read_b128)

// Block id -> (group g = b*nSc + sc, label tile nt).  All nNt tiles of one
// group get ids equal mod 8 (same XCD under round-robin dispatch; speed only).
MPV_DEV void decode_block(int id, int G, int nNt, int& g, int& nt) {
  const int full = (G / 8) * 8 * nNt;
  if (id < full) {
    const int q = id / (8 * nNt), r = id % (8 * nNt);
    nt = r / 8;
    g = q * 8 + (r % 8);
  } else {
    const int r = id - full, Gr = G % 8;
    nt = r / Gr;
    g = (G / 8) * 8 + (r % Gr);
  }
}

// ------------------------------------------------------------ shared epilogue
// Per-lane constants of the label columns this lane owns (MFMA C layout:
// col = lane & 15 within each 16-wide tile), and its running column sums.
template <int TN>
struct FwdLane {
  f32x2 col[TN];  // running column sums of E: label (.x) and feature (.y) branch
};

template <int WN, int TN>
MPV_DEV void fwd_lane_init(FwdLane<TN>& ln) {
#pragma unroll
  for (int n = 0; n < TN; ++n) ln.col[n] = splat2(0.0f);
}

// Label-column constants of the lane (fe_out, fx_out, y of its TN columns).
template <int TN>
struct FwdCols {
  float fe[TN], fx[TN], y[TN];
  int col[TN];
  bool colok[TN], soft[TN];
};

template <int WN, int TN>
MPV_DEV void fwd_cols_load(FwdCols<TN>& c, const FwdParams& p, int b, int n0, int wn, int lr) {
#pragma unroll
  for (int n = 0; n < TN; ++n) {
    const int col = n0 + wn * TN * 16 + n * 16 + lr;
    c.col[n] = col;
    c.colok[n] = col < p.L;
    const int64_t o = (int64_t)b * p.L + (c.colok[n] ? col : 0);
    c.y[n] = p.y[o];
    c.fe[n] = p.fe[o];
    c.fx[n] = p.fx[o];
    c.soft[n] = !(c.y[n] == 0.0f || c.y[n] == 1.0f);
  }
}

// The same from an LDS copy cols[3][BN] (fe, fx, y of the workgroup's label
// tile, staged once by fwd_cols_stage), so nothing is held in registers or
// re-fetched from global memory across tiles.
template <int WN, int TN>
MPV_DEV void fwd_cols_lds(FwdCols<TN>& c, const float* cols, int L, int n0, int wn, int lr) {
  constexpr int BN = WN * TN * 16;
#pragma unroll
  for (int n = 0; n < TN; ++n) {
    const int cl = wn * TN * 16 + n * 16 + lr;
    c.col[n] = n0 + cl;
    c.colok[n] = n0 + cl < L;
    c.fe[n] = cols[cl];
    c.fx[n] = cols[BN + cl];
    c.y[n] = cols[2 * BN + cl];
    c.soft[n] = !(c.y[n] == 0.0f || c.y[n] == 1.0f);
  }
}

template <int BN>
MPV_DEV void fwd_cols_stage(float* cols, const FwdParams& p, int b, int n0, int nthreads) {
  for (int i = threadIdx.x; i < BN; i += nthreads) {
    const int col = n0 + i;
    const bool ok = col < p.L;
    const int64_t o = (int64_t)b * p.L + (ok ? col : 0);
    cols[i] = ok ? p.fe[o] : 0.0f;
    cols[BN + i] = ok ? p.fx[o] : 0.0f;
    cols[2 * BN + i] = ok ? p.y[o] : 0.0f;
  }
}

// The transposed kernel's layout (kColsT * BN floats): (fe, fx) pairs, then
// y[BN], then the epilogue's per-label constants, one BN array each (so a
// lane reads its 4 labels' values as one f32x4): qa, qb (q = qa E + qb: E for
// y = 1, 1 - E for y = 0, 1 for a pad or soft label), sga, sgb (ranking
// exponent sga E + sgb = sg E), wpos, wneg ([y = 1], [y = 0] of a real label).
// Staged once per workgroup: the labels are the same for all its tiles.
constexpr int kColsT = 9;
enum { kCqa = 3, kCqb, kCsga, kCsgb, kCwpos, kCwneg };
template <int BN>
MPV_DEV void fwd_cols_stage_t(float* cols, const FwdParams& p, int b, int n0, int nthreads) {
  for (int i = threadIdx.x; i < BN; i += nthreads) {
    const int col = n0 + i;
    const bool ok = col < p.L;
    const int64_t o = (int64_t)b * p.L + (ok ? col : 0);
    const float y = ok ? p.y[o] : 0.0f;
    // pre-scaled to the probit's argument units: zq = fma(t, kZq, fe kZq)
    cols[2 * i] = ok ? p.fe[o] * kZq : 0.0f;
    cols[2 * i + 1] = ok ? p.fx[o] * kZq : 0.0f;
    cols[2 * BN + i] = y;
    const float sg = y == 1.0f ? -5.0f * 1.4426950408889634f : 5.0f * 1.4426950408889634f;
    const bool hard = ok && (y == 0.0f || y == 1.0f);
    cols[kCqa * BN + i] = !hard ? 0.0f : (y == 0.0f ? -1.0f : 1.0f);
    cols[kCqb * BN + i] = (hard && y == 1.0f) ? 0.0f : 1.0f;  // 1 - E is exact for E >= 0.5
    cols[kCsga * BN + i] = sg;
    cols[kCsgb * BN + i] = 0.0f;
    cols[kCwpos * BN + i] = (ok && y == 1.0f) ? 1.0f : 0.0f;
    cols[kCwneg * BN + i] = (ok && y == 0.0f) ? 1.0f : 0.0f;
  }
}

// One BM x BN tile of t (acc * scale) starting at sample row s0: probit
// decode, row statistics written to rowpart[., nt, b, s], column sums
// accumulated in `ln`, for the rows s_own <= s < S this tile owns.  Called by
// every thread of the workgroup; uses `smem` (>= WN*BM*6 floats).
template <int WM, int WN, int TM, int TN>
MPV_DEV void fwd_tile_epilogue(const FwdParams& p, FwdLane<TN>& ln, f32x4 (&acc)[TM][TN],
                               float scale, int b, int s0, int s_own, int nt, float* smem,
                               const float* cols = nullptr) {
  constexpr int NT = WM * WN * 64, BM = WM * TM * 16, BN = WN * TN * 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN, lr = lane & 15, lg = lane >> 4;
  const int S = p.S, B = p.B, L = p.L;
  FwdCols<TN> cl;
  if (cols != nullptr) {
    // opaque per call: keeps the column constants (and everything derived
    // from them) from being hoisted out of the tile loop into registers that
    // would then live across the main loop
    int zero = 0;
    asm volatile("" : "+s"(zero));
    fwd_cols_lds<WN, TN>(cl, cols + zero, L, nt * BN + zero, wn, lr);
  } else
    fwd_cols_load<WN, TN>(cl, p, b, nt * BN, wn, lr);
  float* red = smem;  // [WN][BM][6]
  lds_barrier();      // the main loop's last LDS reads are done before red is written
#pragma unroll
  for (int m = 0; m < TM; ++m) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = wm * TM * 16 + m * 16 + lg * 4 + i;
      const int s = s0 + rl;
      const bool rowok = s >= s_own && s < S;
      // row sums, label (.x) and feature (.y) branch: log-prob, P, N
      f32x2 sl = splat2(0.0f), sp = splat2(0.0f), sn = splat2(0.0f);
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const bool ok = rowok && cl.colok[n];
        const float t = acc[m][n][i] * scale;
        if (p.T != nullptr && ok) p.T[((int64_t)b * S + s) * p.ldT + cl.col[n]] = t;
        f32x2 phi;
        const f32x2 E = probit_eval2(splat2(t) + f32x2{cl.fe[n], cl.fx[n]}, phi);
        const float y = cl.y[n];
        // BCE log-prob (mpvae.py:184-185): one log for a 0/1 label
        const f32x2 q = (y == 0.0f) ? splat2(1.0f) - E : E;
        f32x2 lp = f32x2{__builtin_amdgcn_logf(q.x), __builtin_amdgcn_logf(q.y)} *
                   0.6931471805599453f;
        if (cl.soft[n]) {
          lp.x = y * fast_log(E.x) + (1.0f - y) * fast_log(1.0f - E.x);
          lp.y = y * fast_log(E.y) + (1.0f - y) * fast_log(1.0f - E.y);
        }
        // ranking factors (mpvae.py:110-114 factorised): pos -> e^{-5E}, neg -> e^{5E}
        const f32x2 a = E * ((y == 1.0f) ? -5.0f : 5.0f) * 1.4426950408889634f;
        const f32x2 r = f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
        const float wpos = (ok && y == 1.0f) ? 1.0f : 0.0f;
        const float wneg = (ok && y == 0.0f) ? 1.0f : 0.0f;
        sl += ok ? lp : splat2(0.0f);
        sp = pk_fma(splat2(wpos), r, sp);
        sn = pk_fma(splat2(wneg), r, sn);
        ln.col[n] += rowok ? E : splat2(0.0f);
      }
      float st6[6] = {sl.x, sl.y, sp.x, sn.x, sp.y, sn.y};
#pragma unroll
      for (int k = 0; k < 6; ++k) st6[k] = row16_sum_to_lane15(st6[k]);
      if (lr == 15) {
#pragma unroll
        for (int k = 0; k < 6; ++k) red[(wn * BM + rl) * 6 + k] = st6[k];
      }
      if (TM * TN > 8) __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);  // bound live ranges to one m-slab
  }
  lds_barrier();
  for (int r = tid; r < BM; r += NT) {
    const int s = s0 + r;
    if (s >= s_own && s < S) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < WN; ++w) v += red[(w * BM + r) * 6 + k];
        p.rowpart[(((int64_t)k * p.nNt + nt) * B + b) * S + s] = v;
      }
    }
  }
  lds_barrier();
}

// Column sums of this workgroup -> colpart[sc, ., b, n0 ...].
template <int WM, int WN, int TM, int TN>
MPV_DEV void fwd_colsum_epilogue(const FwdParams& p, FwdLane<TN>& ln, int b, int sc, int n0,
                                 float* smem) {
  constexpr int NT = WM * WN * 64, BN = WN * TN * 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN, lr = lane & 15, lg = lane >> 4;
  float* cred = smem;  // [WM][BN][2]
#pragma unroll
  for (int n = 0; n < TN; ++n) {
    float e = ln.col[n].x, x = ln.col[n].y;
    e += __shfl_xor(e, 16, 64);
    e += __shfl_xor(e, 32, 64);
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    if (lg == 0) {
      const int cl = wn * TN * 16 + n * 16 + lr;
      cred[(wm * BN + cl) * 2 + 0] = e;
      cred[(wm * BN + cl) * 2 + 1] = x;
    }
  }
  __syncthreads();
  for (int c = tid; c < BN; c += NT) {
    const int col = n0 + c;
    if (col < p.L) {
      float e = 0.f, x = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        e += cred[(w * BN + c) * 2 + 0];
        x += cred[(w * BN + c) * 2 + 1];
      }
      p.colpart[(((int64_t)sc * 2 + 0) * p.B + b) * p.L + col] = e;
      p.colpart[(((int64_t)sc * 2 + 1) * p.B + b) * p.L + col] = x;
    }
  }
}

// ------------------------------------------------------ exact fp32 mainloop
// Kernels whose workgroups share a CU (several per CU) run one workgroup's
// epilogue VALU beside another's MFMAs on the same SIMD; they are compiled
// without packed fp32 (v_pk_*) instructions: in that configuration a packed
// fp32 op has been seen to lose its low-half result now and then (the
// round-3 128 x 128 tile, DESIGN.md section 3 "Round 5: the lost update"),
// and the same kernel in scalar code never did (0 of 120 launches).
#ifdef __HIP_DEVICE_COMPILE__  // a device-code target feature (the host pass has none)
#define MPV_NO_PK_FP32 __attribute__((target("no-packed-fp32-ops")))
#else
#define MPV_NO_PK_FP32
#endif
template <int WM, int WN, int TM, int TN>
__global__ MPV_NO_PK_FP32 __launch_bounds__(WM* WN * 64) void probit_fwd_kernel(FwdParams p) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = WM * TM * 16;
  constexpr int BN = WN * TN * 16;
  constexpr int A4 = BM * kBK / 4;  // float4 slots of the A (eps) tile
  constexpr int B4 = BN * kBK / 4;
  constexpr int AV = (A4 + NT - 1) / NT;
  constexpr int BV = (B4 + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) float smem[(BM + BN) * kLDK];
  float* As = smem;
  float* Bs = smem + BM * kLDK;

  int g, nt;
  decode_block(blockIdx.x, p.B * p.nSc, p.nNt, g, nt);
  const int b = g / p.nSc, sc = g % p.nSc;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int S = p.S, B = p.B, L = p.L, z = p.z;
  const bool zvec = (z & 3) == 0;

  FwdLane<TN> ln;
  fwd_lane_init<WN, TN>(ln);

  const int nK = (z + kBK - 1) / kBK;
  const int st_end = min(p.nSt, (sc + 1) * p.tps);
  for (int st = sc * p.tps; st < st_end; ++st) {
    const int s0 = st * BM;

    // ---- staging helpers (registers -> LDS), zero padded
    f32x4 ra[AV], rb[BV];
    auto load_tiles = [&](int k0) {
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int idx = tid + v * NT;
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (idx < A4) {
          const int r = idx >> 3, kq = k0 + ((idx & 7) << 2);
          const int s = s0 + r;
          if (s < S) {
            const float* src = p.eps + ((int64_t)s * B + b) * z;
            if (zvec && kq + 3 < z) {
              x = *reinterpret_cast<const f32x4*>(src + kq);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q) x[q] = (kq + q < z) ? src[kq + q] : 0.0f;
            }
          }
        }
        ra[v] = x;
      }
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        const int idx = tid + v * NT;
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (idx < B4) {
          const int r = idx >> 3, kq = k0 + ((idx & 7) << 2);
          const int n = n0 + r;
          if (n < L) {
            const float* src = p.R + (int64_t)n * z;
            if (zvec && kq + 3 < z) {
              x = *reinterpret_cast<const f32x4*>(src + kq);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q) x[q] = (kq + q < z) ? src[kq + q] : 0.0f;
            }
          }
        }
        rb[v] = x;
      }
    };
    auto store_tiles = [&]() {
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const int idx = tid + v * NT;
        if (idx < A4) *reinterpret_cast<f32x4*>(&As[(idx >> 3) * kLDK + ((idx & 7) << 2)]) = ra[v];
      }
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        const int idx = tid + v * NT;
        if (idx < B4) *reinterpret_cast<f32x4*>(&Bs[(idx >> 3) * kLDK + ((idx & 7) << 2)]) = rb[v];
      }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    load_tiles(0);
    store_tiles();
    __syncthreads();
    for (int kc = 0; kc < nK; ++kc) {
      if (kc + 1 < nK) load_tiles((kc + 1) * kBK);
#pragma unroll
      for (int kk = 0; kk < kBK / 16; ++kk) {
        // lane group lg supplies k = kk*16 + 4*lg + j at MFMA step j (a
        // permutation of K shared by A and B: one ds_read_b128 per operand)
        f32x4 a[TM], bb[TN];
#pragma unroll
        for (int m = 0; m < TM; ++m)
          a[m] = *reinterpret_cast<const f32x4*>(
              &As[(wm * TM * 16 + m * 16 + lr) * kLDK + kk * 16 + lg * 4]);
#pragma unroll
        for (int n = 0; n < TN; ++n)
          bb[n] = *reinterpret_cast<const f32x4*>(
              &Bs[(wn * TN * 16 + n * 16 + lr) * kLDK + kk * 16 + lg * 4]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int n = 0; n < TN; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][j], bb[n][j], acc[m][n], 0, 0, 0);
      }
      __syncthreads();
      if (kc + 1 < nK) {
        store_tiles();
        __syncthreads();
      }
    }
    fwd_tile_epilogue<WM, WN, TM, TN>(p, ln, acc, 1.0f, b, s0, s0, nt, smem);
  }
  fwd_colsum_epilogue<WM, WN, TM, TN>(p, ln, b, sc, n0, smem);
}

// ------------------------------------------------------ 3xf16 mainloop
// The K axis (z) is streamed in stages of 32 (one MFMA k-step) through a ring
// of NSTAGE LDS stage images filled by LDS-DMA (global_load_lds_dwordx4).  The
// split operands are chunked (mpv_split16): the hi and lo halves of a row's
// 32-element K slice are one 128-B line, and a stage image row is exactly that
// line: [hi 64 B | lo 64 B].  Image: BM eps rows (A), then BN R rows (B).  One
// DMA wave-instruction moves 8 rows (8 lanes x 16 B per row: whole lines).
// The 16-B unit u of row r sits at position u ^ ((r >> 1) & 7), which makes
// the ds_read_b128 fragment reads (16 rows x one unit per lane group)
// conflict-free (checked exhaustively); LDS-DMA writes
// lane-linearly, so the swizzle goes on the per-lane SOURCE address.
constexpr int kKC = 32;     // K elements per stage
constexpr int kRowB = 128;  // bytes per stage-image row (hi + lo)

// First sample row of s-tile st.  With S >= BM the last tile is shifted back
// to end at S (its leading rows, already owned by tile st-1, are recomputed
// and masked), so no tile reads past the last sample row and the per-lane DMA
// offsets are the same for every tile; with S < BM rows are clamped instead.
template <int BM>
MPV_DEV int fwd_tile_s0(int st, int S) {
  return S >= BM ? min(st * BM, S - BM) : 0;
}

// DMA cursor of one wave: the next K stage to stream, walking the stages of
// every tile this workgroup owns in order (so the first stages of tile i+1
// are fetched while tile i's epilogue runs).  Wave w streams the 8-row pieces
// w, w+NW, ... of each operand image.  A source address is a wave-uniform
// operand/tile base plus a tile-invariant 32-bit per-lane byte offset.
template <int BM, int BN, int NW>
struct Fwd16Dma {
  static constexpr int GA = BM / 8, GB = BN / 8;  // pieces per operand image
  static constexpr int JA = (GA + NW - 1) / NW, JB = (GB + NW - 1) / NW;
  static constexpr bool EVEN = GA % NW == 0 && GB % NW == 0;
  const char* a_base;  // eps rows of the current tile
  const char* b_base;  // R rows of the label tile
  uint32_t offa[JA], offb[JB];
  int tile, kc;  // next stage to issue
  int issued;    // stages issued so far
  int wid;

  MPV_DEV void init(const FwdParams& p, int t0, int b, int n0, int wid_, int lane) {
    wid = wid_;
    const int64_t lda = p.eps16.ld, ldb = p.R16.ld;
    const int prow = lane >> 3, u_lds = lane & 7;
    b_base = reinterpret_cast<const char*>(p.R16.data + (int64_t)n0 * ldb);
#pragma unroll
    for (int j = 0; j < JA; ++j) {
      const int r = (wid + j * NW) * 8 + prow;  // row within the tile
      offa[j] = (uint32_t)((int64_t)min(r, p.S - 1) * lda * 2) +  // rows b*S + s: contiguous
                (uint32_t)((u_lds ^ ((r >> 1) & 7)) * 16);
    }
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int r = (wid + j * NW) * 8 + prow;
      offb[j] = (uint32_t)(r * ldb * 2) + (uint32_t)((u_lds ^ ((r >> 1) & 7)) * 16);
    }
    tile = t0;
    kc = 0;
    issued = 0;
    set_tile(p, b);
  }

  MPV_DEV void set_tile(const FwdParams& p, int b) {
    const int64_t o = ((int64_t)b * p.S + fwd_tile_s0<BM>(tile, p.S)) * p.eps16.ld;
    a_base = reinterpret_cast<const char*>(p.eps16.data + o);
  }

  // pieces this wave streams per stage
  MPV_DEV int per_wave() const {
    if (EVEN) return JA + JB;
    return (GA - wid + NW - 1) / NW + (GB - wid + NW - 1) / NW;
  }

  // base: wave-uniform (SGPRs); off: per-lane byte offset (inline-asm DMA, see lds_dma16)
  MPV_DEV static void piece(const char* base, uint32_t off, char* dst) {
    lds_dma16(base, off, lds_addr(dst));
  }

  // Stream the next stage (if any) into stage image `dst`.
  MPV_DEV void issue(const FwdParams& p, char* dst, int tile_end, int nK, int b) {
    if (tile >= tile_end) return;
    const int kb = kc * kRowB;  // byte offset of the K slice within a row
#pragma unroll
    for (int j = 0; j < JA; ++j) {
      const int pc = wid + j * NW;
      if (GA % NW == 0 || pc < GA) piece(a_base + kb, offa[j], dst + pc * 1024);
    }
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int pc = wid + j * NW;
      if (GB % NW == 0 || pc < GB) piece(b_base + kb, offb[j], dst + BM * kRowB + pc * 1024);
    }
    ++issued;
    if (++kc == nK) {
      kc = 0;
      if (++tile < tile_end) set_tile(p, b);
    }
  }
};

// Operand fragments of one K stage: A (eps rows) and B (R rows), hi and lo.
template <int TM, int TN>
struct Frag16 {
  s16x8 ah[TM], al[TM], bh[TN], bl[TN];
};

// coh / col: swizzled byte positions of this lane's hi and lo units
template <int TM, int TN, int BM>
MPV_DEV void fwd16_read(Frag16<TM, TN>& f, const char* base, int wm, int wn, int lr, int coh,
                        int col) {
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const int off = ((wm * TM + m) * 16 + lr) * kRowB;
    f.ah[m] = *reinterpret_cast<const s16x8*>(base + off + coh);
    f.al[m] = *reinterpret_cast<const s16x8*>(base + off + col);
  }
#pragma unroll
  for (int n = 0; n < TN; ++n) {
    const int off = (BM + (wn * TN + n) * 16 + lr) * kRowB;
    f.bh[n] = *reinterpret_cast<const s16x8*>(base + off + coh);
    f.bl[n] = *reinterpret_cast<const s16x8*>(base + off + col);
  }
}

// acc += hi*hi + hi*lo + lo*hi for one K stage.
template <int TM, int TN>
MPV_DEV void fwd16_mfma(f32x4 (&acc)[TM][TN], const Frag16<TM, TN>& f) {
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(f.ah[m]), as_f16x8(f.bh[n]),
                                                         acc[m][n], 0, 0, 0);
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(f.ah[m]), as_f16x8(f.bl[n]),
                                                         acc[m][n], 0, 0, 0);
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(f.al[m]), as_f16x8(f.bh[n]),
                                                         acc[m][n], 0, 0, 0);
    }
}

// Main loop: a ring of NSTAGE stage images, NSTAGE-1 stages in flight, one
// raw barrier per stage (the DMA stream runs across tile seams).
// Two 4-wave workgroups share each CU (the 48-label tile, 70 KB of LDS):
// no packed fp32 (MPV_NO_PK_FP32, above).
template <int WM, int WN, int TM, int TN, int NSTAGE>
__global__ MPV_NO_PK_FP32 __launch_bounds__(WM* WN * 64, (WM * WN <= 4) ? 2 : 1) void probit_fwd16_kernel(FwdParams p) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
  constexpr int STAGE = (BM + BN) * kRowB;
  static_assert(BM % 8 == 0 && BN % 8 == 0, "operand images are whole 8-row DMA pieces");
  constexpr int RED = (WN * BM * 6 > WM * BN * 2 ? WN * BM * 6 : WM * BN * 2) * 4;
  // one __shared__ array: stage ring, the epilogue's reduction area, and the
  // label tile's fe/fx/y
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE + RED + 3 * BN * 4];
  float* red = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  float* cols = reinterpret_cast<float*>(smem + NSTAGE * STAGE + RED);

  int g, nt;
  decode_block(blockIdx.x, p.B * p.nSc, p.nNt, g, nt);
  const int b = g / p.nSc, sc = g % p.nSc;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lr = lane & 15, lg = lane >> 4;

  FwdLane<TN> ln;
  fwd_lane_init<WN, TN>(ln);
  const float scale = 1.0f / (*p.eps16.scale * *p.R16.scale);
  const int nK = (p.z + kKC - 1) / kKC;
  const int sw = (lr >> 1) & 7;
  const int coh = (lg ^ sw) << 4, col = ((4 + lg) ^ sw) << 4;
  const int t_begin = sc * p.tps, t_end = min(p.nSt, (sc + 1) * p.tps);

  fwd_cols_stage<BN>(cols, p, b, n0, NW * 64);  // visible after the first barrier
  Fwd16Dma<BM, BN, NW> dma;
  dma.init(p, t_begin, b, n0, wid, lane);
  const int my_pieces = dma.per_wave();
#pragma unroll
  for (int j = 0; j < NSTAGE - 1; ++j) dma.issue(p, smem + j * STAGE, t_end, nK, b);

  int gs = 0;  // stages consumed so far (global over the tiles)
  for (int st = t_begin; st < t_end; ++st) {
    const int s0 = fwd_tile_s0<BM>(st, p.S);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kc = 0; kc < nK; ++kc, ++gs) {
      // stage gs must have landed; later stages may stay in flight (loads
      // retire in order, so stores issued after them need not be waited for)
      if (NSTAGE == 2)
        wait_vmcnt<0>();
      else
        wait_vmcnt_dyn(min(dma.issued - (gs + 1), NSTAGE - 2) * my_pieces);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_raw();  // stage gs landed for every wave; every wave is done reading gs-1
      dma.issue(p, smem + ((gs + NSTAGE - 1) % NSTAGE) * STAGE, t_end, nK, b);
      Frag16<TM, TN> f;
      fwd16_read<TM, TN, BM>(f, smem + (gs % NSTAGE) * STAGE, wm, wn, lr, coh, col);
      fwd16_mfma<TM, TN>(acc, f);
    }
    fwd_tile_epilogue<WM, WN, TM, TN>(p, ln, acc, scale, b, s0, st * BM, nt, red, cols);
  }
  fwd_colsum_epilogue<WM, WN, TM, TN>(p, ln, b, sc, n0, red);
}

// ------------------------------------------ 3xf16, transposed accumulators
// The same GEMM with the roles of the operands swapped: MFMA-M = labels (R
// rows), MFMA-N = samples (eps rows).  A lane then holds 4 consecutive labels
// of one sample, which makes the epilogue cheap where it was costly:
//   * the 6 row statistics of a sample sum over labels in-lane, then over the
//     4 lane rows with two row-swap permutes (was: 16-lane DPP trees per row);
//   * T is stored as one 16-B vector per (sample, 4 labels);
//   * column sums over samples reduce once per label group into LDS.
template <int TL, int TS>
struct FragT {
  s16x8 rh[TL], rl[TL], eh[TS], el[TS];  // R (labels) and eps (samples), hi / lo
};

template <int WL, int TL, int TS, int BM>
MPV_DEV void fwd16t_read(FragT<TL, TS>& f, const char* base, int wl, int sbo, int lr, int coh,
                         int col) {
#pragma unroll
  for (int m = 0; m < TL; ++m) {
    const int off = (BM + (wl * TL + m) * 16 + lr) * kRowB;
    f.rh[m] = *reinterpret_cast<const s16x8*>(base + off + coh);
    f.rl[m] = *reinterpret_cast<const s16x8*>(base + off + col);
  }
#pragma unroll
  for (int n = 0; n < TS; ++n) {
    const int off = ((sbo + n) * 16 + lr) * kRowB;
    f.eh[n] = *reinterpret_cast<const s16x8*>(base + off + coh);
    f.el[n] = *reinterpret_cast<const s16x8*>(base + off + col);
  }
}

// The same products per accumulator in the same order (hi.hi, hi.lo, lo.hi),
// issued term by term over all tiles: consecutive MFMAs see operands of one
// kind (-0.75 % against accumulator by accumulator).
template <int TL, int TS>
MPV_DEV void fwd16t_mfma(f32x4 (&acc)[TL][TS], const FragT<TL, TS>& f) {
#pragma unroll
  for (int m = 0; m < TL; ++m)
#pragma unroll
    for (int n = 0; n < TS; ++n)
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(f.rh[m]), as_f16x8(f.eh[n]),
                                                         acc[m][n], 0, 0, 0);
#pragma unroll
  for (int m = 0; m < TL; ++m)
#pragma unroll
    for (int n = 0; n < TS; ++n)
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(f.rh[m]), as_f16x8(f.el[n]),
                                                         acc[m][n], 0, 0, 0);
#pragma unroll
  for (int m = 0; m < TL; ++m)
#pragma unroll
    for (int n = 0; n < TS; ++n)
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(f.rl[m]), as_f16x8(f.eh[n]),
                                                         acc[m][n], 0, 0, 0);
}

// Packed fp32 fma with the scalar operands broadcast from one half of a
// register pair by op_sel.  hipcc does not fold such splats of a VGPR element
// (a per-lane label constant) into op_sel: it materialises each splat with
// two v_mov per use, ~10 % of the epilogue's VALU instructions.
// a * b[H] + c[H]
template <int H>
MPV_DEV f32x2 pk_fma_bc(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  if (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[1,1,1]"
        : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
// sp += p[H] * r, sn += q[H] * r, with r fresh from v_exp_f32 (the s_nop is
// the wait state a VALU read of a transcendental's result needs on gfx950,
// which hipcc does not insert for an asm statement's inputs)
template <int H>
MPV_DEV void pk_fma2_acc_bc(f32x2 p, f32x2 q, f32x2 r, f32x2& sp, f32x2& sn) {
  if (H == 0)
    asm("s_nop 0\n\tv_pk_fma_f32 %0, %2, %4, %0 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %1, %3, %4, %1 op_sel_hi:[0,1,1]"
        : "+v"(sp), "+v"(sn) : "v"(p), "v"(q), "v"(r));
  else
    asm("s_nop 0\n\tv_pk_fma_f32 %0, %2, %4, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %1, %3, %4, %1 op_sel:[1,0,0] op_sel_hi:[1,1,1]"
        : "+v"(sp), "+v"(sn) : "v"(p), "v"(q), "v"(r));
}

// acc[m][n][i] = t of sample (ws*TS+n)*16 + lr, label (wl*TL+m)*16 + 4*lg + i.
// Masks are carried as 0/1 float weights (VGPRs) rather than lane masks: the
// 16 per-label masks of a label group would otherwise pin ~40 SGPRs and spill.
// Every element is finite (R pad rows are zero, eps rows are clamped), so
// weighting instead of selecting is exact.
template <int WL, int WS, int TL, int TS, int BMT = WS * TS * 16, bool RED_IN_RING = false,
          int EPI_BLOCKS = kEpiSampleBlocks, bool UNROLL_L = false, bool PUBLISH = true, int CQ = 1>
MPV_DEV void fwd_tile_epilogue_t(const FwdParams& p, f32x4 (&acc)[TL][TS], float scale,
                                 int b, int s0, int s_own, int nt, float* red, float* cacc,
                                 const float* cols, bool soft_any, int sbo = -1) {
  constexpr int NT = WL * WS * 64, BM = BMT, BN = WL * TL * 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wl = wid % WL, ws = wid / WL, lr = lane & 15, lg = lane >> 4;
  if (sbo < 0) sbo = ws * TS;  // first 16-sample block of this wave
  const int S = p.S, B = p.B, L = p.L, n0 = nt * BN;
  f32x2 sl[TS], sp[TS], sn[TS];  // per sample: log-prob, P, N (label .x / feature .y branch)
#pragma unroll
  for (int n = 0; n < TS; ++n) sl[n] = sp[n] = sn[n] = splat2(0.0f);
#pragma unroll
  for (int m = 0; m < TL; ++m)
#pragma unroll
    for (int n = 0; n < TS; ++n) acc[m][n] = acc[m][n] * scale;  // t (exact: power of 2)
  // wave-uniform: the T stash needs no per-lane row / label conditions
  const bool t_plain = s0 + sbo * 16 >= s_own && s0 + (sbo + TS) * 16 <= S && n0 + BN <= L;
  // one label group per iteration, not unrolled (code size / live ranges):
  // the group's accumulators are always acc[0]; the rest rotate down after it
  // (round 2: unrolled by 2, 15 VGPRs spill; fully, 95.  Round 3's compiler
  // unrolls fully without spilling, and the forward measures the same: C4
  // 13.28 / 13.25 vs 13.33 / 13.20 ms, so the rotation's moves are not on the
  // critical path)
  constexpr int kUnrollL = UNROLL_L ? TL : 1;
#pragma unroll kUnrollL
  for (int m = 0; m < TL; ++m) {
    f32x4 am[TS];
#pragma unroll
    for (int n = 0; n < TS; ++n) am[n] = acc[0][n];
#pragma unroll
    for (int mm = 0; mm + 1 < TL; ++mm)
#pragma unroll
      for (int n = 0; n < TS; ++n) acc[mm][n] = acc[mm + 1][n];
    const int lb = (wl * TL + m) * 16 + lg * 4;  // first of the lane's 4 labels in the tile
    // the two waves of a SIMD take turns at priority, one label group each,
    // so that they finish the label loop together (with a fixed order one of
    // them runs its last third alone, at half the issue rate)
    if (((m + __builtin_amdgcn_readfirstlane(wid / (NT / 128))) & 1) != 0)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
    if (p.T != nullptr && t_plain) {
      // every row of the wave is the tile's own and < S, every label < L:
      // plain 16-B stores, no per-lane conditions (their exec-mask branches
      // were ~50 scalar instructions per label group)
#pragma unroll
      for (int n = 0; n < TS; ++n) {
        const int s = s0 + (sbo + n) * 16 + lr;
        *reinterpret_cast<f32x4*>(p.T + ((int64_t)b * S + s) * p.ldT + n0 + lb) = am[n];
      }
    } else if (p.T != nullptr) {
      // T stash of this label group, at the top of its iteration (all 16
      // stores up front kept the prio-0 waves 4-8 K cycles in store issue)
#pragma unroll
      for (int n = 0; n < TS; ++n) {
        const int s = s0 + (sbo + n) * 16 + lr;
        if (s >= s_own && s < S) {
          float* row = p.T + ((int64_t)b * S + s) * p.ldT + n0;
          if (n0 + lb < L) {  // t_cols rows: the pad labels' t (0) may be written
            *reinterpret_cast<f32x4*>(row + lb) = am[n];
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (n0 + lb + i < L) row[lb + i] = am[n][i];
          }
        }
      }
    }
    const f32x4 pa = *reinterpret_cast<const f32x4*>(cols + 2 * lb);  // (fe, fx) of labels 0, 1
    const f32x4 pb = *reinterpret_cast<const f32x4*>(cols + 2 * lb + 4);  // labels 2, 3
    const f32x2 fex[4] = {f32x2{pa[0], pa[1]}, f32x2{pa[2], pa[3]}, f32x2{pb[0], pb[1]},
                          f32x2{pb[2], pb[3]}};
    const f32x4 y4 = *reinterpret_cast<const f32x4*>(cols + 2 * BN + lb);
    // per label: the ranking exponent sg E = sga E + sgb, q = qa E + qb
    // selecting E (y = 1) or 1 - E (y = 0) without a select, and the
    // positive / negative weights, staged per workgroup by fwd_cols_stage_t
    const f32x4 qa = *reinterpret_cast<const f32x4*>(cols + kCqa * BN + lb);
    const f32x4 qb = *reinterpret_cast<const f32x4*>(cols + kCqb * BN + lb);
    const f32x4 sga = *reinterpret_cast<const f32x4*>(cols + kCsga * BN + lb);
    const f32x4 sgb = *reinterpret_cast<const f32x4*>(cols + kCsgb * BN + lb);
    const f32x4 wpos = *reinterpret_cast<const f32x4*>(cols + kCwpos * BN + lb);
    const f32x4 wneg = *reinterpret_cast<const f32x4*>(cols + kCwneg * BN + lb);
    // the same constants as register pairs (labels 0,1 | 2,3) for pk_fma_bc
    const f32x2 qa2[2] = {f32x2{qa[0], qa[1]}, f32x2{qa[2], qa[3]}};
    const f32x2 qb2[2] = {f32x2{qb[0], qb[1]}, f32x2{qb[2], qb[3]}};
    const f32x2 sga2[2] = {f32x2{sga[0], sga[1]}, f32x2{sga[2], sga[3]}};
    const f32x2 sgb2[2] = {f32x2{sgb[0], sgb[1]}, f32x2{sgb[2], sgb[3]}};
    const f32x2 wpos2[2] = {f32x2{wpos[0], wpos[1]}, f32x2{wpos[2], wpos[3]}};
    const f32x2 wneg2[2] = {f32x2{wneg[0], wneg[1]}, f32x2{wneg[2], wneg[3]}};
    f32x2 ce[4] = {splat2(0.0f), splat2(0.0f), splat2(0.0f), splat2(0.0f)};
#pragma unroll
    for (int n = 0; n < TS; ++n) {
      const int s = s0 + (sbo + n) * 16 + lr;
      const float wr = (s >= s_own && s < S) ? 1.0f : 0.0f;
      const f32x4 t4 = am[n];
      f32x2 zq[4], w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) zq[i] = pk_fma(splat2(t4[i]), splat2(kZq), fex[i]);
      probit_w2xN_zq<4>(zq, w4);
      // E in the reference's rounding order (mpvae.py:171-180: cdf = 0.5 (1 +
      // erf) exact from w = 1 + erf, then cdf (1 - eps1) and + eps1/2 each
      // rounded): near E -> 1, where one fp32 ulp of E is several % of 1 - E,
      // the BCE term log(1 - E) -- and through the row's log-sum-exp weights
      // every gradient of the batch row -- then follows the reference's E
      // bit for bit whenever w does ("Full C4")
      // (one fma instead, rounding once: forward -0.4 %, element pass -1.3 %,
      // step -0.35 %, same box -- scratch/eoA in profiles/r05_dr_ab.json)
      f32x2 E4[4];
      {
#pragma clang fp contract(off)
#pragma unroll
        for (int i = 0; i < 4; ++i) E4[i] = w4[i] * kEh + splat2(kC0);
      }
      f32x2 q[4], r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // BCE operand (mpvae.py:184-185): E for y = 1, 1 - E for y = 0, 1 for a pad label
        q[i] = (i & 1) ? pk_fma_bc<1>(E4[i], qa2[i >> 1], qb2[i >> 1])
                       : pk_fma_bc<0>(E4[i], qa2[i >> 1], qb2[i >> 1]);
        // ranking factors (mpvae.py:110-114 factorised): pos -> e^{-5E}, neg -> e^{5E}
        const f32x2 a = (i & 1) ? pk_fma_bc<1>(E4[i], sga2[i >> 1], sgb2[i >> 1])
                                : pk_fma_bc<0>(E4[i], sga2[i >> 1], sgb2[i >> 1]);
        r[i] = f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
      }
      // sum of the 4 labels' log-probs as ONE log of their product (log2 units,
      // ln 2 applied once per sample): every q >= 4.7e-7 (the delta clamp), so
      // the product of 4 stays >= 5e-26, far from underflow
      const f32x2 q4 = (q[0] * q[1]) * (q[2] * q[3]);
      f32x2 lp = f32x2{__builtin_amdgcn_logf(q4.x), __builtin_amdgcn_logf(q4.y)};
      if (soft_any) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float y = y4[i];
          if (n0 + lb + i < L && !(y == 0.0f || y == 1.0f)) {  // soft label: both BCE terms (q = 1)
            const f32x2 E = E4[i];
            lp.x += y * __builtin_amdgcn_logf(E.x) + (1.0f - y) * __builtin_amdgcn_logf(1.0f - E.x);
            lp.y += y * __builtin_amdgcn_logf(E.y) + (1.0f - y) * __builtin_amdgcn_logf(1.0f - E.y);
          }
        }
      }
      // row sums need no validity weight: only the tile's own rows are published
      sl[n] = sl[n] + lp;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i & 1)
          pk_fma2_acc_bc<1>(wpos2[i >> 1], wneg2[i >> 1], r[i], sp[n], sn[n]);
        else
          pk_fma2_acc_bc<0>(wpos2[i >> 1], wneg2[i >> 1], r[i], sp[n], sn[n]);
        ce[i] = pk_fma(splat2(wr), E4[i], ce[i]);  // column sums of E over the wave's samples
      }
      // kEpiSampleBlocks samples at a time: bounded live ranges vs more independent chains
      if ((n + 1) % EPI_BLOCKS == 0) __builtin_amdgcn_sched_barrier(0);
    }
    // column sums of these 4 labels over the wave's samples: 16-lane trees
    // (8 chains step-major), lane 15 of each row accumulates into the
    // (ws, label) slot it owns
    float cs[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cs[2 * i] = ce[i].x;
      cs[2 * i + 1] = ce[i].y;
    }
    if (CQ == 4) {
      // two DPP steps: the last lane of each quad holds the quad's sum, and
      // the four quads of a row accumulate into their own slots (summed
      // once per workgroup by fwd16t_colpart)
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] = dpp_f<0x111>(cs[j]) + cs[j];
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] = dpp_f<0x112>(cs[j]) + cs[j];
      if ((lr & 3) == 3) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* c = cacc + ((ws * 4 + (lr >> 2)) * BN + lb + i) * 2;
          c[0] += cs[2 * i];
          c[1] += cs[2 * i + 1];
        }
      }
    } else {
      row16_sum_to_lane15_n<8>(cs);
      if (lr == 15) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* c = cacc + (ws * BN + lb + i) * 2;
          c[0] += cs[2 * i];
          c[1] += cs[2 * i + 1];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // bound live ranges to one label group
  }
  // The row sums sp / sn were last written inside pk_fma2_acc_bc's asm, which
  // hipcc's hazard recognizer cannot see into; a VALU write must be 2 wait
  // states ahead of the v_permlane*_swap that reads it (sum_lanegroups_n).
  // (The pad is required by the ISA.  It is NOT what made the round-3
  // 4-wave, two-workgroups-per-CU tile repeatable: that tile still loses one
  // label-branch update of one 16-lane row with the pad in place, with no
  // inline asm at all, with ds_bpermute sums instead of permlanes, and without
  // the T stash; only one workgroup per CU removes it.  DESIGN.md section 3,
  // "the round-3 lost update", tools/studies/race_study.sh.)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // row statistics: sum over the 4 lane rows; lanes of row 0 publish
  float v[TS * 6];
#pragma unroll
  for (int n = 0; n < TS; ++n) {
    sl[n] = sl[n] * 0.6931471805599453f;  // rows outside the tile's own range are not published
    v[n * 6 + 0] = sl[n].x;
    v[n * 6 + 1] = sl[n].y;
    v[n * 6 + 2] = sp[n].x;
    v[n * 6 + 3] = sn[n].x;
    v[n * 6 + 4] = sp[n].y;
    v[n * 6 + 5] = sn[n].y;
  }
  sum_lanegroups_n<TS * 6>(v);  // all chains step-major
  // red aliases the stage image the last K stage was read from: every wave
  // is past its fragment reads once all have met here
  if (RED_IN_RING) lds_barrier();
  if (lg == 0) {
#pragma unroll
    for (int n = 0; n < TS; ++n)
#pragma unroll
      for (int k = 0; k < 6; ++k) red[(wl * BM + (sbo + n) * 16 + lr) * 6 + k] = v[n * 6 + k];
  }
  if (!PUBLISH) return;  // a later call on the tile's other sample blocks publishes
  lds_barrier();
  for (int r = tid; r < BM; r += NT) {
    const int s = s0 + r;
    if (s >= s_own && s < S) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < WL; ++w) v += red[(w * BM + r) * 6 + k];
        p.rowpart[(((int64_t)k * p.nNt + nt) * B + b) * S + s] = v;
      }
    }
  }
  lds_barrier();
}

// Column partials of a transposed-tile workgroup -> colpart[sc, ., b, n0 ...]
template <int WS, int BN, int CQ = 1>
MPV_DEV void fwd16t_colpart(const FwdParams& p, const float* cacc, int b, int sc, int n0,
                            int nthreads) {
  lds_barrier();
  for (int c = threadIdx.x; c < BN; c += nthreads) {
    const int l = n0 + c;
    if (l < p.L) {
      float e = 0.f, x = 0.f;
#pragma unroll
      for (int w = 0; w < WS * CQ; ++w) {
        e += cacc[(w * BN + c) * 2 + 0];
        x += cacc[(w * BN + c) * 2 + 1];
      }
      p.colpart[(((int64_t)sc * 2 + 0) * p.B + b) * p.L + l] = e;
      p.colpart[(((int64_t)sc * 2 + 1) * p.B + b) * p.L + l] = x;
    }
  }
}

// Does the workgroup's label tile hold soft (non 0/1) labels?  (uniform;
// enables the two-log BCE path of the epilogue)
template <int BN>
MPV_DEV bool fwd_tile_soft(const FwdParams& p, int b, int n0, int nthreads) {
  bool my_soft = false;
  for (int i = threadIdx.x; i < BN; i += nthreads) {
    const int l = n0 + i;
    if (l < p.L) {
      const float yv = p.y[(int64_t)b * p.L + l];
      my_soft |= !(yv == 0.0f || yv == 1.0f);
    }
  }
  return __builtin_amdgcn_readfirstlane(__syncthreads_or(my_soft)) != 0;
}

// The transposed 3xf16 tile with an even sample split (launch_fwd: 96 labels x
// 128 samples for 48 < L <= 96: 8 waves of 48 labels x 32 samples), 2-stage
// ring.  The waves of the second half issue the stage DMA at static priority 1
// (the other half starts its MFMAs at the barrier).
// LDS_MIN: the LDS size at least (one workgroup per CU whatever the register
// count: packed fp32 VALU beside another workgroup's waves is not used, see
// MPV_NO_PK_FP32).
template <int WL, int WS, int TL, int TS, int NSTAGE, int LDS_MIN = 0>
__global__ __launch_bounds__(WL* WS * 64, 8 / (WL * WS)) void probit_fwd16t_kernel(FwdParams p) {
  constexpr int NW = WL * WS;
  constexpr int BM = WS * TS * 16, BN = WL * TL * 16;  // samples, labels
  constexpr int STAGE = (BM + BN) * kRowB;
  constexpr int RED = WL * BM * 6, CACC = WS * BN * 2;  // floats
  constexpr int LDS = NSTAGE * STAGE + (RED + CACC + kColsT * BN) * 4;
  __shared__ __attribute__((aligned(1024))) char smem[LDS > LDS_MIN ? LDS : LDS_MIN];
  float* red = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  float* cacc = red + RED;
  float* cols = cacc + CACC;

  int g, nt;
  decode_block(blockIdx.x, p.B * p.nSc, p.nNt, g, nt);
  const int b = g / p.nSc, sc = g % p.nSc;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wl = wid % WL, ws = wid / WL;
  const int lr = lane & 15, lg = lane >> 4;

  const float scale = 1.0f / (*p.eps16.scale * *p.R16.scale);
  const int nK = (p.z + kKC - 1) / kKC;
  const int sw = (lr >> 1) & 7;
  const int coh = (lg ^ sw) << 4, col = ((4 + lg) ^ sw) << 4;
  const int t_begin = sc * p.tps, t_end = min(p.nSt, (sc + 1) * p.tps);

  fwd_cols_stage_t<BN>(cols, p, b, n0, NW * 64);
  for (int i = tid; i < CACC; i += NW * 64) cacc[i] = 0.0f;
  const bool soft_any = fwd_tile_soft<BN>(p, b, n0, NW * 64);
  constexpr int NWD = NW / 2;  // DMA-issuing waves: the prio-1 half
  const bool dmaw = wid >= NW / 2;
  Fwd16Dma<BM, BN, NWD> dma;
  dma.init(p, t_begin, b, n0, wid % NWD, lane);
  if (dmaw) {
#pragma unroll
    for (int j = 0; j < NSTAGE - 1; ++j) dma.issue(p, smem + j * STAGE, t_end, nK, b);
  }

  int gs = 0;
  // the second half of the waves loses every age arbitration on its SIMD;
  // static priority (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  for (int st = t_begin; st < t_end; ++st) {
    const int s0 = fwd_tile_s0<BM>(st, p.S);
    f32x4 acc[TL][TS];
#pragma unroll
    for (int m = 0; m < TL; ++m)
#pragma unroll
      for (int n = 0; n < TS; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kc = 0; kc < nK; ++kc, ++gs) {
      if (NSTAGE == 2)
        wait_vmcnt<0>();
      else
        wait_vmcnt_dyn(min(dma.issued - (gs + 1), NSTAGE - 2) * dma.per_wave());
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_raw();  // stage gs landed for every wave; every wave is done reading gs-1
      FragT<TL, TS> f;
      if (dmaw) dma.issue(p, smem + ((gs + NSTAGE - 1) % NSTAGE) * STAGE, t_end, nK, b);
      fwd16t_read<WL, TL, TS, BM>(f, smem + (gs % NSTAGE) * STAGE, wl, ws * TS, lr, coh, col);
      fwd16t_mfma<TL, TS>(acc, f);
    }
    __builtin_amdgcn_s_setprio(0);
    fwd_tile_epilogue_t<WL, WS, TL, TS>(p, acc, scale, b, s0, st * BM, nt, red, cacc, cols,
                                        soft_any);
    // back to the K-loop priorities
    if (wid >= NW / 2)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
  }
  fwd16t_colpart<WS, BN>(p, cacc, b, sc, n0, NW * 64);
}

// ------------------------- 3xf16, asymmetric sample split (probit_fwd16a)
// The transposed 3xf16 tile for L > 48: (TL * 64) labels x 128 samples, 8
// waves (4 label groups x 2 sample groups), 2-stage LDS-DMA ring, one
// workgroup per CU.  The 128 samples are split unevenly between the two waves
// of each SIMD: waves 0-3 own TSA 16-sample blocks, waves 4-7 TSB (< TSA) and
// stream every stage's DMA at static priority 1.  With an even split the DMA half
// runs its 48 MFMAs after ~800 cycles of DMA issue while the other half is
// already done and waits at the barrier; here the DMA half has less MFMA
// work, so its DMA issue hides under the other half's longer MFMA phase.
// IS_A: waves 0-3 (TSA blocks); else waves 4-7 (TSB blocks, DMA).
template <int TSW, bool IS_A, int TSA, int TSB, int TL>
MPV_DEV void fwd16a_tiles(const FwdParams& p, char* smem, float* red, float* cacc,
                          const float* cols, Fwd16Dma<128, TL * 64, 4>& dma, bool dmaw, int b, int nt,
                          int t_begin, int t_end, int nK, bool soft_any, int wl, int sbo, int lr,
                          int coh, int col, float scale, bool prio1) {
  constexpr int WL = 4, BM = 128, NSTAGE = 2;
  constexpr int STAGE = (BM + TL * 64) * kRowB;
  int gs = 0;
  for (int st = t_begin; st < t_end; ++st) {
    const int s0 = fwd_tile_s0<BM>(st, p.S);
    f32x4 acc[TL][TSW];
#pragma unroll
    for (int m = 0; m < TL; ++m)
#pragma unroll
      for (int n = 0; n < TSW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < nK; ++kc, ++gs) {
      wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_raw();  // stage gs landed for every wave; every wave is done reading gs-1
      if (dmaw) {
        dma.issue(p, smem + ((__builtin_amdgcn_readfirstlane(gs) + NSTAGE - 1) % NSTAGE) * STAGE,
                  t_end, nK, b);
      }
      FragT<TL, TSW> f;
      fwd16t_read<WL, TL, TSW, BM>(f, smem + (gs % NSTAGE) * STAGE, wl, sbo, lr, coh, col);
      fwd16t_mfma<TL, TSW>(acc, f);
    }
    __builtin_amdgcn_s_setprio(0);
    fwd_tile_epilogue_t<WL, 2, TL, TSW, BM>(p, acc, scale, b, s0, st * BM, nt, red, cacc, cols,
                                            soft_any, sbo);
    if (prio1)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
  }
}

template <int TSA, int TSB, int TL>
__global__ __launch_bounds__(512, 1) void probit_fwd16a_kernel(FwdParams p) {
  constexpr int WL = 4, WS = 2, NW = 8, NSTAGE = 2;
  constexpr int BM = (TSA + TSB) * 16, BN = WL * TL * 16;
  static_assert(BM == 128, "the sample tile stays 128");
  constexpr int STAGE = (BM + BN) * kRowB;
  constexpr int RED = WL * BM * 6, CACC = WS * BN * 2;  // floats
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE + (RED + CACC + kColsT * BN) * 4];
  float* red = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  float* cacc = red + RED;
  float* cols = cacc + CACC;

  int g, nt;
  decode_block(blockIdx.x, p.B * p.nSc, p.nNt, g, nt);
  const int b = g / p.nSc, sc = g % p.nSc;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wl = wid % WL;
  const int lr = lane & 15, lg = lane >> 4;
  const float scale = 1.0f / (*p.eps16.scale * *p.R16.scale);
  const int nK = (p.z + kKC - 1) / kKC;
  const int sw = (lr >> 1) & 7;
  const int coh = (lg ^ sw) << 4, col = ((4 + lg) ^ sw) << 4;
  const int t_begin = sc * p.tps, t_end = min(p.nSt, (sc + 1) * p.tps);

  fwd_cols_stage_t<BN>(cols, p, b, n0, NW * 64);
  for (int i = tid; i < CACC; i += NW * 64) cacc[i] = 0.0f;
  const bool soft_any = fwd_tile_soft<BN>(p, b, n0, NW * 64);
  const bool dmaw = wid >= NW / 2;  // the TSB half streams the stages
  Fwd16Dma<BM, BN, NW / 2> dma;
  dma.init(p, t_begin, b, n0, wid % (NW / 2), lane);
  if (dmaw) {
#pragma unroll
    for (int j = 0; j < NSTAGE - 1; ++j) dma.issue(p, smem + j * STAGE, t_end, nK, b);
  }
  // the second half of the waves loses every age arbitration on its SIMD;
  // static priority (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  const bool prio1 = dmaw;
  if (prio1) __builtin_amdgcn_s_setprio(1);
  if (wid < NW / 2)
    fwd16a_tiles<TSA, true, TSA, TSB, TL>(p, smem, red, cacc, cols, dma, false, b, nt, t_begin, t_end,
                                      nK, soft_any, wl, 0, lr, coh, col, scale, prio1);
  else
    fwd16a_tiles<TSB, false, TSA, TSB, TL>(p, smem, red, cacc, cols, dma, true, b, nt, t_begin, t_end,
                                       nK, soft_any, wl, TSA, lr, coh, col, scale, prio1);
  fwd16t_colpart<WS, BN>(p, cacc, b, sc, n0, NW * 64);
}

// ------------- 3xf16, 256 labels x 256 samples (probit_fwd16b, the C4/C5 tile)
// probit_fwd16a with twice the samples per tile (dispatched for L > 128 and
// S >= 256; C4 forward 13.6 -> 12.5 ms, round 6): the stage image streams
// (256 + 256) rows for 256 x 256 x 32 products instead of (256 + 128) for
// 256 x 128 x 32 (a third fewer operand bytes per product), and each wave's
// fragment reads cover 64 x TS*16 products.  The accumulators (TL x TSW
// blocks) leave room for all R fragments of a stage but not all eps ones, so
// the eps fragments of one 16-sample block are read right before its
// products (one block ahead).  The row-statistics exchange (red, 24 KB)
// lives in the stage image the tile's last K stage was read from; the
// epilogue runs in parts of kFwdBPart sample blocks.
//
// Fwd16Dma for S >= BM (no row clamp): the pieces of one operand image are
// 32 rows apart, and (r >> 1) & 7 repeats every 16 rows, so every piece of an
// image has the same per-lane offset from its (wave-uniform) row base -- two
// offset VGPRs instead of JA + JB.
template <int BM, int BN, int NW>
struct Fwd16DmaLin {
  static constexpr int GA = BM / 8, GB = BN / 8;
  static constexpr int JA = GA / NW, JB = GB / NW;
  static_assert(GA % NW == 0 && GB % NW == 0, "pieces split evenly over the DMA waves");
  const char* a_base;  // eps rows of the current tile, this wave's first piece
  const char* b_base;  // R rows of the label tile, this wave's first piece
  int64_t a_step, b_step;  // bytes between a wave's consecutive pieces (NW * 8 rows)
  uint32_t offa, offb;
  int tile, kc, issued, wid;

  MPV_DEV void init(const FwdParams& p, int t0, int b, int n0, int wid_, int lane) {
    wid = wid_;
    const int64_t lda = p.eps16.ld, ldb = p.R16.ld;
    const int prow = lane >> 3, u_lds = lane & 7;
    a_step = (int64_t)NW * 8 * lda * 2;
    b_step = (int64_t)NW * 8 * ldb * 2;
    b_base = reinterpret_cast<const char*>(p.R16.data + ((int64_t)n0 + wid * 8) * ldb);
    offa = (uint32_t)(prow * lda * 2) + (uint32_t)((u_lds ^ (((wid * 8 + prow) >> 1) & 7)) * 16);
    offb = (uint32_t)(prow * ldb * 2) + (uint32_t)((u_lds ^ (((wid * 8 + prow) >> 1) & 7)) * 16);
    tile = t0;
    kc = 0;
    issued = 0;
    set_tile(p, b);
  }
  MPV_DEV void set_tile(const FwdParams& p, int b) {
    const int64_t o = ((int64_t)b * p.S + fwd_tile_s0<BM>(tile, p.S) + wid * 8) * p.eps16.ld;
    a_base = reinterpret_cast<const char*>(p.eps16.data + o);
  }
  MPV_DEV void issue(const FwdParams& p, char* dst, int tile_end, int nK, int b) {
    if (tile >= tile_end) return;
    const int kb = kc * kRowB;
#pragma unroll
    for (int j = 0; j < JA; ++j)
      lds_dma16(a_base + kb + j * a_step, offa, lds_addr(dst + (wid + j * NW) * 1024));
#pragma unroll
    for (int j = 0; j < JB; ++j)
      lds_dma16(b_base + kb + j * b_step, offb, lds_addr(dst + BM * kRowB + (wid + j * NW) * 1024));
    ++issued;
    if (++kc == nK) {
      kc = 0;
      if (++tile < tile_end) set_tile(p, b);
    }
  }
};

template <int TSW, int TL>
MPV_DEV void fwd16b_stage(f32x4 (&acc)[TL][TSW], const char* base, int wl, int sbo, int lr, int coh,
                          int col) {
  constexpr int BM = 256;
  s16x8 rh[TL], rl[TL];
#pragma unroll
  for (int m = 0; m < TL; ++m) {
    const int off = (BM + (wl * TL + m) * 16 + lr) * kRowB;
    rh[m] = *reinterpret_cast<const s16x8*>(base + off + coh);
    rl[m] = *reinterpret_cast<const s16x8*>(base + off + col);
  }
  s16x8 eh = *reinterpret_cast<const s16x8*>(base + (sbo * 16 + lr) * kRowB + coh);
  s16x8 el = *reinterpret_cast<const s16x8*>(base + (sbo * 16 + lr) * kRowB + col);
#pragma unroll
  for (int n = 0; n < TSW; ++n) {
    s16x8 eh2, el2;
    if (n + 1 < TSW) {  // the next block's fragments, in flight under these MFMAs
      const int off = ((sbo + n + 1) * 16 + lr) * kRowB;
      eh2 = *reinterpret_cast<const s16x8*>(base + off + coh);
      el2 = *reinterpret_cast<const s16x8*>(base + off + col);
    }
#pragma unroll
    for (int m = 0; m < TL; ++m)
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(rh[m]), as_f16x8(eh), acc[m][n], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < TL; ++m)
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(rh[m]), as_f16x8(el), acc[m][n], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < TL; ++m)
      acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(rl[m]), as_f16x8(eh), acc[m][n], 0, 0, 0);
    if (n + 1 < TSW) {
      eh = eh2;
      el = el2;
    }
  }
}

template <int PART, int NP, int TL, int TSW, int BM>
MPV_DEV void fwd16b_epilogue_parts(const FwdParams& p, f32x4 (&acc)[TL][TSW], float scale, int b, int s0,
                                   int s_own, int nt, float* red, float* cacc, const float* cols,
                                   bool soft_any, int sbo) {
  constexpr int H0 = TSW / NP, H = PART + 1 < NP ? H0 : TSW - (NP - 1) * H0;  // the last takes the rest
  static_assert(H0 >= 1, "a block per part at least");
  f32x4 a[TL][H];
#pragma unroll
  for (int m = 0; m < TL; ++m)
#pragma unroll
    for (int n = 0; n < H; ++n) a[m][n] = acc[m][PART * H0 + n];
  fwd_tile_epilogue_t<4, 2, TL, H, BM, PART == 0, kFwdBEpi, kFwdBUnroll, PART == NP - 1, kFwdBCQ>(
      p, a, scale, b, s0, s_own, nt, red, cacc, cols, soft_any, sbo + PART * H0);
  if constexpr (PART + 1 < NP)
    fwd16b_epilogue_parts<PART + 1, NP, TL, TSW, BM>(p, acc, scale, b, s0, s_own, nt, red, cacc, cols,
                                                     soft_any, sbo);
}

template <int TSW, int TSA, int TSB, int TL>
MPV_DEV void fwd16b_tiles(const FwdParams& p, char* smem, float* cacc, const float* cols,
                          Fwd16DmaLin<256, TL * 64, 4>& dma, bool dmaw, int b, int nt, int t_begin,
                          int t_end, int nK, bool soft_any, int wl, int sbo, int lr, int coh, int col,
                          float scale, bool prio1) {
  constexpr int BM = 256, NSTAGE = 2;
  constexpr int STAGE = (BM + TL * 64) * kRowB;
  int gs = 0;
  for (int st = t_begin; st < t_end; ++st) {
    const int s0 = fwd_tile_s0<BM>(st, p.S);
    f32x4 acc[TL][TSW];
#pragma unroll
    for (int m = 0; m < TL; ++m)
#pragma unroll
      for (int n = 0; n < TSW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < nK; ++kc, ++gs) {
      wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_raw();  // stage gs landed for every wave; every wave is done reading gs-1
      if (dmaw) {
        dma.issue(p, smem + ((__builtin_amdgcn_readfirstlane(gs) + NSTAGE - 1) % NSTAGE) * STAGE,
                  t_end, nK, b);
      }
      fwd16b_stage<TSW, TL>(acc, smem + (gs % NSTAGE) * STAGE, wl, sbo, lr, coh, col);
    }
    __builtin_amdgcn_s_setprio(0);
    // the image of stage gs-1 (read last) is free until the next tile's first
    // barrier; stage gs streams into the other one meanwhile
    float* red = reinterpret_cast<float*>(smem + ((gs + NSTAGE - 1) % NSTAGE) * STAGE);
    // in parts of kFwdBPart sample blocks (the row statistics of
    // one part in registers at a time)
    fwd16b_epilogue_parts<0, (TSW / kFwdBPart > 0 ? TSW / kFwdBPart : 1), TL, TSW, BM>(p, acc, scale, b, s0, st * BM, nt, red, cacc,
                                                      cols, soft_any, sbo);
    if (prio1)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
  }
}

template <int TSA, int TSB, int TL>
__global__ __launch_bounds__(512, 1) void probit_fwd16b_kernel(FwdParams p) {
  constexpr int WL = 4, WS = 2, NW = 8, NSTAGE = 2;
  constexpr int BM = (TSA + TSB) * 16, BN = WL * TL * 16;
  static_assert(BM == 256, "the sample tile is 256");
  constexpr int STAGE = (BM + BN) * kRowB;
  static_assert(WL * BM * 6 * 4 <= STAGE, "red fits one stage image");
  constexpr int CACC = WS * kFwdBCQ * BN * 2;  // floats
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE + (CACC + kColsT * BN) * 4];
  float* cacc = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  float* cols = cacc + CACC;

  int g, nt;
  decode_block(blockIdx.x, p.B * p.nSc, p.nNt, g, nt);
  const int b = g / p.nSc, sc = g % p.nSc;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wl = wid % WL;
  const int lr = lane & 15, lg = lane >> 4;
  const float scale = 1.0f / (*p.eps16.scale * *p.R16.scale);
  const int nK = (p.z + kKC - 1) / kKC;
  const int sw = (lr >> 1) & 7;
  const int coh = (lg ^ sw) << 4, col = ((4 + lg) ^ sw) << 4;
  const int t_begin = sc * p.tps, t_end = min(p.nSt, (sc + 1) * p.tps);

  fwd_cols_stage_t<BN>(cols, p, b, n0, NW * 64);
  for (int i = tid; i < CACC; i += NW * 64) cacc[i] = 0.0f;
  const bool soft_any = fwd_tile_soft<BN>(p, b, n0, NW * 64);
  const bool dmaw = wid >= NW / 2;  // the TSB half streams the stages
  Fwd16DmaLin<BM, BN, NW / 2> dma;
  dma.init(p, t_begin, b, n0, wid % (NW / 2), lane);
  if (dmaw) {
#pragma unroll
    for (int j = 0; j < NSTAGE - 1; ++j) dma.issue(p, smem + j * STAGE, t_end, nK, b);
  }
  const bool prio1 = dmaw;
  if (prio1) __builtin_amdgcn_s_setprio(1);
  if (wid < NW / 2)
    fwd16b_tiles<TSA, TSA, TSB, TL>(p, smem, cacc, cols, dma, false, b, nt, t_begin, t_end, nK,
                                    soft_any, wl, 0, lr, coh, col, scale, prio1);
  else
    fwd16b_tiles<TSB, TSA, TSB, TL>(p, smem, cacc, cols, dma, true, b, nt, t_begin, t_end, nK,
                                    soft_any, wl, TSA, lr, coh, col, scale, prio1);
  fwd16t_colpart<WS, BN, kFwdBCQ>(p, cacc, b, sc, n0, NW * 64);
}

// The six scalars of compute_loss (mpvae.py:147-148 KL, :188-190 nll, :122
// ranking mean, :207-208 total) from the per-row statistics, by ONE block of
// kFinalThreads threads.  row(b, v) yields row b's (M, Z, M_x, Z_x, c, c_x);
// both finalize variants sum in this same order.
#ifndef MPV_FINAL_THREADS
#define MPV_FINAL_THREADS 1024
#endif
constexpr int kFinalThreads = MPV_FINAL_THREADS;
template <class Row>
MPV_DEV void finalize_scalars(const mpv_final_args& a, int B, float S_total, Row row) {
  __shared__ float red[16 * 5];
  const int tid = threadIdx.x;
  float ne = 0.f, nx = 0.f, ce = 0.f, cx = 0.f;
  for (int b = tid; b < B; b += blockDim.x) {
    float v[6];
    row(b, v);
    // nll = mean_b(-log(mean_s exp(logp - max)) - max)   (mpvae.py:188-190)
    ne += -logf(v[1] / S_total) - v[0];
    nx += -logf(v[3] / S_total) - v[2];
    ce += v[4];
    cx += v[5];
  }
  float kl = 0.f;
  const int64_t nd = (int64_t)B * a.d;
  auto klt = [](float lve, float lvx, float mue, float mux) {
    const float dm = mux - mue;
    return (lvx - lve) - 1.0f + expf(lve - lvx) + dm * dm / (expf(lvx) + kKlEps);
  };
  const bool vec = (nd & 3) == 0 &&
                   ((reinterpret_cast<uintptr_t>(a.fe_logvar) | reinterpret_cast<uintptr_t>(a.fx_logvar) |
                     reinterpret_cast<uintptr_t>(a.fe_mu) | reinterpret_cast<uintptr_t>(a.fx_mu)) & 15) == 0;
  if (vec) {  // four elements per thread and pass, 16-B loads (one block does all of B x d:
              // the scalar loop's dependent loads made this launch 20 us at C4)
    for (int64_t i = 4 * (int64_t)tid; i < nd; i += 4 * (int64_t)blockDim.x) {
      const f32x4 le = *reinterpret_cast<const f32x4*>(a.fe_logvar + i);
      const f32x4 lx = *reinterpret_cast<const f32x4*>(a.fx_logvar + i);
      const f32x4 me = *reinterpret_cast<const f32x4*>(a.fe_mu + i);
      const f32x4 mx = *reinterpret_cast<const f32x4*>(a.fx_mu + i);
#pragma unroll
      for (int q = 0; q < 4; ++q) kl += klt(le[q], lx[q], me[q], mx[q]);
    }
  } else {
#pragma unroll 4
    for (int64_t i = tid; i < nd; i += blockDim.x)
      kl += klt(a.fe_logvar[i], a.fx_logvar[i], a.fe_mu[i], a.fx_mu[i]);
  }
  float r5[5] = {ne, nx, ce, cx, kl};
  block_reduce_n<5, false>(r5, red);  // one barrier pair; each value as block_reduce sums it
  ne = r5[0], nx = r5[1], ce = r5[2], cx = r5[3], kl = r5[4];
  if (tid == 0) {
    const float nll = ne / (float)B, nll_x = nx / (float)B;
    const float c = ce / (S_total * (float)B), c_x = cx / (S_total * (float)B);
    const float klv = 0.5f * kl / (float)B;
    *a.nll = nll;
    *a.nll_x = nll_x;
    *a.c = c;
    *a.c_x = c_x;
    *a.kl = klv;
    // total (mpvae.py:207-208)
    *a.total = (nll + nll_x) * a.nll_coeff + (c + c_x) * a.c_coeff + klv * kKlWeight;
  }
}

// indiv_prob_label / indiv_prob (mpvae.py:203-204) of element i = b L + l
MPV_DEV void write_indiv(const mpv_final_args& a, int64_t n, int64_t i, float e, float x,
                         float S_total) {
  a.indiv_prob_label[i] = e / S_total;
  a.indiv_prob[i] = x / S_total;
  (void)n;
}

// One block per batch row b.  rowpart -> rowstat, bstat.
// (Round 6 measured the finalize folded into this kernel's last-arriving
// block: the device-scope release fence each block then needs writes back its
// XCD's L2, and the combine ran 13 -> 53 us at C2, 77 -> 270 us at C4.)
__global__ __launch_bounds__(kCombineThreads) void fwd_combine_kernel(const float* __restrict__ y,
                                                         const float* __restrict__ rowpart,
                                                         float* __restrict__ rowstat,
                                                         float* __restrict__ bstat, int S, int B,
                                                         int L, int nNt,
                                                         const float* __restrict__ colpart,
                                                         float* __restrict__ colsum, int nSc) {
  __shared__ float red[32], red2[32];
  const int b = blockIdx.x, tid = threadIdx.x;
  // this row's column sums over the s-chunks (colpart != NULL: the workgroups
  // of several s-chunks wrote partials), summed in chunk order
  if (colpart != nullptr) {
    const int64_t n = 2 * (int64_t)B * L;
    for (int i = tid; i < 2 * L; i += blockDim.x) {
      const int k = i / L, l = i - k * L;
      const int64_t o = ((int64_t)k * B + b) * L + l;
      float acc = 0.0f;
      for (int sc = 0; sc < nSc; ++sc) acc += colpart[sc * n + o];
      colsum[o] = acc;
    }
  }
  float np = 0.f, nn = 0.f;
  for (int l = tid; l < L; l += blockDim.x) {
    const float v = y[(int64_t)b * L + l];
    np += (v == 1.0f) ? 1.0f : 0.0f;
    nn += (v == 0.0f) ? 1.0f : 0.0f;
  }
  block_reduce2<false>(np, nn, red);
  const float nrm = np * nn;  // normalizers = |pos| * |neg|  (mpvae.py:115-117)

  float me = -INFINITY, mx = -INFINITY, ce = 0.f, cx = 0.f;
  // the row's first kCombineKeep passes of log-probs stay in registers for the
  // log-sum-exp pass (no second read of rowstat for S <= kCombineKeep * 1024)
  float keep0[kCombineKeep], keep1[kCombineKeep];
  auto sample = [&](int s, float& l0, float& l1) {
    float v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      float a = 0.f;
      for (int nt = 0; nt < nNt; ++nt) a += rowpart[(((int64_t)k * nNt + nt) * B + b) * S + s];
      v[k] = a;
      rowstat[((int64_t)k * B + b) * S + s] = a;
    }
    me = fmaxf(me, v[0]);
    mx = fmaxf(mx, v[1]);
    // loss = sums / (5 * normalizers); inf/nan -> 0   (mpvae.py:118-121)
    const float le = (v[2] * v[3]) / (5.0f * nrm);
    const float lx = (v[4] * v[5]) / (5.0f * nrm);
    ce += isfinite(le) ? le : 0.0f;
    cx += isfinite(lx) ? lx : 0.0f;
    l0 = v[0];
    l1 = v[1];
  };
  // S % 4 == 0: the kept samples are four consecutive ones per thread, read
  // and written as 16-B vectors (rowpart is 200 MB per launch at C4)
  const bool vec = kCombineKeep == 4 && (S & 3) == 0;
  if (vec) {
    const int s0 = 4 * tid;
    if (s0 < S) {
      f32x4 v[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        f32x4 a{0.f, 0.f, 0.f, 0.f};
        for (int nt = 0; nt < nNt; ++nt)
          a += *reinterpret_cast<const f32x4*>(rowpart + (((int64_t)k * nNt + nt) * B + b) * S + s0);
        v[k] = a;
        *reinterpret_cast<f32x4*>(rowstat + ((int64_t)k * B + b) * S + s0) = a;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        me = fmaxf(me, v[0][j]);
        mx = fmaxf(mx, v[1][j]);
        const float le = (v[2][j] * v[3][j]) / (5.0f * nrm);
        const float lx = (v[4][j] * v[5][j]) / (5.0f * nrm);
        ce += isfinite(le) ? le : 0.0f;
        cx += isfinite(lx) ? lx : 0.0f;
        keep0[j] = v[0][j];
        keep1[j] = v[1][j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kCombineKeep; ++j) {
      const int s = tid + j * (int)blockDim.x;
      if (s < S) sample(s, keep0[j], keep1[j]);
    }
  }
  for (int s = tid + kCombineKeep * (int)blockDim.x; s < S; s += blockDim.x) {
    float l0, l1;
    sample(s, l0, l1);
  }
  {  // the two maxima and the two ranking sums with one barrier pair, each
     // combined in block_reduce's order
    const int lane = tid & 63, wid = tid >> 6, nw = (blockDim.x + 63) >> 6;
    me = wave_max(me);
    mx = wave_max(mx);
    ce = wave_sum(ce);
    cx = wave_sum(cx);
    __syncthreads();
    if (lane == 0) red[wid] = me, red[16 + wid] = mx, red2[wid] = ce, red2[16 + wid] = cx;
    __syncthreads();
    me = mx = -INFINITY;
    ce = cx = 0.0f;
    for (int i = 0; i < nw; ++i) {
      me = fmaxf(me, red[i]);
      mx = fmaxf(mx, red[16 + i]);
      ce += red2[i];
      cx += red2[16 + i];
    }
  }
  float ze = 0.f, zx = 0.f;
#pragma unroll
  for (int j = 0; j < kCombineKeep; ++j) {
    const int s = vec ? 4 * tid + j : tid + j * (int)blockDim.x;
    if (s < S) {
      ze += expf(keep0[j] - me);
      zx += expf(keep1[j] - mx);
    }
  }
  for (int s = tid + kCombineKeep * (int)blockDim.x; s < S; s += blockDim.x) {
    ze += expf(rowstat[((int64_t)0 * B + b) * S + s] - me);
    zx += expf(rowstat[((int64_t)1 * B + b) * S + s] - mx);
  }
  block_reduce2<false>(ze, zx, red);
  if (tid == 0) {
    bstat[0 * B + b] = me;
    bstat[1 * B + b] = ze;
    bstat[2 * B + b] = mx;
    bstat[3 * B + b] = zx;
    bstat[4 * B + b] = ce;
    bstat[5 * B + b] = cx;
  }
}

// Block 0: the six scalars; blocks >= 1: indiv_prob / indiv_prob_label.
// SLOTS (the sharded path): a.bstat is the all-reduced (nslots, 6, B) slot
// buffer of the shards' statistics; block 0 combines each row exactly
// (bstat_combine_row, as mpv_bstat_combine) into bstat_out for the backward
// and finalizes from the combined values: one launch instead of two.
template <bool SLOTS>
__global__ __launch_bounds__(kFinalThreads) void finalize_kernel(mpv_final_args a, int B, int L,
                                                               float S_total, int nslots,
                                                               float* __restrict__ bstat_out) {
  if (blockIdx.x > 0) {
    const int64_t n = (int64_t)B * L;
    for (int64_t i = (int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)(gridDim.x - 1) * blockDim.x)
      write_indiv(a, n, i, a.colsum[i], a.colsum[n + i], S_total);
    return;
  }
  // the step's noise has been drawn (stream order): advance its device key
  if (a.seed_advance != nullptr && threadIdx.x == 0) *a.seed_advance += 1ull;
  finalize_scalars(a, B, S_total, [&](int b, float (&v)[6]) {
    if (SLOTS) {
      bstat_combine_row(a.bstat, nslots, B, b, v);
#pragma unroll
      for (int k = 0; k < 6; ++k) bstat_out[(int64_t)k * B + b] = v[k];
    } else {
#pragma unroll
      for (int k = 0; k < 6; ++k) v[k] = a.bstat[(int64_t)k * B + b];
    }
  });
}

// ---------------------------------------------------------------- host side
struct FwdPlan {
  int cfg;  // tile configuration, see launch_fwd
  int BM, BN, nNt, nSt, nSc, tps;
  size_t rowpart_bytes, colpart_bytes;
};

static FwdPlan plan_fwd(const mpv_shape* s, int gemm) {
  FwdPlan pl;
  // tile configurations: 0 = 48 labels (L <= 48), 1 = 96 labels (fp32 mode,
  // L <= 96; 3xf16: the transposed 96 x 128 tile), 2 = 128 labels (transposed
  // 3xf16 tile, or the fp32 64 x 64 waves), 3 = 256 labels (3xf16, L > 128).
  // (Round 2 measured the 3xf16 96-label tile of probit_fwd16, MFMA-layout
  // accumulators, slower at C3 than the 128-label transposed tile; the
  // transposed 96-label tile is the one used now.)
  const bool f16 = gemm == MPV_GEMM_F16X3;
  pl.cfg = s->L <= 48 ? 0 : (s->L <= 96 ? 1 : ((f16 && s->L > 128) ? 3 : 2));
  // (the 256 x 256 tile streams whole tiles: S >= 256, Fwd16DmaLin.
  // MPVAE_FWD_TILE=256x128 selects round 5's tile instead: a diagnostic for
  // the tests that compare the two, not a tuning knob)
  const char* tile_env = std::getenv("MPVAE_FWD_TILE");
  const bool tile128 = tile_env != nullptr && std::strcmp(tile_env, "256x128") == 0;
  pl.BM = (f16 && pl.cfg == 0) ? kFwd48BM
                               : ((f16 && pl.cfg == 3 && kFwdB && !tile128 && s->S_local >= 256) ? 256
                                                                                                 : 128);
  pl.BN = pl.cfg == 0 ? 48 : (pl.cfg == 1 ? 96 : (pl.cfg == 2 ? 128 : 256));
  pl.nNt = (int)cdiv(s->L, pl.BN);
  pl.nSt = (int)cdiv(s->S_local, pl.BM);
  // 3xf16: s-chunks until the grid is one round of resident workgroups (one
  // per CU: every 3xf16 tile is 8 waves); longer runs per
  // workgroup amortize its prologue (C3 step 0.534 -> 0.510 ms against a
  // 2048-workgroup target, C2 the same; C4 has one s-chunk either way)
  const int64_t target = f16 ? (int64_t)num_cus() : kFwdWant;
  int64_t want = cdiv(target, s->B * (int64_t)pl.nNt);
  if (want < 1) want = 1;
  if (want > pl.nSt) want = pl.nSt;
  pl.tps = (int)cdiv(pl.nSt, want);
  pl.nSc = (int)cdiv(pl.nSt, pl.tps);
  pl.rowpart_bytes = align_up(sizeof(float) * 6 * (size_t)pl.nNt * s->B * s->S_local, 256);
  pl.colpart_bytes = pl.nSc > 1 ? align_up(sizeof(float) * (size_t)pl.nSc * 2 * s->B * s->L, 256) : 0;
  return pl;
}

static void launch_fwd(const FwdPlan& pl, int gemm, dim3 grid, hipStream_t st, const FwdParams& p) {
  if (gemm == MPV_GEMM_F32) {
    switch (pl.cfg) {
      case 0:
        MPV_LAUNCH("probit_fwd", (probit_fwd_kernel<4, 1, 2, 3>), grid, dim3(256), 0, st, p);
        break;
      case 1:
        MPV_LAUNCH("probit_fwd", (probit_fwd_kernel<4, 1, 2, 6>), grid, dim3(256), 0, st, p);
        break;
      default:
        MPV_LAUNCH("probit_fwd", (probit_fwd_kernel<2, 2, 4, 4>), grid, dim3(256), 0, st, p);
        break;
    }
  } else {
    switch (pl.cfg) {
      case 0:  // 48 labels x kFwd48BM samples, transposed, 8 waves, one workgroup per CU
        MPV_LAUNCH("probit_fwd", (probit_fwd16t_kernel<1, 8, 3, kFwd48BM / 128, 2, 82 * 1024>), grid,
                   dim3(512), 0, st, p);
        break;
      case 3:  // 256 labels x 128 samples, 8 waves, asymmetric 80 / 48 sample split
        if (pl.BM == 256)
          MPV_LAUNCH("probit_fwd", (probit_fwd16b_kernel<kFwdBA, 16 - kFwdBA, 4>), grid, dim3(512), 0, st, p);
        else
          MPV_LAUNCH("probit_fwd", (probit_fwd16a_kernel<5, 3, 4>), grid, dim3(512), 0, st, p);
        break;
      case 1:  // 96 labels x 128 samples (48 < L <= 96), 8 waves of 48 x 32, even split
        MPV_LAUNCH("probit_fwd", (probit_fwd16t_kernel<2, 4, 3, 2, 2>), grid, dim3(512), 0, st, p);
        break;
      default:
        // 128 labels x 128 samples (96 < L <= 128), 8 waves, asymmetric 80 / 48
        // sample split (C3 before the 96-label tile: forward 0.187 -> 0.181 ms
        // against the even 64 / 64 split).  A
        // 4-wave version of this tile (64 x 64 per wave, two workgroups per CU)
        // ran 0.031 ms faster at C3 but was not repeatable: 10-13 % of its
        // launches at C3 differed in one label-branch row statistic of a
        // 16-sample block (never with one workgroup per CU, the same code padded
        // to 81 KB of LDS; DESIGN.md section 4, tools/repeat_probe.py)
        MPV_LAUNCH("probit_fwd", (probit_fwd16a_kernel<5, 3, 2>), grid, dim3(512), 0, st, p);
        break;
    }
  }
}

static int check_split_operand(const mpv_split16& o, int64_t rows, int64_t ld_min,
                               const char* what) {
  MPV_REQUIRE(o.data && o.scale, "%s: NULL plane", what);
  MPV_REQUIRE(o.rows_pad >= rows, "%s: rows_pad %lld < %lld", what, (long long)o.rows_pad,
              (long long)rows);
  MPV_REQUIRE(o.ld >= ld_min && (o.ld % 64) == 0,
              "%s: ld %lld must be >= %lld and a multiple of 64", what, (long long)o.ld,
              (long long)ld_min);
  return MPV_OK;
}

}  // namespace mpv

using namespace mpv;

extern "C" {

size_t mpv_fwd_workspace_bytes(const mpv_shape* shape) {
  if (check_shape(shape) != MPV_OK) return 0;
  size_t most = 0;  // enough for either GEMM mode's tiling
  for (int gemm : {MPV_GEMM_F16X3, MPV_GEMM_F32}) {
    const FwdPlan pl = plan_fwd(shape, gemm);
    most = std::max(most, pl.rowpart_bytes + pl.colpart_bytes);
  }
  return most;
}

}  // extern "C"

namespace mpv {

static int check_final_args(const mpv_final_args* a, bool need_stats) {
  MPV_REQUIRE(a && (!need_stats || (a->bstat && a->colsum)) && a->fe_mu && a->fe_logvar &&
                  a->fx_mu && a->fx_logvar && a->total && a->nll && a->nll_x && a->c && a->c_x &&
                  a->kl && a->indiv_prob && a->indiv_prob_label && a->d > 0,
              "NULL pointer in mpv_final_args");
  return MPV_OK;
}

template <bool SLOTS>
static int launch_finalize(const mpv_shape* shape, const mpv_final_args& a, int nslots,
                           float* bstat_out, hipStream_t st) {
  const int64_t n = shape->B * shape->L;
  int64_t nb = cdiv(n, kFinalThreads);
  if (nb > 2048) nb = 2048;
  MPV_LAUNCH("finalize", finalize_kernel<SLOTS>, dim3((unsigned)(1 + nb)), dim3(kFinalThreads), 0,
             st, a, (int)shape->B, (int)shape->L, (float)shape->S_total, nslots, bstat_out);
  return check_launch("finalize");
}

static int run_fwd(const mpv_shape* shape, const mpv_fwd_args* a, void* stream) {
  if (int rc = check_shape(shape)) return rc;
  MPV_REQUIRE(a != nullptr, "args is NULL");
  MPV_REQUIRE(a->y && a->fe_out && a->fx_out && a->rowstat && a->bstat && a->colsum &&
                  a->workspace,
              "NULL pointer in mpv_fwd_args");
  MPV_REQUIRE(a->gemm == MPV_GEMM_F32 || a->gemm == MPV_GEMM_F16X3, "unknown gemm mode %d",
              a->gemm);
  const FwdPlan pl = plan_fwd(shape, a->gemm);
  if (a->gemm == MPV_GEMM_F32) {
    MPV_REQUIRE(a->R32 && a->eps, "MPV_GEMM_F32 needs R32 and eps");
  } else {
    const int64_t ldk = 2 * cdiv(shape->z, kKC) * kKC;  // K slices the main loop reads
    if (int rc = check_split_operand(a->R16, (int64_t)pl.nNt * pl.BN, ldk, "R16")) return rc;
    if (int rc = check_split_operand(a->eps16, shape->S_local * shape->B, ldk, "eps16")) return rc;
    // the DMA issue keeps per-lane byte offsets within one s/l tile in 32 bits
    MPV_REQUIRE((int64_t)pl.BM * a->eps16.ld * 2 < (int64_t(1) << 32) &&
                    (int64_t)pl.BN * a->R16.ld * 2 < (int64_t(1) << 32),
                "ld too large for the f16x3 tile offsets");
  }
  const size_t need = pl.rowpart_bytes + pl.colpart_bytes;
  MPV_REQUIRE(a->workspace_bytes >= need, "workspace too small: %zu < %zu", a->workspace_bytes,
              need);
  hipStream_t st = as_stream(stream);
  FwdParams p;
  p.y = a->y;
  p.fe = a->fe_out;
  p.fx = a->fx_out;
  p.R = a->R32;
  p.eps = a->eps;
  p.R16 = a->R16;
  p.eps16 = a->eps16;
  p.T = a->T;
  p.rowpart = reinterpret_cast<float*>(a->workspace);
  p.colpart = pl.nSc > 1 ? reinterpret_cast<float*>((char*)a->workspace + pl.rowpart_bytes)
                         : a->colsum;
  p.S = (int)shape->S_local;
  p.B = (int)shape->B;
  p.L = (int)shape->L;
  p.ldT = (int)t_cols(shape->L);
  p.z = (int)shape->z;
  p.nNt = pl.nNt;
  p.nSc = pl.nSc;
  p.tps = pl.tps;
  p.nSt = pl.nSt;
  const int64_t blocks = (int64_t)shape->B * pl.nSc * pl.nNt;
  MPV_REQUIRE(blocks < (int64_t(1) << 31), "grid too large");
  launch_fwd(pl, a->gemm, dim3((unsigned)blocks), st, p);
  if (int rc = check_launch("probit_fwd")) return rc;
  // few s-chunks: fwd_combine sums the column partials too (one launch less);
  // many (small B, long S): the slab-sum kernel's split reduction
  const bool fold = pl.nSc > 1 && pl.nSc <= kCombineFoldSlabs;
  MPV_LAUNCH("fwd_combine", fwd_combine_kernel, dim3((unsigned)shape->B), dim3(kCombineThreads), 0,
             st, a->y, p.rowpart, a->rowstat, a->bstat, p.S, p.B, p.L, pl.nNt,
             fold ? p.colpart : nullptr, a->colsum, pl.nSc);
  if (int rc = check_launch("fwd_combine")) return rc;
  if (pl.nSc > 1 && !fold) {
    if (int rc = launch_sum_slabs(p.colpart, pl.nSc, 2 * shape->B * shape->L, a->colsum, MPV_F32, st))
      return rc;
  }
  return MPV_OK;
}

}  // namespace mpv

extern "C" {

int mpv_probit_fwd(const mpv_shape* shape, const mpv_fwd_args* a, void* stream) {
  return run_fwd(shape, a, stream);
}

int mpv_probit_finalize(const mpv_shape* shape, const mpv_final_args* a, void* stream) {
  MPV_REQUIRE(shape && shape->B > 0 && shape->L > 0 && shape->S_total > 0, "bad shape");
  if (int rc = check_final_args(a, true)) return rc;
  return launch_finalize<false>(shape, *a, 0, nullptr, as_stream(stream));
}

int mpv_probit_finalize_shards(const mpv_shape* shape, const float* slots, int64_t nslots,
                               float* bstat_out, const mpv_final_args* a, void* stream) {
  MPV_REQUIRE(shape && shape->B > 0 && shape->L > 0 && shape->S_total > 0, "bad shape");
  MPV_REQUIRE(slots && bstat_out && nslots > 0 && nslots < (int64_t(1) << 20),
              "bad slot arguments");
  if (int rc = check_final_args(a, false)) return rc;
  MPV_REQUIRE(a->colsum != nullptr, "colsum is NULL");
  mpv_final_args f = *a;
  f.bstat = slots;  // (nslots, 6, B), combined row by row in the kernel
  return launch_finalize<true>(shape, f, (int)nslots, bstat_out, as_stream(stream));
}

}  // extern "C"
