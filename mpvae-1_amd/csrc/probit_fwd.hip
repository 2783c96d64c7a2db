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
  float* T;
  float* rowpart;  // [6][nNt][B][S]
  float* colpart;  // [nSc][2][B][L]
  int S, B, L, z;
  int nNt, nSc, tps, nSt;
};

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
  float fe[TN], fx[TN], y[TN], colE[TN], colEx[TN];
  int col[TN];
  bool colok[TN], soft[TN];
};

template <int WN, int TN>
MPV_DEV void fwd_lane_init(FwdLane<TN>& ln, const FwdParams& p, int b, int n0, int wn, int lr) {
#pragma unroll
  for (int n = 0; n < TN; ++n) {
    const int col = n0 + wn * TN * 16 + n * 16 + lr;
    ln.col[n] = col;
    ln.colok[n] = col < p.L;
    const int64_t o = (int64_t)b * p.L + (ln.colok[n] ? col : 0);
    ln.y[n] = ln.colok[n] ? p.y[o] : 0.0f;
    ln.fe[n] = ln.colok[n] ? p.fe[o] : 0.0f;
    ln.fx[n] = ln.colok[n] ? p.fx[o] : 0.0f;
    ln.soft[n] = !(ln.y[n] == 0.0f || ln.y[n] == 1.0f);
    ln.colE[n] = ln.colEx[n] = 0.0f;
  }
}

// One BM x BN tile of t (acc * scale): probit decode, row statistics written
// to rowpart[., nt, b, s], column sums accumulated in `ln`.  Called by every
// thread of the workgroup; uses `smem` (>= WN*BM*6 floats) after a barrier.
template <int WM, int WN, int TM, int TN>
MPV_DEV void fwd_tile_epilogue(const FwdParams& p, FwdLane<TN>& ln, f32x4 (&acc)[TM][TN],
                               float scale, int b, int s0, int nt, float* smem) {
  constexpr int NT = WM * WN * 64, BM = WM * TM * 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN, lr = lane & 15, lg = lane >> 4;
  const int S = p.S, B = p.B, L = p.L;
  float* red = smem;  // [WN][BM][6]
  __syncthreads();    // the main loop's last LDS reads are done before red is written
#pragma unroll
  for (int m = 0; m < TM; ++m) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = wm * TM * 16 + m * 16 + lg * 4 + i;
      const int s = s0 + rl;
      const bool rowok = s < S;
      float st6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const bool ok = rowok && ln.colok[n];
        const float t = acc[m][n][i] * scale;
        if (p.T != nullptr && ok) p.T[((int64_t)b * S + s) * L + ln.col[n]] = t;
        const float E = probit_prob(t + ln.fe[n]);
        const float Ex = probit_prob(t + ln.fx[n]);
        const float y = ln.y[n];
        // BCE log-prob (mpvae.py:184-185): one log for a 0/1 label
        float le = fast_log(y == 0.0f ? 1.0f - E : E);
        float lx = fast_log(y == 0.0f ? 1.0f - Ex : Ex);
        if (ln.soft[n]) {
          le = y * fast_log(E) + (1.0f - y) * fast_log(1.0f - E);
          lx = y * fast_log(Ex) + (1.0f - y) * fast_log(1.0f - Ex);
        }
        // ranking factors (mpvae.py:110-114 factorised): pos -> e^{-5E}, neg -> e^{5E}
        const float sg = (y == 1.0f) ? -5.0f : 5.0f;
        const float re = fast_exp(sg * E), rx = fast_exp(sg * Ex);
        const float wpos = (ok && y == 1.0f) ? 1.0f : 0.0f;
        const float wneg = (ok && y == 0.0f) ? 1.0f : 0.0f;
        st6[0] += ok ? le : 0.0f;
        st6[1] += ok ? lx : 0.0f;
        st6[2] += wpos * re;
        st6[3] += wneg * re;
        st6[4] += wpos * rx;
        st6[5] += wneg * rx;
        ln.colE[n] += rowok ? E : 0.0f;
        ln.colEx[n] += rowok ? Ex : 0.0f;
      }
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
  __syncthreads();
  for (int r = tid; r < BM; r += NT) {
    const int s = s0 + r;
    if (s < S) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < WN; ++w) v += red[(w * BM + r) * 6 + k];
        p.rowpart[(((int64_t)k * p.nNt + nt) * B + b) * S + s] = v;
      }
    }
  }
  __syncthreads();
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
    float e = ln.colE[n], x = ln.colEx[n];
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
template <int WM, int WN, int TM, int TN>
__global__ __launch_bounds__(WM* WN * 64) void probit_fwd_kernel(FwdParams p) {
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
  fwd_lane_init<WN, TN>(ln, p, b, n0, wn, lr);

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
    fwd_tile_epilogue<WM, WN, TM, TN>(p, ln, acc, 1.0f, b, s0, nt, smem);
  }
  fwd_colsum_epilogue<WM, WN, TM, TN>(p, ln, b, sc, n0, smem);
}

// ------------------------------------------------------ 3xf16 mainloop
// The K axis (z) is streamed in stages of 32 halves (one MFMA k-step) through a
// ring of NSTAGE LDS buffers filled by LDS-DMA (global_load_lds_dwordx4), with
// NSTAGE-1 stages in flight and one barrier per stage.  Stage image:
// [A_hi | A_lo | B_hi | B_lo], each row 64 B; the 16-B chunk c of row r sits at
// position c ^ ((r >> 1) & 3), which makes the ds_read_b128 fragment reads
// (16 rows x one 16-B column per lane group) hit 16 distinct slots of the
// 256-B bank row (exhaustively checked).  LDS-DMA writes
// lane-linearly, so the swizzle goes on the per-lane SOURCE address and the
// same XOR is applied on the read.
constexpr int kKC = 32;    // K halves per stage
constexpr int kRowB = 64;  // bytes per plane row per stage

// One K stage (k0 halves in) of this wave's DMA groups into stage image `dst`.
// A device function rather than a lambda: hipcc drops the host stub of a
// template kernel whose lambda captures arrays.
template <int GMAX, int GROUPS, int NW>
MPV_DEV void fwd16_issue(char* dst, int k0, int wid, const char* const (&gbase)[GMAX],
                         const uint32_t (&goff)[GMAX]) {
#pragma unroll
  for (int i = 0; i < GMAX; ++i) {
    const int grp = wid + i * NW;
    if (GROUPS % NW != 0 && grp >= GROUPS) break;
    __builtin_amdgcn_global_load_lds(gbase[i] + 2 * k0 + goff[i],
                                     (__attribute__((address_space(3))) void*)(dst + grp * 1024),
                                     16, 0, 0);
  }
}

template <int WM, int WN, int TM, int TN, int NSTAGE>
__global__ __launch_bounds__(WM* WN * 64, (WM * WN <= 4) ? 2 : 1) void probit_fwd16_kernel(FwdParams p) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
  constexpr int PLANE_A = BM * kRowB, PLANE_B = BN * kRowB;
  constexpr int STAGE = 2 * PLANE_A + 2 * PLANE_B;
  static_assert(STAGE % 1024 == 0, "stage must be whole 1-KB DMA groups");
  constexpr int GROUPS = STAGE / 1024;  // 16 rows each
  constexpr int GMAX = (GROUPS + NW - 1) / NW;
  constexpr int P = NSTAGE - 1;         // stages in flight
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE];

  int g, nt;
  decode_block(blockIdx.x, p.B * p.nSc, p.nNt, g, nt);
  const int b = g / p.nSc, sc = g % p.nSc;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int S = p.S, B = p.B;
  const int64_t lda = p.eps16.ld, ldb = p.R16.ld;

  FwdLane<TN> ln;
  fwd_lane_init<WN, TN>(ln, p, b, n0, wn, lr);
  const float scale = 1.0f / (*p.eps16.scale * *p.R16.scale);
  const int nK = (p.z + kKC - 1) / kKC;
  const int coff = (lg ^ ((lr >> 1) & 3)) << 4;  // swizzled 16-B column of this lane's reads
  const int my_groups = (GROUPS - wid + NW - 1) / NW;
  const int dma_row = lane >> 2, dma_pos = lane & 3;

  const int st_end = min(p.nSt, (sc + 1) * p.tps);
  for (int st = sc * p.tps; st < st_end; ++st) {
    const int s0 = st * BM;
    // DMA sources of this wave's groups (wid, wid+NW, ... of 16 rows; a group
    // never straddles planes): a wave-uniform 64-bit plane/tile base plus a
    // 32-bit per-lane byte offset (row within the tile, swizzled chunk), so
    // the loop carries one VGPR per group and issues the saddr form.
    const char* gbase[GMAX];
    uint32_t goff[GMAX];
#pragma unroll
    for (int i = 0; i < GMAX; ++i) {
      const int grp = min(wid + i * NW, GROUPS - 1);
      const int row0 = grp * 16;  // wave-uniform first row of the group
      const int r16 = dma_row;
      int r;
      if (row0 < 2 * BM) {
        const int plane = row0 >= BM;
        const int rb = row0 - plane * BM;  // uniform
        r = rb + r16;
        const int s = min(s0 + r, S - 1);
        gbase[i] = reinterpret_cast<const char*>((plane ? p.eps16.lo : p.eps16.hi) +
                                                 ((int64_t)s0 * B + b) * lda);
        goff[i] = (uint32_t)((int64_t)(s - s0) * B * lda * 2);
      } else {
        const int plane = row0 >= 2 * BM + BN;
        const int rb = row0 - 2 * BM - plane * BN;
        r = rb + r16;
        gbase[i] = reinterpret_cast<const char*>((plane ? p.R16.lo : p.R16.hi) +
                                                 (int64_t)n0 * ldb);
        goff[i] = (uint32_t)(r * ldb * 2);
      }
      goff[i] += (uint32_t)((dma_pos ^ ((r >> 1) & 3)) * 16);
    }

    f32x4 acc[TM][TN];
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int j = 0; j < P && j < nK; ++j) fwd16_issue<GMAX, GROUPS, NW>(smem + j * STAGE, j * kKC, wid, gbase, goff);
    for (int kc = 0; kc < nK; ++kc) {
      // stages issued after kc may stay in flight; kc itself must have landed
      wait_vmcnt_dyn(min(P - 1, nK - 1 - kc) * my_groups);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier_raw();  // kc landed for every wave; every wave is done reading kc-1
      if (kc + P < nK) fwd16_issue<GMAX, GROUPS, NW>(smem + ((kc + P) % NSTAGE) * STAGE, (kc + P) * kKC, wid,
                                                gbase, goff);
      const char* base = smem + (kc % NSTAGE) * STAGE;
      s16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int m = 0; m < TM; ++m) {
        const int off = ((wm * TM + m) * 16 + lr) * kRowB + coff;
        ah[m] = *reinterpret_cast<const s16x8*>(base + off);
        al[m] = *reinterpret_cast<const s16x8*>(base + PLANE_A + off);
      }
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const int off = 2 * PLANE_A + ((wn * TN + n) * 16 + lr) * kRowB + coff;
        bh[n] = *reinterpret_cast<const s16x8*>(base + off);
        bl[n] = *reinterpret_cast<const s16x8*>(base + PLANE_B + off);
      }
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(ah[m]), as_f16x8(bh[n]),
                                                             acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(ah[m]), as_f16x8(bl[n]),
                                                             acc[m][n], 0, 0, 0);
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(as_f16x8(al[m]), as_f16x8(bh[n]),
                                                             acc[m][n], 0, 0, 0);
        }
    }
    fwd_tile_epilogue<WM, WN, TM, TN>(p, ln, acc, scale, b, s0, nt,
                                      reinterpret_cast<float*>(smem));
  }
  fwd_colsum_epilogue<WM, WN, TM, TN>(p, ln, b, sc, n0, reinterpret_cast<float*>(smem));
}

// One block per batch row b.  rowpart -> rowstat, bstat.
__global__ __launch_bounds__(256) void fwd_combine_kernel(const float* __restrict__ y,
                                                         const float* __restrict__ rowpart,
                                                         float* __restrict__ rowstat,
                                                         float* __restrict__ bstat, int S, int B,
                                                         int L, int nNt) {
  __shared__ float red[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  float np = 0.f, nn = 0.f;
  for (int l = tid; l < L; l += blockDim.x) {
    const float v = y[(int64_t)b * L + l];
    np += (v == 1.0f) ? 1.0f : 0.0f;
    nn += (v == 0.0f) ? 1.0f : 0.0f;
  }
  np = block_reduce<false>(np, red);
  nn = block_reduce<false>(nn, red);
  const float nrm = np * nn;  // normalizers = |pos| * |neg|  (mpvae.py:115-117)

  float me = -INFINITY, mx = -INFINITY, ce = 0.f, cx = 0.f;
  for (int s = tid; s < S; s += blockDim.x) {
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
  }
  me = block_reduce<true>(me, red);
  mx = block_reduce<true>(mx, red);
  ce = block_reduce<false>(ce, red);
  cx = block_reduce<false>(cx, red);
  float ze = 0.f, zx = 0.f;
  for (int s = tid; s < S; s += blockDim.x) {
    ze += expf(rowstat[((int64_t)0 * B + b) * S + s] - me);
    zx += expf(rowstat[((int64_t)1 * B + b) * S + s] - mx);
  }
  ze = block_reduce<false>(ze, red);
  zx = block_reduce<false>(zx, red);
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
__global__ __launch_bounds__(256) void finalize_kernel(mpv_final_args a, int B, int L,
                                                      float S_total) {
  if (blockIdx.x > 0) {
    const int64_t n = (int64_t)B * L;
    for (int64_t i = (int64_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)(gridDim.x - 1) * blockDim.x) {
      a.indiv_prob_label[i] = a.colsum[i] / S_total;
      a.indiv_prob[i] = a.colsum[n + i] / S_total;
    }
    return;
  }
  __shared__ float red[16];
  const int tid = threadIdx.x;
  float ne = 0.f, nx = 0.f, ce = 0.f, cx = 0.f;
  for (int b = tid; b < B; b += blockDim.x) {
    // nll = mean_b(-log(mean_s exp(logp - max)) - max)   (mpvae.py:188-190)
    ne += -logf(a.bstat[1 * B + b] / S_total) - a.bstat[0 * B + b];
    nx += -logf(a.bstat[3 * B + b] / S_total) - a.bstat[2 * B + b];
    ce += a.bstat[4 * B + b];
    cx += a.bstat[5 * B + b];
  }
  float kl = 0.f;
  const int64_t nd = (int64_t)B * a.d;
  for (int64_t i = tid; i < nd; i += blockDim.x) {
    const float lve = a.fe_logvar[i], lvx = a.fx_logvar[i];
    const float dm = a.fx_mu[i] - a.fe_mu[i];
    kl += (lvx - lve) - 1.0f + expf(lve - lvx) + dm * dm / (expf(lvx) + kKlEps);
  }
  ne = block_reduce<false>(ne, red);
  nx = block_reduce<false>(nx, red);
  ce = block_reduce<false>(ce, red);
  cx = block_reduce<false>(cx, red);
  kl = block_reduce<false>(kl, red);
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

// ---------------------------------------------------------------- host side
struct FwdPlan {
  int cfg;  // tile configuration, see launch_fwd
  int BM, BN, nNt, nSt, nSc, tps;
  size_t rowpart_bytes, colpart_bytes;
};

static FwdPlan plan_fwd(const mpv_shape* s) {
  FwdPlan pl;
  pl.cfg = s->L <= 48 ? 0 : (s->L <= 96 ? 1 : 2);
  pl.BM = 128;
  pl.BN = pl.cfg == 0 ? 48 : (pl.cfg == 1 ? 96 : 128);
  pl.nNt = (int)cdiv(s->L, pl.BN);
  pl.nSt = (int)cdiv(s->S_local, pl.BM);
  // enough workgroups to fill 256 CUs several times; fewer s-chunks = fewer partials
  int64_t want = cdiv(2048, s->B * (int64_t)pl.nNt);
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
      case 0:  // BN 48, 4 waves, 3-stage ring (66 KB LDS: 2 workgroups per CU)
        MPV_LAUNCH("probit_fwd", (probit_fwd16_kernel<4, 1, 2, 3, 3>), grid, dim3(256), 0, st, p);
        break;
      case 1:  // BN 96, 8 waves, 4-stage ring (112 KB)
        MPV_LAUNCH("probit_fwd", (probit_fwd16_kernel<4, 2, 2, 3, 4>), grid, dim3(512), 0, st, p);
        break;
      default:  // 128 x 128 tile, 4 waves of 64 x 64 (3 MFMAs per 1.33 fragment
                // reads), 2-stage ring (64 KB): 2 workgroups per CU, so one
                // workgroup's epilogue (VALU) overlaps the other's MFMA phase
        MPV_LAUNCH("probit_fwd", (probit_fwd16_kernel<2, 2, 4, 4, 2>), grid, dim3(256), 0, st, p);
        break;
    }
  }
}

static int check_split_operand(const mpv_split16& o, int64_t rows, int64_t ld_min,
                               const char* what) {
  MPV_REQUIRE(o.hi && o.lo && o.scale, "%s: NULL plane", what);
  MPV_REQUIRE(o.rows_pad >= rows, "%s: rows_pad %lld < %lld", what, (long long)o.rows_pad,
              (long long)rows);
  MPV_REQUIRE(o.ld >= ld_min && (o.ld % 8) == 0, "%s: ld %lld must be >= %lld and a multiple of 8",
              what, (long long)o.ld, (long long)ld_min);
  return MPV_OK;
}

}  // namespace mpv

using namespace mpv;

extern "C" {

size_t mpv_fwd_workspace_bytes(const mpv_shape* shape) {
  if (check_shape(shape) != MPV_OK) return 0;
  const FwdPlan pl = plan_fwd(shape);
  return pl.rowpart_bytes + pl.colpart_bytes;
}

int mpv_probit_fwd(const mpv_shape* shape, const mpv_fwd_args* a, void* stream) {
  if (int rc = check_shape(shape)) return rc;
  MPV_REQUIRE(a != nullptr, "args is NULL");
  MPV_REQUIRE(a->y && a->fe_out && a->fx_out && a->rowstat && a->bstat && a->colsum &&
                  a->workspace,
              "NULL pointer in mpv_fwd_args");
  MPV_REQUIRE(a->gemm == MPV_GEMM_F32 || a->gemm == MPV_GEMM_F16X3, "unknown gemm mode %d",
              a->gemm);
  const FwdPlan pl = plan_fwd(shape);
  if (a->gemm == MPV_GEMM_F32) {
    MPV_REQUIRE(a->R32 && a->eps, "MPV_GEMM_F32 needs R32 and eps");
  } else {
    const int64_t zp = cdiv(shape->z, 64) * 64;
    if (int rc = check_split_operand(a->R16, (int64_t)pl.nNt * pl.BN, zp, "R16")) return rc;
    if (int rc = check_split_operand(a->eps16, shape->S_local * shape->B, zp, "eps16")) return rc;
    // the DMA issue keeps per-lane byte offsets within one s/l tile in 32 bits
    MPV_REQUIRE((int64_t)pl.BM * shape->B * a->eps16.ld * 2 < (int64_t(1) << 32) &&
                    (int64_t)pl.BN * a->R16.ld * 2 < (int64_t(1) << 32),
                "B * ld too large for the f16x3 tile offsets");
  }
  MPV_REQUIRE(a->workspace_bytes >= pl.rowpart_bytes + pl.colpart_bytes,
              "workspace too small: %zu < %zu", a->workspace_bytes,
              pl.rowpart_bytes + pl.colpart_bytes);
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
  p.z = (int)shape->z;
  p.nNt = pl.nNt;
  p.nSc = pl.nSc;
  p.tps = pl.tps;
  p.nSt = pl.nSt;
  const int64_t blocks = (int64_t)shape->B * pl.nSc * pl.nNt;
  MPV_REQUIRE(blocks < (int64_t(1) << 31), "grid too large");
  launch_fwd(pl, a->gemm, dim3((unsigned)blocks), st, p);
  if (int rc = check_launch("probit_fwd")) return rc;
  MPV_LAUNCH("fwd_combine", fwd_combine_kernel, dim3((unsigned)shape->B), dim3(256), 0, st, a->y,
             p.rowpart, a->rowstat, a->bstat, p.S, p.B, p.L, pl.nNt);
  if (int rc = check_launch("fwd_combine")) return rc;
  if (pl.nSc > 1) {
    if (int rc = launch_sum_slabs(p.colpart, pl.nSc, 2 * shape->B * shape->L, a->colsum, MPV_F32, st))
      return rc;
  }
  return MPV_OK;
}

int mpv_probit_finalize(const mpv_shape* shape, const mpv_final_args* a, void* stream) {
  MPV_REQUIRE(shape && shape->B > 0 && shape->L > 0 && shape->S_total > 0, "bad shape");
  MPV_REQUIRE(a && a->bstat && a->colsum && a->fe_mu && a->fe_logvar && a->fx_mu &&
                  a->fx_logvar && a->total && a->nll && a->nll_x && a->c && a->c_x && a->kl &&
                  a->indiv_prob && a->indiv_prob_label && a->d > 0,
              "NULL pointer in mpv_final_args");
  const int64_t n = shape->B * shape->L;
  int64_t nb = cdiv(n, 256);
  if (nb > 4096) nb = 4096;
  MPV_LAUNCH("finalize", finalize_kernel, dim3((unsigned)(1 + nb)), dim3(256), 0,
             as_stream(stream), *a, (int)shape->B, (int)shape->L, (float)shape->S_total);
  return check_launch("finalize");
}

}  // extern "C"
