// Encoder / decoder Linear layers of the VAE (reference mpvae.py:14-38, used
// at :51-84) and their backward, on the fp32 matrix cores.
//
//   out(i, j) = act(alpha * (sum_r A(i, r) B(j, r) + bias(j)))
//
// with A and B addressed by (row, reduction) strides, so one kernel serves
//   forward   y  = x W^T        A = x (M x K), B = W (N x K)
//   grad in   dx = (dy . m) W   A = dy masked by the ReLU output, B = W^T view
//   grad W,b  dW = (dy . m)^T x A = dy^T view, B = x^T view, plus a column of
//                                 ones in B whose output column is db.
// The reference's shapes are small-batch (B = 32..512 rows, K <= ~1100, N <=
// 512): a library GEMM tiles them into 2-16 workgroups that each walk the
// whole reduction on one CU (hipBLASLt MT256x256x32 at C3: 65-155 us per
// GEMM).  Here the output is cut into 64 x 64 tiles and the reduction into
// chunks until the launch has ~512 workgroups; chunk partials are summed in
// a fixed order by lin_reduce (deterministic, no atomics).
//
// Tile: 4 waves of 32 x 32 (2 x 2 v_mfma_f32_16x16x4_f32 blocks); 16
// reduction rows per LDS stage (64 measured no faster: 0.46 vs 0.36 ms for
// the 43 GEMMs of a C3 training step); the next stage's global loads are
// issued before the current stage's MFMAs (register double buffer).
// A problem may have a second reduction segment (other A and B pointers for
// reduction indices >= R1): the two heads' dx of one input as one GEMM.
// Independent GEMMs (a layer's dx and dW; both heads of an encoder, or of
// the stacked decoder, with their gradients) go in one launch: up to
// kLinMaxProb problems, told apart by blockIdx.z ranges.
#include "abi_util.h"
#include "mpv_common.h"

namespace mpv {
namespace {

constexpr int kLinTile = 64;      // output tile edge (i and j)
constexpr int kLinStep = 16;      // reduction rows per LDS stage
constexpr int kLinPer = kLinTile * kLinStep / 256;  // operand elements per thread per stage
constexpr int kLinThreads = 256;  // 4 waves
constexpr int kLinWant = 512;     // workgroups per launch to aim for (2 per CU)
constexpr int kLinMinChunk = 32;  // reduction rows per split, at least

struct LinParams {
  int64_t M, N, R;
  const float* a;
  int64_t a_si, a_sr;
  const float* a_mask;
  float a_scale;
  const float* b;
  int64_t b_sj, b_sr;
  int64_t ones_col;  // j == ones_col reads B = 1 (bias-gradient column), -1: none
  const float* bias;
  float alpha;
  int relu;
  float* out;
  int64_t out_si;
  float* out_col;
  float* part;    // (nsplit, M, N) chunk partials, null: direct epilogue
  int64_t chunk;  // reduction rows per split
  // second reduction segment (a2 != null): reduction index r >= R1 reads
  // A = a2 (row stride a2_si) and B = b2 (B's strides) at r - R1
  const float* a2;
  int64_t a2_si;
  const float* b2;
  int64_t R1;
};

// kLinPer elements of a 64-row x 64-reduction operand tile, mapped so that
// consecutive threads read consecutive addresses in either orientation
// (reduction-contiguous: 4 threads cover 256 B of a row; row-contiguous: 64
// threads cover 64 rows of one reduction index).
struct LinSlot {
  int row, red;  // of the thread's first element; its elements step the reduction
};

MPV_DEV LinSlot lin_slot(int64_t s_row, int64_t s_red) {
  const int t = threadIdx.x;
  if (s_red == 1 && s_row != 1) return LinSlot{t >> 2, (t & 3) * kLinPer};
  return LinSlot{t & 63, (t >> 6) * kLinPer};
}

template <bool IS_A>
MPV_DEV void lin_load(const LinParams& p, const LinSlot& sl, int64_t row0, int64_t r0, int64_t r_end,
                      float v[kLinPer]) {
  const int64_t rows = IS_A ? p.M : p.N;
  const int64_t row = row0 + sl.row;
  const float* src = IS_A ? p.a : p.b;
  const int64_t s_row = IS_A ? p.a_si : p.b_sj, s_red = IS_A ? p.a_sr : p.b_sr;
#pragma unroll
  for (int q = 0; q < kLinPer; ++q) {
    const int64_t r = r0 + sl.red + q;
    float x = 0.0f;
    if (row < rows && r < r_end) {
      if (!IS_A && row == p.ones_col) {
        x = 1.0f;
      } else {
        const bool seg2 = (IS_A ? p.a2 : p.b2) != nullptr && r >= p.R1;
        const int64_t o = seg2 ? row * (IS_A ? p.a2_si : s_row) + (r - p.R1) * s_red
                               : row * s_row + r * s_red;
        x = seg2 ? (IS_A ? p.a2 : p.b2)[o] : src[o];
        if (IS_A) {
          // ReLU backward: torch's threshold_backward zeroes the gradient
          // where the layer output is <= 0 (a NaN output passes it, as in
          // torch).  With dropout folded in (the mask is the dropout output)
          // the one difference from torch is a dropped element whose ReLU
          // output is NaN: NaN * 0 is NaN here, so its gradient passes, where
          // torch's dropout backward zeroes it first.
          if (p.a_mask != nullptr && p.a_mask[o] <= 0.0f) x = 0.0f;
          x *= p.a_scale;
        }
      }
    }
    v[q] = x;
  }
}

MPV_DEV void lin_stash(float (*s)[kLinTile + 4], const LinSlot& sl, const float v[kLinPer]) {
#pragma unroll
  for (int q = 0; q < kLinPer; ++q) s[sl.red + q][sl.row] = v[q];
}

MPV_DEV void lin_finish(const LinParams& p, int64_t i, int64_t j, float s) {
  if (j == p.ones_col) {
    p.out_col[i] = s;
    return;
  }
  if (p.bias != nullptr) s += p.bias[j];
  s *= p.alpha;
  if (p.relu) s = s <= 0.0f ? 0.0f : s;  // NaN passes, as torch.relu
  p.out[i * p.out_si + j] = s;
}

constexpr int kLinMaxProb = 4;

struct LinBatch {
  LinParams p[kLinMaxProb];
  int n;
  int ti[kLinMaxProb], tj[kLinMaxProb];
  int zoff[kLinMaxProb + 1];      // blockIdx.z range of each problem (its chunks)
  int64_t eoff[kLinMaxProb + 1];  // lin_reduce element range (0 long without split)
};

__global__ __launch_bounds__(kLinThreads) void lin_gemm_kernel(LinBatch bt) {
  __shared__ float sa[kLinStep][kLinTile + 4];
  __shared__ float sb[kLinStep][kLinTile + 4];
  int q = 0;  // the problem whose chunk range holds blockIdx.z
#pragma unroll
  for (int k = 1; k < kLinMaxProb; ++k)
    if (k < bt.n && (int)blockIdx.z >= bt.zoff[k]) q = k;
  const LinParams& p = bt.p[q];
  if ((int)blockIdx.x >= bt.ti[q] || (int)blockIdx.y >= bt.tj[q])
    return;  // this problem has fewer tiles than the grid
  const int split = (int)blockIdx.z - bt.zoff[q];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kLinTile, j0 = (int64_t)blockIdx.y * kLinTile;
  const int64_t rb = (int64_t)split * p.chunk, re = min(p.R, rb + p.chunk);
  const int wi = (w & 1) * 32, wj = (w >> 1) * 32;
  const LinSlot sla = lin_slot(p.a_si, p.a_sr), slb = lin_slot(p.b_sj, p.b_sr);

  f32x4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  float va[kLinPer], vb[kLinPer];
  if (rb < re) {
    lin_load<true>(p, sla, i0, rb, re, va);
    lin_load<false>(p, slb, j0, rb, re, vb);
  }
  for (int64_t r0 = rb; r0 < re; r0 += kLinStep) {
    __syncthreads();  // every wave is done reading the previous stage
    lin_stash(sa, sla, va);
    lin_stash(sb, slb, vb);
    __syncthreads();
    if (r0 + kLinStep < re) {
      lin_load<true>(p, sla, i0, r0 + kLinStep, re, va);
      lin_load<false>(p, slb, j0, r0 + kLinStep, re, vb);
    }
#pragma unroll
    for (int ks = 0; ks < kLinStep / 4; ++ks) {
      // 16x16x4 f32: lane l holds A(l % 16, l / 16) and B(l / 16, l % 16)
      const int rr = ks * 4 + (lane >> 4), c = lane & 15;
      const float a0 = sa[rr][wi + c], a1 = sa[rr][wi + 16 + c];
      const float b0 = sb[rr][wj + c], b1 = sb[rr][wj + 16 + c];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // accumulator v of lane l: row 4 (l / 16) + v, column l % 16 of its block
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t i = i0 + wi + m * 16 + (lane >> 4) * 4 + v;
        const int64_t j = j0 + wj + n * 16 + (lane & 15);
        if (i < p.M && j < p.N) {
          if (p.part != nullptr)
            p.part[((int64_t)split * p.M + i) * p.N + j] = acc[m][n][v];
          else
            lin_finish(p, i, j, acc[m][n][v]);
        }
      }
}

// Chunk partials -> outputs, summed in chunk order (problems with a split).
__global__ __launch_bounds__(256) void lin_reduce_kernel(LinBatch bt) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < bt.eoff[bt.n];
       e += (int64_t)gridDim.x * blockDim.x) {
    int q = 0;
#pragma unroll
    for (int k = 1; k < kLinMaxProb; ++k)
      if (k < bt.n && e >= bt.eoff[k]) q = k;
    const LinParams& p = bt.p[q];
    const int64_t le = e - bt.eoff[q], n = p.M * p.N;
    const int nsplit = bt.zoff[q + 1] - bt.zoff[q];
    float s = 0.0f;
    for (int k = 0; k < nsplit; ++k) s += p.part[k * n + le];
    lin_finish(p, le / p.N, le % p.N, s);
  }
}

struct LinPlan {
  int64_t ti, tj, nsplit, chunk;
  size_t part_bytes;
};

LinPlan plan_linear(int64_t M, int64_t N, int64_t R) {
  LinPlan pl;
  pl.ti = cdiv(M, kLinTile);
  pl.tj = cdiv(N, kLinTile);
  int64_t want = kLinWant / std::max<int64_t>(1, pl.ti * pl.tj);
  want = std::max<int64_t>(1, std::min<int64_t>(want, cdiv(R, kLinMinChunk)));
  pl.chunk = std::max<int64_t>(kLinStep, cdiv(cdiv(R, want), kLinStep) * kLinStep);
  pl.nsplit = std::max<int64_t>(1, cdiv(R, pl.chunk));
  pl.part_bytes = pl.nsplit > 1 ? align_up(sizeof(float) * pl.nsplit * M * N, 256) : 0;
  return pl;
}

}  // namespace
}  // namespace mpv

using namespace mpv;

extern "C" {

size_t mpv_linear_workspace_bytes(int64_t M, int64_t N, int64_t R) {
  if (M <= 0 || N <= 0 || R < 0) return 0;
  return plan_linear(M, N, R).part_bytes;
}

size_t mpv_linear_batch_workspace_bytes(const mpv_linear_args* args, int n) {
  size_t total = 0;
  for (int q = 0; args != nullptr && q < n; ++q)
    total += mpv_linear_workspace_bytes(args[q].M, args[q].N, args[q].R);
  return total;
}

int mpv_linear_batch(const mpv_linear_args* args, int n, void* workspace, size_t workspace_bytes,
                     void* stream) {
  MPV_REQUIRE(args != nullptr && n >= 1 && n <= kLinMaxProb, "linear: 1..%d problems per launch",
              kLinMaxProb);
  LinBatch bt;
  bt.n = 0;
  bt.zoff[0] = 0;
  bt.eoff[0] = 0;
  int64_t gx = 0, gy = 0;
  size_t off = 0;
  char* ws = reinterpret_cast<char*>(workspace);
  for (int k = 0; k < n; ++k) {
    const mpv_linear_args* a = &args[k];
    MPV_REQUIRE(a->M >= 0 && a->N >= 0 && a->R >= 0, "bad linear sizes (problem %d)", k);
    if (a->M == 0 || a->N == 0) continue;
    MPV_REQUIRE(a->out != nullptr && (a->R == 0 || (a->a != nullptr && a->b != nullptr)),
                "linear: NULL operand (problem %d)", k);
    MPV_REQUIRE(a->ones_col < 0 || (a->ones_col == a->N - 1 && a->out_col != nullptr),
                "linear: the ones column must be the last output column, with out_col");
    MPV_REQUIRE(a->M < 65535ll * kLinTile && a->N < 65535ll * kLinTile,
                "linear: output too large for the grid");
    const LinPlan pl = plan_linear(a->M, a->N, a->R);
    MPV_REQUIRE(bt.zoff[bt.n] + pl.nsplit < 65535, "linear: too many reduction chunks");
    MPV_REQUIRE(off + pl.part_bytes <= workspace_bytes && (pl.part_bytes == 0 || workspace != nullptr),
                "linear: workspace %zu < %zu bytes", workspace_bytes, off + pl.part_bytes);
    LinParams& p = bt.p[bt.n];
    p.M = a->M;
    p.N = a->N;
    p.R = a->R;
    p.a = a->a;
    p.a_si = a->a_si;
    p.a_sr = a->a_sr;
    p.a_mask = a->a_mask;
    p.a_scale = a->a_scale;
    p.b = a->b;
    p.b_sj = a->b_sj;
    p.b_sr = a->b_sr;
    p.ones_col = a->ones_col < 0 ? -1 : a->ones_col;
    p.bias = a->bias;
    p.alpha = a->alpha;
    p.relu = a->relu;
    p.out = a->out;
    p.out_si = a->out_si;
    p.out_col = a->out_col;
    MPV_REQUIRE((a->a2 == nullptr) == (a->b2 == nullptr) &&
                    (a->a2 == nullptr || (a->a_mask == nullptr && a->R1 >= 0 && a->R1 <= a->R)),
                "linear: a second segment needs a2 and b2, no mask, 0 <= R1 <= R (problem %d)", k);
    p.a2 = a->a2;
    p.a2_si = a->a2_si;
    p.b2 = a->b2;
    p.R1 = a->a2 != nullptr ? a->R1 : a->R;
    p.part = pl.nsplit > 1 ? reinterpret_cast<float*>(ws + off) : nullptr;
    p.chunk = pl.chunk;
    off += pl.part_bytes;
    bt.ti[bt.n] = (int)pl.ti;
    bt.tj[bt.n] = (int)pl.tj;
    bt.zoff[bt.n + 1] = bt.zoff[bt.n] + (int)pl.nsplit;
    bt.eoff[bt.n + 1] = bt.eoff[bt.n] + (pl.nsplit > 1 ? a->M * a->N : 0);
    gx = std::max<int64_t>(gx, pl.ti);
    gy = std::max<int64_t>(gy, pl.tj);
    ++bt.n;
  }
  if (bt.n == 0) return MPV_OK;
  for (int k = bt.n; k < kLinMaxProb; ++k) {  // unused slots: never selected
    bt.p[k] = bt.p[0];
    bt.ti[k] = bt.tj[k] = 0;
    bt.zoff[k + 1] = bt.zoff[k];
    bt.eoff[k + 1] = bt.eoff[k];
  }
  const hipStream_t st = as_stream(stream);
  MPV_LAUNCH("linear", lin_gemm_kernel, dim3((unsigned)gx, (unsigned)gy, (unsigned)bt.zoff[bt.n]),
             dim3(kLinThreads), 0, st, bt);
  if (bt.eoff[bt.n] > 0)
    MPV_LAUNCH("linear", lin_reduce_kernel,
               dim3((unsigned)std::min<int64_t>(cdiv(bt.eoff[bt.n], 256), 2048)), dim3(256), 0, st, bt);
  return check_launch("linear");
}

int mpv_linear(const mpv_linear_args* a, void* workspace, size_t workspace_bytes, void* stream) {
  return mpv_linear_batch(a, 1, workspace, workspace_bytes, stream);
}

}  // extern "C"
