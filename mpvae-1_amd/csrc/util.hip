// Small kernels of the hot path: Philox noise (a7), dtype conversion (a8
// prep / fp64 gradient), slab reductions, the cross-shard statistic combine,
// the fused two-encoder reparameterisation (a3) and the KL backward (a5).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "abi_util.h"
#include "mpv_common.h"

namespace mpv {

static thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MPV_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return MPV_OK;
}

// ---------------------------------------------------------- launch timing
struct TimerSlot {
  std::string name;
  std::vector<hipEvent_t> start, stop;
  size_t used = 0;
};
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<TimerSlot> g_slots;

TimedLaunch::TimedLaunch(const char* kernel, hipStream_t s) : s_(s) {
  if (!g_timing) return;
  std::lock_guard<std::mutex> lk(g_tmu);
  int k = -1;
  for (size_t i = 0; i < g_slots.size(); ++i)
    if (g_slots[i].name == kernel) k = (int)i;
  if (k < 0) {
    g_slots.push_back(TimerSlot{kernel, {}, {}, 0});
    k = (int)g_slots.size() - 1;
  }
  TimerSlot& t = g_slots[k];
  if (t.used == t.start.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return;
    if (hipEventCreate(&b) != hipSuccess) return;
    t.start.push_back(a);
    t.stop.push_back(b);
  }
  pair_ = t.used++;
  slot_ = k;
  (void)hipEventRecord(t.start[pair_], s_);
}

TimedLaunch::~TimedLaunch() {
  if (slot_ < 0) return;
  std::lock_guard<std::mutex> lk(g_tmu);
  (void)hipEventRecord(g_slots[slot_].stop[pair_], s_);
}

int check_shape(const mpv_shape* s) {
  MPV_REQUIRE(s != nullptr, "shape is NULL");
  MPV_REQUIRE(s->B > 0 && s->L > 0 && s->z > 0, "B, L, z must be positive (got %lld, %lld, %lld)",
              (long long)s->B, (long long)s->L, (long long)s->z);
  MPV_REQUIRE(s->S_local > 0 && s->S_total >= s->S_local && s->s_offset >= 0 &&
                  s->s_offset + s->S_local <= s->S_total,
              "bad sample range: S_local=%lld S_total=%lld s_offset=%lld",
              (long long)s->S_local, (long long)s->S_total, (long long)s->s_offset);
  MPV_REQUIRE(s->B * s->S_local < (int64_t(1) << 31), "B*S_local must fit in int32");
  MPV_REQUIRE(s->L < (1 << 24) && s->z < (1 << 24), "L and z must be < 2^24");
  return MPV_OK;
}

// ------------------------------------------------------------- Philox noise
// One thread = one Philox counter = 4 consecutive noise elements.
// The Philox key: the host value, or (seed_dev != nullptr) the 64-bit word
// at seed_dev, read on the device at run time -- so a captured graph draws
// fresh noise each replay when the step bumps that word.
MPV_DEV void philox_key(const uint64_t* seed_dev, uint32_t& k0, uint32_t& k1) {
  if (seed_dev != nullptr) {
    const uint64_t k = __builtin_nontemporal_load(seed_dev);
    k0 = (uint32_t)k;
    k1 = (uint32_t)(k >> 32);
  }
}

__global__ void noise_philox_kernel(float* __restrict__ eps, int64_t e_begin, int64_t e_count,
                                    uint32_t k0, uint32_t k1, uint64_t offset,
                                    const uint64_t* __restrict__ seed_dev) {
  philox_key(seed_dev, k0, k1);
  const int64_t g0 = e_begin >> 2;  // first counter touching the shard
  const int64_t e_end = e_begin + e_count;
  // grid-stride: a launch is capped below 2^32 threads, a C5 shard is not
  for (int64_t g = g0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; (g << 2) < e_end;
       g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t ctr = (uint64_t)g + offset;
    const u32x4 w = philox4x32_10(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u}, k0, k1);
    float n[4];
    box_muller(w.x, w.y, n[0], n[1]);
    box_muller(w.z, w.w, n[2], n[3]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t e = (g << 2) + q;
      if (e >= e_begin && e < e_end) eps[e - e_begin] = n[q];
    }
  }
}

__global__ void philox_raw_kernel(uint32_t* out, int64_t n, uint64_t ctr0, uint32_t k0,
                                  uint32_t k1) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t c = ctr0 + (uint64_t)i;
  const u32x4 w = philox4x32_10(u32x4{(uint32_t)c, (uint32_t)(c >> 32), 0u, 0u}, k0, k1);
  out[4 * i + 0] = w.x;
  out[4 * i + 1] = w.y;
  out[4 * i + 2] = w.z;
  out[4 * i + 3] = w.w;
}

// ------------------------------------------------------------- conversions
template <typename S, typename D>
__global__ void convert_kernel(const S* __restrict__ src, D* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (D)src[i];
}

// out[i] = sum_k in[k*n + i], k < nslab (fixed order -> deterministic).
template <typename D>
__global__ void sum_slabs_kernel(const float* __restrict__ in, int64_t nslab, int64_t n,
                                 D* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.0f;
    // fixed summation order (deterministic); unrolled so that the loads of
    // several slabs are in flight together
#pragma unroll 8
    for (int64_t k = 0; k < nslab; ++k) acc += in[k * n + i];
    out[i] = (D)acc;
  }
}

// Few columns over many slabs (small L x z, or the column partials): 16 waves
// per workgroup split the slabs (wave g sums slabs g, g+16, ..., one coalesced
// 256-B row each), then a fixed-order sum of the 16 partials through LDS: the
// serial chain per lane is nslab/16 loads instead of nslab.
template <typename D>
__global__ __launch_bounds__(1024) void sum_slabs_split_kernel(const float* __restrict__ in,
                                                               int64_t nslab, int64_t n,
                                                               D* __restrict__ out) {
  __shared__ float part[16][65];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  float acc = 0.0f;
  if (i < n) {
#pragma unroll 4
    for (int64_t k = g; k < nslab; k += 16) acc += in[k * n + i];
  }
  part[g][lane] = acc;
  __syncthreads();
  if (g == 0 && i < n) {
    float t = part[0][lane];
#pragma unroll
    for (int j = 1; j < 16; ++j) t += part[j][lane];
    out[i] = (D)t;
  }
}

// Two slab sums in one launch (the backward's column partials and its dR
// slabs): workgroups [0, a.blocks) sum problem a, the rest problem b, each in
// the layout and order of sum_slabs_kernel (plain: a thread per element, the
// slabs in order) or sum_slabs_split_kernel (split: 64 columns per workgroup,
// 16 slab groups, partials added in order), so results are the bits of the
// separate launches.
struct SlabSum {
  const float* in;
  int64_t nslab, n;
  void* out;
  int f64;     // out is double
  int split;   // the split layout (few columns, many slabs)
  int vec;     // 4 consecutive elements per thread (16-B loads): n % 4 == 0, aligned
  int64_t blocks;
};

MPV_DEV void slab_store(const SlabSum& q, int64_t i, float v) {
  if (q.f64)
    reinterpret_cast<double*>(q.out)[i] = (double)v;
  else
    reinterpret_cast<float*>(q.out)[i] = v;
}

__global__ __launch_bounds__(1024) void sum_slabs_pair_kernel(SlabSum a, SlabSum b) {
  __shared__ float part[16][65];
  const bool second = (int64_t)blockIdx.x >= a.blocks;
  const SlabSum q = second ? b : a;
  const int64_t blk = second ? (int64_t)blockIdx.x - a.blocks : (int64_t)blockIdx.x;
  if (q.split) {
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t i = blk * 64 + lane;
    float acc = 0.0f;
    if (i < q.n) {
#pragma unroll 4
      for (int64_t k = g; k < q.nslab; k += 16) acc += q.in[k * q.n + i];
    }
    part[g][lane] = acc;
    __syncthreads();
    if (g == 0 && i < q.n) {
      float t = part[0][lane];
#pragma unroll
      for (int j = 1; j < 16; ++j) t += part[j][lane];
      slab_store(q, i, t);
    }
  } else if (q.vec) {  // the same sums, four elements per thread (16-B loads)
    const int64_t i = (blk * 1024 + threadIdx.x) * 4;
    if (i < q.n) {
      f32x4 acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int64_t k = 0; k < q.nslab; ++k) acc += *reinterpret_cast<const f32x4*>(q.in + k * q.n + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) slab_store(q, i + j, acc[j]);
    }
  } else {
    const int64_t i = blk * 1024 + threadIdx.x;
    if (i < q.n) {
      float acc = 0.0f;
#pragma unroll 8
      for (int64_t k = 0; k < q.nslab; ++k) acc += q.in[k * q.n + i];
      slab_store(q, i, acc);
    }
  }
}

// gathered (R,6,B) -> out (6,B)
__global__ void bstat_combine_kernel(const float* __restrict__ g, int64_t R, int64_t B,
                                     float* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float v[6];
  bstat_combine_row(g, R, B, b, v);
#pragma unroll
  for (int k = 0; k < 6; ++k) out[k * B + b] = v[k];
}

// ------------------------------------------------------ reparameterisation
// z = mu + eps * exp(0.5 * logvar)  (mpvae.py:67-69, 72-74), both encoders.
__global__ void reparam_fwd_kernel(mpv_reparam_args a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n_e) {
    const float mu = a.mu_e[i], lv = a.logvar_e[i];
    a.z_e[i] = mu + a.eps_e[i] * expf(0.5f * lv);
    if (a.mu_e_out != nullptr) a.mu_e_out[i] = mu;
    if (a.logvar_e_out != nullptr) a.logvar_e_out[i] = lv;
  } else if (i - a.n_e < a.n_x) {
    const int64_t j = i - a.n_e;
    const float mu = a.mu_x[j], lv = a.logvar_x[j];
    a.z_x[j] = mu + a.eps_x[j] * expf(0.5f * lv);
    if (a.mu_x_out != nullptr) a.mu_x_out[j] = mu;
    if (a.logvar_x_out != nullptr) a.logvar_x_out[j] = lv;
  }
}

__global__ void reparam_bwd_kernel(mpv_reparam_bwd_args a) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float* gz;
  const float* lv;
  const float* ep;
  float* gmu;
  float* glv;
  int64_t j;
  if (i < a.n_e) {
    gz = a.gz_e; lv = a.logvar_e; ep = a.eps_e; gmu = a.gmu_e; glv = a.glogvar_e; j = i;
  } else if (i - a.n_e < a.n_x) {
    gz = a.gz_x; lv = a.logvar_x; ep = a.eps_x; gmu = a.gmu_x; glv = a.glogvar_x; j = i - a.n_e;
  } else {
    return;
  }
  const float* amu = i < a.n_e ? a.gmu_add_e : a.gmu_add_x;
  const float* alv = i < a.n_e ? a.glogvar_add_e : a.glogvar_add_x;
  // the gradients mu / logvar also receive elsewhere (compute_loss's KL),
  // added as autograd would add them: one rounded add (fp contract off above)
  const float g = gz ? gz[j] : 0.0f;
  const float r = g * ep[j] * 0.5f * expf(0.5f * lv[j]);
  gmu[j] = amu ? g + amu[j] : g;
  glv[j] = alv ? r + alv[j] : r;
}

// d KL / d (mu, logvar) of mpvae.py:147-148 (kl_bwd_range, mpv_common.h).
__global__ void kl_bwd_kernel(mpv_kl_bwd_args a) {
  kl_bwd_range(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// --------------------------------------------------------- 3xf16 operands
constexpr int kMaxBlocks = 1024;  // block maxima of maxabs_kernel (workspace size)
constexpr int kSplitMaxBlocks = 256;  // maxabs blocks of mpv_split_f16 (read by every split wave)

template <typename T>
__global__ __launch_bounds__(256) void maxabs_kernel(const T* __restrict__ x, int64_t n,
                                                    float* __restrict__ block_max) {
  __shared__ float red[16];
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf((float)x[i]));
  m = block_reduce<true>(m, red);
  if (threadIdx.x == 0) block_max[blockIdx.x] = m;
}


// maxabs_kernel on 16-B vectors with four independent maxima per thread (the
// scalar loop kept a dependent max chain and few loads in flight: 10.6 us for
// r_sqrt_sigma at C4).  x 16-B aligned; the n % VEC tail is block 0's.
template <typename T>
__global__ __launch_bounds__(256) void maxabs_vec_kernel(const T* __restrict__ x, int64_t n,
                                                        float* __restrict__ block_max) {
  constexpr int VEC = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(VEC)));
  __shared__ float red[16];
  const vec_t* xv = reinterpret_cast<const vec_t*>(x);
  const int64_t nv = n / VEC, st = (int64_t)gridDim.x * blockDim.x;
  float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * st < nv; i += 4 * st) {
    const vec_t a = xv[i], b = xv[i + st], c = xv[i + 2 * st], d = xv[i + 3 * st];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      m0 = fmaxf(m0, fabsf((float)a[k]));
      m1 = fmaxf(m1, fabsf((float)b[k]));
      m2 = fmaxf(m2, fabsf((float)c[k]));
      m3 = fmaxf(m3, fabsf((float)d[k]));
    }
  }
  for (; i < nv; i += st) {
    const vec_t a = xv[i];
#pragma unroll
    for (int k = 0; k < VEC; ++k) m0 = fmaxf(m0, fabsf((float)a[k]));
  }
  if (blockIdx.x == 0)
    for (int64_t j = nv * VEC + threadIdx.x; j < n; j += blockDim.x) m1 = fmaxf(m1, fabsf((float)x[j]));
  float m = block_reduce<true>(fmaxf(fmaxf(m0, m1), fmaxf(m2, m3)), red);
  if (threadIdx.x == 0) block_max[blockIdx.x] = m;
}

// split_kernel for cols % 8 == 0 and a 16-B aligned x: a thread splits 8
// consecutive columns of one row (vector loads) and writes their hi and lo
// halves as two 16-B stores (the scalar kernel's 2-B stores: 7.5 us for
// r_sqrt_sigma at C4).  Same values as split_kernel.
template <typename T>
__global__ __launch_bounds__(256) void split8_kernel(const T* __restrict__ x, int64_t rows,
                                                    int64_t cols, mpv_split16 out,
                                                    const float* __restrict__ bmax, int nb) {
  constexpr int VEC = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(VEC)));
  const float s = wave_pow2_scale(bmax, nb);
  if (blockIdx.x == 0 && threadIdx.x == 0) *out.scale = s;
  const int64_t g8 = (out.ld >> 1) / 8;  // 8-column groups per plane row
  const int64_t n = out.rows_pad * g8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / g8, c0 = (i - r * g8) * 8;
    float v[8];
    if (r < rows && c0 < cols) {  // cols % 8 == 0: all 8 columns are in range
      const vec_t* xv = reinterpret_cast<const vec_t*>(x + r * cols + c0);
#pragma unroll
      for (int q = 0; q < 8 / VEC; ++q) {
        const vec_t a = xv[q];
#pragma unroll
        for (int k = 0; k < VEC; ++k) v[q * VEC + k] = (float)a[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = 0.0f;
    }
    uint16_t h[8], l[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) split_f16(v[k], s, h[k], l[k]);
    const int64_t o = chunked_index(r, out.ld, c0);
    *reinterpret_cast<s16x8*>(out.data + o) =
        s16x8{(short)h[0], (short)h[1], (short)h[2], (short)h[3], (short)h[4], (short)h[5], (short)h[6], (short)h[7]};
    *reinterpret_cast<s16x8*>(out.data + o + kLoOff) =
        s16x8{(short)l[0], (short)l[1], (short)l[2], (short)l[3], (short)l[4], (short)l[5], (short)l[6], (short)l[7]};
  }
}

// (rows, cols) row-major -> chunked split planes (rows_pad x ld/2 columns),
// zero padded.  Thread i owns logical element (r, c) = (i / cols_pad, i % cols_pad).
// The scale comes from the nb block maxima of maxabs_kernel, taken by every
// wave itself (wave_pow2_scale: the same bits as a scale launch of its own,
// one launch fewer); block 0 publishes it.
template <typename T>
__global__ __launch_bounds__(256) void split_kernel(const T* __restrict__ x, int64_t rows,
                                                   int64_t cols, mpv_split16 out,
                                                   const float* __restrict__ bmax, int nb) {
  const float s = wave_pow2_scale(bmax, nb);
  if (blockIdx.x == 0 && threadIdx.x == 0) *out.scale = s;
  const int64_t cp = out.ld >> 1;
  const int64_t n = out.rows_pad * cp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cp, c = i - r * cp;
    const float v = (r < rows && c < cols) ? (float)x[r * cols + c] : 0.0f;
    uint16_t h, l;
    split_f16(v, s, h, l);
    const int64_t o = chunked_index(r, out.ld, c);
    out.data[o] = h;
    out.data[o + kLoOff] = l;
  }
}

// A small operand (r_sqrt_sigma at L, z <= 128): every workgroup takes max |x|
// over the whole input itself (at most kSplitSmall elements, L2-resident) and
// splits its own share of the planes: one launch instead of three, and the
// same scale bits in every workgroup (the max is exact in any order).
constexpr int64_t kSplitSmall = 16384;  // input elements

// (block `blk` of `nblk` doing this split; split_small_kernel's whole grid, or
// the extra workgroups of noise_philox16_kernel, mpv_noise_philox_f16_split)
template <typename T>
MPV_DEV void split_small_body(const T* __restrict__ x, int rows, int cols, const mpv_split16& out,
                              int blk, int nblk) {
  __shared__ float red[16];
  const int n = rows * cols, st = blockDim.x;
  // four independent chains (the loads in flight together; a max is exact in
  // any order)
  float m0 = 0.0f, m1 = 0.0f, m2 = 0.0f, m3 = 0.0f;
  int i = threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    m0 = fmaxf(m0, fabsf((float)x[i]));
    m1 = fmaxf(m1, fabsf((float)x[i + st]));
    m2 = fmaxf(m2, fabsf((float)x[i + 2 * st]));
    m3 = fmaxf(m3, fabsf((float)x[i + 3 * st]));
  }
  for (; i < n; i += st) m0 = fmaxf(m0, fabsf((float)x[i]));
  const float m = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
  const float s = pow2_scale(block_reduce<true>(m, red));
  if (blk == 0 && threadIdx.x == 0) *out.scale = s;
  const int cp = (int)(out.ld >> 1), np = (int)out.rows_pad * cp;
  for (int i = blk * blockDim.x + threadIdx.x; i < np; i += nblk * blockDim.x) {
    const int r = i / cp, c = i - r * cp;
    const float v = (r < rows && c < cols) ? (float)x[r * cols + c] : 0.0f;
    uint16_t h, l;
    split_f16(v, s, h, l);
    const int64_t o = chunked_index(r, out.ld, c);
    out.data[o] = h;
    out.data[o + kLoOff] = l;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void split_small_kernel(const T* __restrict__ x, int rows,
                                                         int cols, mpv_split16 out) {
  split_small_body<T>(x, rows, cols, out, blockIdx.x, gridDim.x);
}

// A small operand split riding on the noise launch (mpv_noise_philox_f16_split).
struct SmallSplit {
  const void* x;
  int f64, rows, cols;
  mpv_split16 out;
  int nblocks;  // the grid's last nblocks workgroups split; 0: none
};

// Philox noise straight into 3xf16 planes: plane row r = b*S_local + s holds
// the noise of (s, b) (same values as the fp32 (S, B, z) draw, rows reordered
// so that the s rows of one batch row are contiguous for the GEMMs).
// Box-Muller output is bounded by sqrt(-2 ln 2^-25) < 5.9, so the scale is
// the constant 2^12 (max |n| * s < 24200 < 65504).
constexpr float kNoiseScale = 4096.0f;

// A block makes kNoiseRows plane rows r = b*S + s; a thread makes 8
// consecutive columns at a time (two groups of 4: the 4 words of ONE Philox
// call when z % 4 == 0, else words of two calls), stored as two 16-B vectors.
// Planes narrower than 8 x blockDim columns give each row cols/8 threads and
// the block several rows at once.
#ifndef MPV_NOISE_ROWS
#define MPV_NOISE_ROWS 16
#endif
#ifndef MPV_NOISE_NT
#define MPV_NOISE_NT 0  // nontemporal plane stores: 1.69 -> 2.61 ms at C4 (r06_noise_ab.json)
#endif
constexpr int kNoiseRows = MPV_NOISE_ROWS;  // plane rows per block (1: 2.08 ms, 4: 1.99, 16: 1.93 at C4; 8, 32: as 16)
constexpr int kNoiseCols = 8;   // plane columns per thread (4: 1.78 ms, 8: 1.69 ms at C4)
#ifndef MPV_NOISE_PASSES
#define MPV_NOISE_PASSES 2
#endif
constexpr int kNoisePasses = MPV_NOISE_PASSES;  // narrow planes: row passes per block
// Plane columns the noise kernel writes: z rounded up to the GEMMs' 32-wide K
// slices (zeros past z).  Columns beyond that (the dR tile's padding) are left
// as they are: the forward GEMM never reads them, and in the dR GEMM they only
// meet output columns >= z, which are not stored.
__host__ __device__ inline int noise_written_cols(const mpv_split16& out, int z) {
  return (int)min(out.ld >> 1, (int64_t)((z + 31) / 32 * 32));
}

// Normals of columns c0 .. c0+7 (c0 % 8 == 0) of the plane row whose first
// global element is e_row; zero past z.  Element e draws normal e & 3 of
// Philox counter e >> 2; the row's first element is at phase sh (0 whenever
// z % 4 == 0; uniform over the row), so the 8 columns take normals sh..sh+7
// of two consecutive counters when aligned and of three otherwise (two
// 4-column groups made four calls, round 2).
MPV_DEV void noise16_oct(int64_t e_row, int c0, int z, uint64_t offset, uint32_t k0, uint32_t k1,
                         float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = 0.0f;
  if (c0 >= z) return;
  const int sh = (int)(e_row & 3);
  const uint64_t ctr = (uint64_t)((e_row + c0) >> 2) + offset;
  if (sh == 0) {  // aligned rows (z % 4 == 0): two counters, no selects
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const uint64_t c = ctr + g;
      const u32x4 w = philox4x32_10(u32x4{(uint32_t)c, (uint32_t)(c >> 32), 0u, 0u}, k0, k1);
      box_muller(w.x, w.y, v[4 * g], v[4 * g + 1]);
      box_muller(w.z, w.w, v[4 * g + 2], v[4 * g + 3]);
    }
#pragma unroll
    for (int i = 1; i < 8; ++i)
      if (c0 + i >= z) v[i] = 0.0f;  // padding columns of the last group
    return;
  }
  float a[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) a[i] = 0.0f;
  const u32x4 w0 = philox4x32_10(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u}, k0, k1);
  if (sh == 1) box_muller(w0.x, w0.y, a[0], a[1]);
  box_muller(w0.z, w0.w, a[2], a[3]);
  const uint64_t c1 = ctr + 1;
  const u32x4 w1 = philox4x32_10(u32x4{(uint32_t)c1, (uint32_t)(c1 >> 32), 0u, 0u}, k0, k1);
  box_muller(w1.x, w1.y, a[4], a[5]);
  box_muller(w1.z, w1.w, a[6], a[7]);
  {
    const uint64_t c2 = ctr + 2;
    const u32x4 w2 = philox4x32_10(u32x4{(uint32_t)c2, (uint32_t)(c2 >> 32), 0u, 0u}, k0, k1);
    box_muller(w2.x, w2.y, a[8], a[9]);
    if (sh == 3) box_muller(w2.z, w2.w, a[10], a[11]);
  }
  // v[i] = a[sh + i], sh in 1..3 (uniform per row: selects, not a dynamic index)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = sh == 1 ? a[i + 1] : (sh == 2 ? a[i + 2] : a[i + 3]);
    v[i] = c0 + i < z ? x : 0.0f;
  }
}

// Lanes per plane row of a narrow plane: the 8-column groups that hold normals.
__host__ __device__ inline int noise_narrow_tpr(int z) { return (z + kNoiseCols - 1) / kNoiseCols; }

// Zero columns c_first .. cols-1 (whole 8-column groups) of plane row r.
template <int CPT>
MPV_DEV void noise16_zero_tail(const mpv_split16& out, int r, int c_first, int cols) {
  for (int c0 = c_first; c0 < cols; c0 += CPT) {
    const int64_t o = chunked_index(r, out.ld, c0);
    *reinterpret_cast<s16x8*>(out.data + o) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    *reinterpret_cast<s16x8*>(out.data + o + kLoOff) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// Columns c_first, c_first + c_step, ... (CPT each, two 16-B stores) of
// plane row r.
template <int CPT>
MPV_DEV void noise16_row(const mpv_split16& out, int S, int B, int z, int64_t s_off, uint32_t k0,
                         uint32_t k1, uint64_t offset, int r, int c_first, int c_step) {
  const int bb = r / S, ss = r - bb * S;
  const int64_t e_row = ((s_off + ss) * B + bb) * (int64_t)z;  // first global element of the row
  const int cols = noise_written_cols(out, z);
  for (int c0 = c_first; c0 < cols; c0 += c_step) {
    static_assert(CPT == 8, "noise16_oct: 8 columns per thread");
    float v[CPT];
    noise16_oct(e_row, c0, z, offset, k0, k1, v);
    uint16_t h[CPT], l[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) split_f16(v[q], kNoiseScale, h[q], l[q]);
    static_assert(CPT == 8, "two 16-B stores per thread");
    const int64_t o = chunked_index(r, out.ld, c0);
    const s16x8 hv{(short)h[0], (short)h[1], (short)h[2], (short)h[3],
                   (short)h[4], (short)h[5], (short)h[6], (short)h[7]};
    const s16x8 lv{(short)l[0], (short)l[1], (short)l[2], (short)l[3],
                   (short)l[4], (short)l[5], (short)l[6], (short)l[7]};
#if MPV_NOISE_NT
    __builtin_nontemporal_store(hv, reinterpret_cast<s16x8*>(out.data + o));
    __builtin_nontemporal_store(lv, reinterpret_cast<s16x8*>(out.data + o + kLoOff));
#else
    *reinterpret_cast<s16x8*>(out.data + o) = hv;
    *reinterpret_cast<s16x8*>(out.data + o + kLoOff) = lv;
#endif
  }
}

__global__ __launch_bounds__(256) void noise_philox16_kernel(mpv_split16 out, int S, int B,
                                                            int z, int64_t s_off, uint32_t k0,
                                                            uint32_t k1, uint64_t offset,
                                                            int rows, int rpb,
                                                            const uint64_t* __restrict__ seed_dev,
                                                            SmallSplit ss) {
  // r_sqrt_sigma's split, beside the noise (one launch): the first workgroups,
  // so that they start with the noise's and finish under it
  if ((int)blockIdx.x < ss.nblocks) {
    if (ss.f64)
      split_small_body<double>((const double*)ss.x, ss.rows, ss.cols, ss.out, blockIdx.x,
                               ss.nblocks);
    else
      split_small_body<float>((const float*)ss.x, ss.rows, ss.cols, ss.out, blockIdx.x,
                              ss.nblocks);
    return;
  }
  const int nblk = (int)blockIdx.x - ss.nblocks;  // this workgroup's noise block
  philox_key(seed_dev, k0, k1);
  // the planes' constant scale (no launch of its own; the GEMMs that read it
  // run after this kernel)
  if (nblk == 0 && threadIdx.x == 0) *out.scale = kNoiseScale;
  const int cols = noise_written_cols(out, z);
  const int r_end = min(rows, (int)(nblk + 1) * rpb);
  constexpr int CPT = kNoiseCols;
  if (cols / CPT >= (int)blockDim.x) {  // wide planes: the row (and its index math) is block-uniform
    for (int r = nblk * rpb; r < r_end; ++r)
      noise16_row<CPT>(out, S, B, z, s_off, k0, k1, offset, r, threadIdx.x * CPT,
                       blockDim.x * CPT);
  } else {
    // narrow planes (C2, C3): a lane per 8 columns holding normals (the zero
    // columns z .. cols-1 past them are stored by the row's last lane, not
    // given lanes of their own), several rows per pass of the block
    const int tpr = noise_narrow_tpr(z);
    const int rpi = (int)blockDim.x / tpr;
    if ((int)threadIdx.x >= rpi * tpr) return;
    const int t = (int)threadIdx.x % tpr;
    for (int r = nblk * rpb + (int)threadIdx.x / tpr; r < r_end; r += rpi) {
      noise16_row<CPT>(out, S, B, z, s_off, k0, k1, offset, r, t * CPT, cols);
      if (t == tpr - 1) noise16_zero_tail<CPT>(out, r, tpr * CPT, cols);
    }
  }
}


static unsigned grid_for(int64_t n, int threads, int64_t cap = 65536) {
  int64_t g = cdiv(n, threads);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace mpv

using namespace mpv;

extern "C" {

int mpv_abi_version(void) { return MPV_ABI_VERSION; }

int mpv_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_timing = on != 0;
  return MPV_OK;
}

int mpv_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_tmu);
  for (auto& t : g_slots) t.used = 0;
  return MPV_OK;
}

int mpv_timing_query(const char* kernel, int64_t* launches, double* total_ms) {
  MPV_REQUIRE(kernel && launches && total_ms, "bad timing_query arguments");
  std::lock_guard<std::mutex> lk(g_tmu);
  *launches = 0;
  *total_ms = 0.0;
  for (auto& t : g_slots) {
    if (t.name != kernel) continue;
    for (size_t i = 0; i < t.used; ++i) {
      float ms = 0.0f;
      hipError_t e = hipEventSynchronize(t.stop[i]);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, t.start[i], t.stop[i]);
      if (e != hipSuccess) return fail(MPV_ELAUNCH, "timing %s: %s", kernel, hipGetErrorString(e));
      *total_ms += ms;
      *launches += 1;
    }
  }
  return MPV_OK;
}

const char* mpv_last_error(void) { return g_err; }

static int noise_philox(float* eps, const mpv_shape* shape, uint64_t seed,
                        const uint64_t* seed_dev, uint64_t offset, void* stream) {
  if (int rc = check_shape(shape)) return rc;
  MPV_REQUIRE(eps != nullptr, "eps is NULL");
  const int64_t per_s = shape->B * shape->z;
  const int64_t e_begin = shape->s_offset * per_s;
  const int64_t e_count = shape->S_local * per_s;
  const int64_t first = e_begin >> 2, last = (e_begin + e_count - 1) >> 2;
  const int64_t nthreads = last - first + 1;
  const int threads = 256;
  const int64_t blocks = std::min<int64_t>(cdiv(nthreads, threads), int64_t(1) << 22);
  MPV_LAUNCH("noise_philox", noise_philox_kernel, dim3((unsigned)blocks), dim3(threads), 0,
                     as_stream(stream), eps, e_begin, e_count, (uint32_t)seed,
                     (uint32_t)(seed >> 32), offset, seed_dev);
  return check_launch("noise_philox");
}

int mpv_noise_philox(float* eps, const mpv_shape* shape, uint64_t seed, uint64_t offset,
                     void* stream) {
  return noise_philox(eps, shape, seed, nullptr, offset, stream);
}

int mpv_noise_philox_dev(float* eps, const mpv_shape* shape, const uint64_t* seed_dev,
                         uint64_t offset, void* stream) {
  MPV_REQUIRE(seed_dev != nullptr, "seed_dev is NULL");
  return noise_philox(eps, shape, 0, seed_dev, offset, stream);
}

int mpv_philox_raw(uint32_t* out, int64_t n, uint64_t ctr0, uint64_t key, void* stream) {
  MPV_REQUIRE(out != nullptr && n > 0, "bad philox_raw arguments");
  MPV_LAUNCH("philox_raw", philox_raw_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), out, n, ctr0, (uint32_t)key, (uint32_t)(key >> 32));
  return check_launch("philox_raw");
}

static int check_split(const mpv_split16* o) {
  MPV_REQUIRE(o && o->data && o->scale, "NULL pointer in mpv_split16");
  MPV_REQUIRE(o->rows_pad > 0 && o->ld > 0 && (o->ld % 64) == 0, "mpv_split16: ld must be a "
              "positive multiple of 64 (got %lld)", (long long)o->ld);
  return MPV_OK;
}

size_t mpv_split_workspace_bytes(void) { return sizeof(float) * kMaxBlocks; }

int mpv_split_f16(const void* x, int x_dtype, int64_t rows, int64_t cols, const mpv_split16* out,
                  void* workspace, void* stream) {
  if (int rc = check_split(out)) return rc;
  MPV_REQUIRE(x && workspace && rows > 0 && cols > 0, "bad mpv_split_f16 arguments");
  MPV_REQUIRE(rows <= out->rows_pad && cols <= out->ld / 2, "planes smaller than the input");
  MPV_REQUIRE(x_dtype == MPV_F32 || x_dtype == MPV_F64, "unsupported dtype %d", x_dtype);
  hipStream_t s = as_stream(stream);
  const int64_t plane_elems = out->rows_pad * (out->ld / 2);
  if (rows * cols <= kSplitSmall && plane_elems < (int64_t(1) << 31)) {
    const dim3 g((unsigned)std::min<int64_t>(cdiv(plane_elems, 256 * 4), 256));
    if (x_dtype == MPV_F64)
      MPV_LAUNCH("split", split_small_kernel<double>, g, dim3(256), 0, s, (const double*)x,
                 (int)rows, (int)cols, *out);
    else
      MPV_LAUNCH("split", split_small_kernel<float>, g, dim3(256), 0, s, (const float*)x,
                 (int)rows, (int)cols, *out);
    return check_launch("split_f16");
  }
  float* bmax = reinterpret_cast<float*>(workspace);
  const int64_t n = rows * cols;
  const unsigned g = grid_for(n, 256, kSplitMaxBlocks);
  const bool aligned = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const bool f64 = x_dtype == MPV_F64;
  if (aligned && f64)
    MPV_LAUNCH("split", maxabs_vec_kernel<double>, dim3(g), dim3(256), 0, s, (const double*)x, n, bmax);
  else if (aligned)
    MPV_LAUNCH("split", maxabs_vec_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, n, bmax);
  else if (f64)
    MPV_LAUNCH("split", maxabs_kernel<double>, dim3(g), dim3(256), 0, s, (const double*)x, n, bmax);
  else
    MPV_LAUNCH("split", maxabs_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)x, n, bmax);
  if (aligned && cols % 8 == 0) {  // whole 8-column groups: vector loads, 16-B stores
    const unsigned g2 = grid_for(out->rows_pad * (out->ld / 2) / 8, 256, 16384);
    if (f64)
      MPV_LAUNCH("split", split8_kernel<double>, dim3(g2), dim3(256), 0, s, (const double*)x, rows,
                 cols, *out, bmax, (int)g);
    else
      MPV_LAUNCH("split", split8_kernel<float>, dim3(g2), dim3(256), 0, s, (const float*)x, rows,
                 cols, *out, bmax, (int)g);
    return check_launch("split_f16");
  }
  const unsigned g2 = grid_for(out->rows_pad * (out->ld / 2), 256, 16384);
  if (f64)
    MPV_LAUNCH("split", split_kernel<double>, dim3(g2), dim3(256), 0, s, (const double*)x, rows,
               cols, *out, bmax, (int)g);
  else
    MPV_LAUNCH("split", split_kernel<float>, dim3(g2), dim3(256), 0, s, (const float*)x, rows,
               cols, *out, bmax, (int)g);
  return check_launch("split_f16");
}

static int noise_philox_f16(const mpv_shape* shape, uint64_t seed, const uint64_t* seed_dev,
                            uint64_t offset, const mpv_split16* out, void* stream,
                            SmallSplit ss = SmallSplit{}) {
  if (int rc = check_shape(shape)) return rc;
  if (int rc = check_split(out)) return rc;
  const int64_t rows = shape->S_local * shape->B;
  MPV_REQUIRE(out->rows_pad >= rows && out->ld / 2 >= shape->z, "noise planes too small");
  hipStream_t s = as_stream(stream);
  MPV_REQUIRE(rows < (int64_t(1) << 31) && shape->z < (int64_t(1) << 31), "noise too large");
  const int64_t tpr = noise_written_cols(*out, (int)shape->z) / kNoiseCols;  // threads per plane row
  // narrow planes (fewer than 256 8-column groups per row): 256-thread blocks
  // of several rows per pass, kNoisePasses passes (short one-wave blocks were
  // dispatch-bound at C2)
  const bool narrow = tpr < 256 && !(tpr % 64 == 0);
  const unsigned threads = narrow || tpr >= 256 ? 256 : (unsigned)tpr;
  int rpb = kNoiseRows;
  if (narrow) rpb = (256 / noise_narrow_tpr((int)shape->z)) * kNoisePasses;
  if (ss.x != nullptr) {
    const int64_t plane_elems = ss.out.rows_pad * (ss.out.ld / 2);
    ss.nblocks = (int)std::min<int64_t>(cdiv(plane_elems, (int64_t)threads * 8), 64);
  }
  const int64_t nb = cdiv(rows, rpb) + ss.nblocks;
  MPV_REQUIRE(nb < (int64_t(1) << 31), "noise grid too large");
  MPV_LAUNCH("noise_philox", noise_philox16_kernel, dim3((unsigned)nb), dim3(threads), 0, s, *out,
             (int)shape->S_local, (int)shape->B, (int)shape->z, shape->s_offset, (uint32_t)seed,
             (uint32_t)(seed >> 32), offset, (int)rows, rpb, seed_dev, ss);
  return check_launch("noise_philox_f16");
}

int mpv_noise_philox_f16(const mpv_shape* shape, uint64_t seed, uint64_t offset,
                         const mpv_split16* out, void* stream) {
  return noise_philox_f16(shape, seed, nullptr, offset, out, stream);
}

int mpv_noise_philox_f16_dev(const mpv_shape* shape, const uint64_t* seed_dev, uint64_t offset,
                             const mpv_split16* out, void* stream) {
  MPV_REQUIRE(seed_dev != nullptr, "seed_dev is NULL");
  return noise_philox_f16(shape, 0, seed_dev, offset, out, stream);
}

int mpv_noise_philox_f16_split(const mpv_shape* shape, uint64_t seed, const uint64_t* seed_dev,
                               uint64_t offset, const mpv_split16* out, const void* x,
                               int x_dtype, int64_t rows, int64_t cols,
                               const mpv_split16* x_out, void* stream) {
  if (int rc = check_split(x_out)) return rc;
  MPV_REQUIRE(x && rows > 0 && cols > 0 && rows * cols <= kSplitSmall,
              "the split rides on the noise launch for at most %lld elements",
              (long long)kSplitSmall);
  MPV_REQUIRE(rows <= x_out->rows_pad && cols <= x_out->ld / 2, "planes smaller than the input");
  MPV_REQUIRE(x_out->rows_pad * (x_out->ld / 2) < (int64_t(1) << 31), "planes too large");
  MPV_REQUIRE(x_dtype == MPV_F32 || x_dtype == MPV_F64, "unsupported dtype %d", x_dtype);
  SmallSplit ss{x, x_dtype == MPV_F64, (int)rows, (int)cols, *x_out, 0};
  return noise_philox_f16(shape, seed, seed_dev, offset, out, stream, ss);
}

int mpv_convert(const void* src, int sd, void* dst, int dd, int64_t n, void* stream) {
  MPV_REQUIRE(src && dst && n >= 0, "bad convert arguments");
  MPV_REQUIRE((sd == MPV_F32 || sd == MPV_F64) && (dd == MPV_F32 || dd == MPV_F64),
              "unsupported dtype pair %d -> %d", sd, dd);
  if (n == 0) return MPV_OK;
  const unsigned g = grid_for(n, 256);
  hipStream_t s = as_stream(stream);
  if (sd == MPV_F64 && dd == MPV_F32)
    MPV_LAUNCH("convert", (convert_kernel<double, float>), dim3(g), dim3(256), 0, s,
                       (const double*)src, (float*)dst, n);
  else if (sd == MPV_F32 && dd == MPV_F64)
    MPV_LAUNCH("convert", (convert_kernel<float, double>), dim3(g), dim3(256), 0, s,
                       (const float*)src, (double*)dst, n);
  else if (sd == MPV_F32)
    MPV_LAUNCH("convert", (convert_kernel<float, float>), dim3(g), dim3(256), 0, s,
                       (const float*)src, (float*)dst, n);
  else
    MPV_LAUNCH("convert", (convert_kernel<double, double>), dim3(g), dim3(256), 0, s,
                       (const double*)src, (double*)dst, n);
  return check_launch("convert");
}

int mpv_bstat_combine(const float* gathered, int64_t nshards, int64_t B, float* out,
                      void* stream) {
  MPV_REQUIRE(gathered && out && nshards > 0 && B > 0, "bad bstat_combine arguments");
  MPV_LAUNCH("bstat_combine", bstat_combine_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0,
                     as_stream(stream), gathered, nshards, B, out);
  return check_launch("bstat_combine");
}

int mpv_reparam_fwd(const mpv_reparam_args* a, void* stream) {
  MPV_REQUIRE(a != nullptr && a->n_e >= 0 && a->n_x >= 0, "bad reparam arguments");
  MPV_REQUIRE(a->n_e == 0 || (a->mu_e && a->logvar_e && a->eps_e && a->z_e), "label encoder NULL");
  MPV_REQUIRE(a->n_x == 0 || (a->mu_x && a->logvar_x && a->eps_x && a->z_x), "feat encoder NULL");
  const int64_t n = a->n_e + a->n_x;
  if (n == 0) return MPV_OK;
  MPV_LAUNCH("reparam_fwd", reparam_fwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), *a);
  return check_launch("reparam_fwd");
}

int mpv_reparam_bwd(const mpv_reparam_bwd_args* a, void* stream) {
  MPV_REQUIRE(a != nullptr && a->n_e >= 0 && a->n_x >= 0, "bad reparam_bwd arguments");
  MPV_REQUIRE(a->n_e == 0 || (a->logvar_e && a->eps_e && a->gmu_e && a->glogvar_e),
              "label encoder NULL");
  MPV_REQUIRE(a->n_x == 0 || (a->logvar_x && a->eps_x && a->gmu_x && a->glogvar_x),
              "feat encoder NULL");
  const int64_t n = a->n_e + a->n_x;
  if (n == 0) return MPV_OK;
  MPV_LAUNCH("reparam_bwd", reparam_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), *a);
  return check_launch("reparam_bwd");
}

int mpv_kl_bwd(const mpv_kl_bwd_args* a, void* stream) {
  MPV_REQUIRE(a && a->fe_mu && a->fe_logvar && a->fx_mu && a->fx_logvar && a->gscal &&
                  a->g_fe_mu && a->g_fe_logvar && a->g_fx_mu && a->g_fx_logvar,
              "bad kl_bwd arguments");
  MPV_REQUIRE(a->B > 0 && a->d > 0, "bad kl_bwd sizes");
  MPV_LAUNCH("kl_bwd", kl_bwd_kernel, dim3(grid_for(a->B * a->d, 256, 4096)), dim3(256), 0,
                     as_stream(stream), *a);
  return check_launch("kl_bwd");
}

}  // extern "C"

namespace mpv {
// Used by the forward / backward translation units.

static SlabSum slab_problem(const float* in, int64_t nslab, int64_t n, void* out, int out_dtype) {
  SlabSum q;
  q.in = in;
  q.nslab = nslab;
  q.n = n;
  q.out = out;
  q.f64 = out_dtype == MPV_F64;
  q.split = nslab >= 64 && n <= 256 * 256;  // the rule of launch_sum_slabs
  q.vec = !q.split && n % 4 == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  q.blocks = q.split ? cdiv(n, 64) : (q.vec ? cdiv(n, 4096) : cdiv(n, 1024));
  return q;
}

int launch_sum_slabs_pair(const float* in0, int64_t nslab0, int64_t n0, void* out0,
                          int out0_dtype, const float* in1, int64_t nslab1, int64_t n1,
                          void* out1, int out1_dtype, hipStream_t s) {
  const SlabSum a = slab_problem(in0, nslab0, n0, out0, out0_dtype);
  const SlabSum b = slab_problem(in1, nslab1, n1, out1, out1_dtype);
  MPV_REQUIRE(a.blocks + b.blocks < (int64_t(1) << 31), "slab sums too large");
  MPV_LAUNCH("sum_slabs", sum_slabs_pair_kernel, dim3((unsigned)(a.blocks + b.blocks)), dim3(1024),
             0, s, a, b);
  return check_launch("sum_slabs");
}

int launch_sum_slabs(const float* in, int64_t nslab, int64_t n, void* out, int out_dtype,
                     hipStream_t s) {
  if (nslab >= 64 && n <= 256 * 256) {  // too few columns to hide the slab chain
    const unsigned gs = (unsigned)((n + 63) / 64);
    if (out_dtype == MPV_F64)
      MPV_LAUNCH("sum_slabs", (sum_slabs_split_kernel<double>), dim3(gs), dim3(1024), 0, s, in,
                 nslab, n, (double*)out);
    else
      MPV_LAUNCH("sum_slabs", (sum_slabs_split_kernel<float>), dim3(gs), dim3(1024), 0, s, in,
                 nslab, n, (float*)out);
    return check_launch("sum_slabs");
  }
  const unsigned g = grid_for(n, 256, 8192);
  if (out_dtype == MPV_F64)
    MPV_LAUNCH("sum_slabs", (sum_slabs_kernel<double>), dim3(g), dim3(256), 0, s, in, nslab, n,
                       (double*)out);
  else
    MPV_LAUNCH("sum_slabs", (sum_slabs_kernel<float>), dim3(g), dim3(256), 0, s, in, nslab, n,
                       (float*)out);
  return check_launch("sum_slabs");
}
}  // namespace mpv
