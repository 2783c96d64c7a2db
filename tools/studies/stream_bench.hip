// Microbenchmark of the element pass's memory stream (study tool, not product
// code): T (fp32, rows of L floats) is read once and the G planes (chunked
// 3xf16 split: every 32 columns = 32 hi halves then 32 lo halves) are written
// once, 8 bytes per element in all, at C4's shape (B 512 x S 4096 rows of
// L 1024).  Variants of the access pattern, no element math:
//   copy4   : float4 read, float4 write of the same bytes (the reference rate)
//   elem4   : bwd_elem's pattern: a lane owns 4 columns: one 16-B T load,
//             two 8-B plane stores (hi, lo) per row
//   elem8   : a lane owns 8 columns: two 16-B T loads, two 16-B plane stores
//   elem4x2 : as elem4 with two rows per iteration (more loads in flight)
// each with default and nontemporal policy.  Prints TB/s of (read + write).
//
//   hipcc --offload-arch=gfx950 -O3 tools/studies/stream_bench.hip -o scratch/stream_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int B = 512, S = 4096, L = 1024;
constexpr int ROWS_PER_BLOCK = 256;

__device__ __forceinline__ void split4(f32x4 v, s16x4& h, s16x4& l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x = v[i] * 4096.0f;
    const _Float16 hh = (_Float16)x;
    const _Float16 ll = (_Float16)(x - (float)hh);
    h[i] = __builtin_bit_cast(short, hh);
    l[i] = __builtin_bit_cast(short, ll);
  }
}

template <typename T>
__device__ __forceinline__ T ld(const T* p, bool nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T>
__device__ __forceinline__ void st(T* p, T v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const float* __restrict__ T, void* __restrict__ out) {
  const int b = blockIdx.x, sc = blockIdx.y, tid = threadIdx.x;
  const int64_t row0 = (int64_t)b * S + (int64_t)sc * ROWS_PER_BLOCK;
  if (MODE == 0) {  // copy4
    float* o = (float*)out;
    for (int r = 0; r < ROWS_PER_BLOCK; ++r) {
      const int64_t off = (row0 + r) * L + tid * 4;
      st((f32x4*)(o + off), ld((const f32x4*)(T + off), NT), NT);
    }
  } else if (MODE == 1 || MODE == 3) {  // elem4 (one or two rows per iteration)
    uint16_t* g = (uint16_t*)out;
    const int c0 = tid * 4;
    const int64_t cidx = ((c0 >> 5) << 6) + (c0 & 31);
    constexpr int RPI = MODE == 3 ? 2 : 1;
    for (int r = 0; r < ROWS_PER_BLOCK; r += RPI) {
      f32x4 v[RPI];
#pragma unroll
      for (int k = 0; k < RPI; ++k) v[k] = ld((const f32x4*)(T + (row0 + r + k) * L + c0), NT);
#pragma unroll
      for (int k = 0; k < RPI; ++k) {
        s16x4 h, l;
        split4(v[k], h, l);
        uint16_t* p = g + (row0 + r + k) * (2 * L) + cidx;
        st((s16x4*)p, h, NT);
        st((s16x4*)(p + 32), l, NT);
      }
    }
  } else {  // elem8: 512 lanes' worth of columns: two rows per block pass
    uint16_t* g = (uint16_t*)out;
    const int half = tid >> 7, c0 = (tid & 127) * 8;
    const int64_t cidx = ((c0 >> 5) << 6) + (c0 & 31);
    for (int r = half; r < ROWS_PER_BLOCK; r += 2) {
      const float* src = T + (row0 + r) * L + c0;
      const f32x4 a = ld((const f32x4*)src, NT), c = ld((const f32x4*)(src + 4), NT);
      s16x4 h0, l0, h1, l1;
      split4(a, h0, l0);
      split4(c, h1, l1);
      const s16x8 h{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      const s16x8 l{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      uint16_t* p = g + (row0 + r) * (2 * L) + cidx;
      st((s16x8*)p, h, NT);
      st((s16x8*)(p + 32), l, NT);
    }
  }
}

template <int MODE, bool NT>
static void run(const char* name, const float* T, void* out) {
  const dim3 grid(B, S / ROWS_PER_BLOCK);
  stream_kernel<MODE, NT><<<grid, 256>>>(T, out);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(a);
    stream_kernel<MODE, NT><<<grid, 256>>>(T, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  const double bytes = 8.0 * B * (double)S * L;
  printf("%-8s %-3s %.3f ms  %.2f TB/s\n", name, NT ? "nt" : "def", best, bytes / best / 1e9);
}

int main() {
  const size_t n = (size_t)B * S * L;
  float* T;
  void* out;
  if (hipMalloc(&T, n * 4) != hipSuccess || hipMalloc(&out, n * 4) != hipSuccess) return 1;
  (void)hipMemset(T, 0x3c, n * 4);
  run<0, false>("copy4", T, out);
  run<0, true>("copy4", T, out);
  run<1, false>("elem4", T, out);
  run<1, true>("elem4", T, out);
  run<3, false>("elem4x2", T, out);
  run<3, true>("elem4x2", T, out);
  run<2, false>("elem8", T, out);
  run<2, true>("elem8", T, out);
  (void)hipFree(T);
  (void)hipFree(out);
  return 0;
}
