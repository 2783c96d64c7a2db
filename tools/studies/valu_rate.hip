// VALU issue rates on gfx950: v_fma_f32 vs v_pk_fma_f32 vs v_exp_f32, 8
// independent chains per wave, 1 or 2 waves per SIMD.  Relative times of the
// same instruction count tell whether packed fp32 issues at full rate.
// hipcc --offload-arch=gfx950 -O3 tools/studies/valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
  float c[8];
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c[i]) : "v"(a), "v"(b));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk(float* out, float a, float b) {
  f32x2 c[8];
  const f32x2 av{a, a}, bv{b, b};
  for (int i = 0; i < 8; ++i) c[i] = f32x2{(float)threadIdx.x + i, (float)i};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[i]) : "v"(av), "v"(bv));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += c[i].x + c[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_exp(float* out, float a, float b) {
  float c[8];
  for (int i = 0; i < 8; ++i) c[i] = (threadIdx.x + i) * 1e-3f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(c[i]));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mad64(float* out, float a, float b) {
  uint64_t c[8];
  const uint32_t m = 0xD2511F53u;
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t lo = (uint32_t)c[i];
      uint64_t carry;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c[i]), "=s"(carry) : "v"(lo), "s"(m));
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += (float)(c[i] & 0xffff);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mulhi(float* out, float a, float b) {
  uint32_t c[8];
  const uint32_t m = 0xD2511F53u;
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(c[i]) : "s"(m));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += (float)(c[i] & 0xffff);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_xor(float* out, float a, float b) {
  uint32_t c[8];
  const uint32_t m = 0xD2511F53u;
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(c[i]) : "s"(m));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += (float)(c[i] & 0xffff);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
float run(K k, int blocks, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1.0001f, 1e-7f);  // warm-up
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1.0001f, 1e-7f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* d;
  hipMalloc(&d, sizeof(float) * 256 * cus * 8);
  for (int wps = 1; wps <= 2; ++wps) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
    const int blocks = cus * wps;
    const double winst = (double)blocks * 4 * ITERS * 8;  // wave-instructions per launch
    const double per_simd = winst / (cus * 4);
    const float tf = run(k_fma, blocks, d), tp = run(k_pk, blocks, d), te = run(k_exp, blocks, d);
    const float tm = run(k_mad64, blocks, d), th = run(k_mulhi, blocks, d), tx = run(k_xor, blocks, d);
    // ns per wave-instruction per SIMD
    printf("waves/SIMD %d: v_fma_f32 %.3f ns/instr/SIMD, v_pk_fma_f32 %.3f, v_exp_f32 %.3f, "
           "v_mad_u64_u32 %.3f, v_mul_hi_u32 %.3f, v_xor_b32 %.3f\n",
           wps, tf * 1e6 / per_simd, tp * 1e6 / per_simd, te * 1e6 / per_simd, tm * 1e6 / per_simd,
           th * 1e6 / per_simd, tx * 1e6 / per_simd);
  }
  hipFree(d);
  return 0;
}
