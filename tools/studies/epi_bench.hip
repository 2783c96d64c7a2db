// Microbenchmark of the forward epilogue's element math (study tool, not
// product code): what bounds the VALU part of probit_fwd16a's epilogue?
//
// Every wave runs ITER iterations of one epilogue "sample block" exactly as
// fwd_tile_epilogue_t does it for 4 labels x 2 branches (probit_w2xN_zq<4>,
// the BCE operand and ranking exponent by op_sel broadcasts, exp2, the
// 4-label log, the P / N and column-sum accumulations) on register data, in
// variants that drop one class of instruction at a time.  Prints cycles per
// block per SIMD (s_memtime of the slowest wave) for 1 and 2 waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -I../../mpvae-1_amd/csrc -I../../include \
//         tools/studies/epi_bench.hip -o scratch/epi_bench && scratch/epi_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "mpv_common.h"

using namespace mpv;

// a * b[H] + c[H] (as probit_fwd.hip)
template <int H>
__device__ __forceinline__ f32x2 bc_fma(f32x2 a, f32x2 b, f32x2 c) {
  f32x2 d;
  if (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[1,1,1]"
        : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// VAR bits: 1 = no transcendentals (exp2 / log / rcp -> an fma),
//           2 = no ranking exponential, 4 = no BCE log, 8 = two sample blocks
//           per iteration (8 independent chains instead of 4)
template <int VAR>
__device__ __forceinline__ float tr_exp(float x) {
  if (VAR & 1) return fmaf(x, 0.5f, 1.0f);
  return __builtin_amdgcn_exp2f(x);
}
template <int VAR>
__device__ __forceinline__ float tr_rcp(float x) {
  if (VAR & 1) return fmaf(x, -0.25f, 1.5f);
  return __builtin_amdgcn_rcpf(x);
}

template <int VAR, int NB>
__device__ __forceinline__ void block(const f32x4 (&t4)[NB], const f32x2 (&fex)[4], const f32x2 (&qa2)[2],
                                      const f32x2 (&qb2)[2], const f32x2 (&sga2)[2],
                                      const f32x2 (&sgb2)[2], const f32x2 (&wp2)[2],
                                      const f32x2 (&wn2)[2], f32x2 (&sl)[NB], f32x2 (&sp)[NB],
                                      f32x2 (&sn)[NB], f32x2 (&ce)[4]) {
#pragma clang fp contract(off)
  constexpr float kL2e = 1.4426950408889634f;
  constexpr float c[7] = {-0.139353514f * kL2e, 0.777093824f * kL2e, -1.58356997f * kL2e,
                          1.19629222f * kL2e,  -0.0702797193f * kL2e, 1.09342452f * kL2e,
                          -1.27360696f * kL2e};
  constexpr int N = 4 * NB;
  f32x2 zq[N], t[N], p[N], w[N];
#pragma unroll
  for (int j = 0; j < N; ++j) zq[j] = pk_fma(splat2(t4[j / 4][j % 4]), splat2(kZq), fex[j % 4]);
#pragma unroll
  for (int j = 0; j < N; ++j)
    t[j] = f32x2{tr_rcp<VAR>(fmaf(0.5f / kSqL2e, fabsf(zq[j].x), 1.0f)),
                 tr_rcp<VAR>(fmaf(0.5f / kSqL2e, fabsf(zq[j].y), 1.0f))};
#pragma unroll
  for (int j = 0; j < N; ++j) p[j] = pk_fma(t[j], splat2(c[0]), splat2(c[1]));
#pragma unroll
  for (int k = 2; k < 7; ++k)
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = pk_fma(t[j], p[j], splat2(c[k]));
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 a = pk_fma(-zq[j], zq[j], p[j]);
    const f32x2 erfc = t[j] * f32x2{tr_exp<VAR>(a.x), tr_exp<VAR>(a.y)};
    const f32x2 om = splat2(1.0f) - erfc;
    w[j] = splat2(1.0f) + f32x2{__builtin_copysignf(om.x, zq[j].x), __builtin_copysignf(om.y, zq[j].y)};
  }
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    f32x2 q[4], r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x2 ww = w[4 * n + i];
      q[i] = (i & 1) ? bc_fma<1>(ww, qa2[i >> 1], qb2[i >> 1]) : bc_fma<0>(ww, qa2[i >> 1], qb2[i >> 1]);
      const f32x2 a = (i & 1) ? bc_fma<1>(ww, sga2[i >> 1], sgb2[i >> 1])
                              : bc_fma<0>(ww, sga2[i >> 1], sgb2[i >> 1]);
      r[i] = (VAR & 2) ? a : f32x2{tr_exp<VAR>(a.x), tr_exp<VAR>(a.y)};
    }
    const f32x2 q4 = (q[0] * q[1]) * (q[2] * q[3]);
    const f32x2 lp = (VAR & 4) ? q4
                               : ((VAR & 1) ? q4 * 0.5f
                                            : f32x2{__builtin_amdgcn_logf(q4.x), __builtin_amdgcn_logf(q4.y)});
    sl[n] = sl[n] + lp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sp[n] = pk_fma(splat2(wp2[i >> 1][i & 1]), r[i], sp[n]);
      sn[n] = pk_fma(splat2(wn2[i >> 1][i & 1]), r[i], sn[n]);
      ce[i] = ce[i] + w[4 * n + i];
    }
  }
}

template <int VAR, int NB>
__global__ __launch_bounds__(512) void epi_kernel(float* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  const float base = 0.001f * (float)(threadIdx.x + blockIdx.x);
  f32x4 t4[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n)
    t4[n] = f32x4{base - 1.5f + n, base - 0.5f, base + 0.5f, base + 1.5f};
  f32x2 fex[4], qa2[2], qb2[2], sga2[2], sgb2[2], wp2[2], wn2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) fex[i] = f32x2{0.1f * i + base, -0.1f * i - base};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    qa2[i] = f32x2{-kEh, kEh};
    qb2[i] = f32x2{1.0f - kC0, kC0};
    sga2[i] = f32x2{5.0f * kEh, -5.0f * kEh};
    sgb2[i] = f32x2{5.0f * kC0, -5.0f * kC0};
    wp2[i] = f32x2{0.0f, 1.0f};
    wn2[i] = f32x2{1.0f, 0.0f};
  }
  f32x2 sl[NB], sp[NB], sn[NB], ce[4];
#pragma unroll
  for (int n = 0; n < NB; ++n) sl[n] = sp[n] = sn[n] = splat2(0.0f);
#pragma unroll
  for (int i = 0; i < 4; ++i) ce[i] = splat2(0.0f);
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    block<VAR, NB>(t4, fex, qa2, qb2, sga2, sgb2, wp2, wn2, sl, sp, sn, ce);
#pragma unroll
    for (int n = 0; n < NB; ++n) t4[n] = t4[n] + 1e-7f;  // a new block each iteration
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.0f;
#pragma unroll
  for (int n = 0; n < NB; ++n) acc += sl[n].x + sl[n].y + sp[n].x + sn[n].y;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc += ce[i].x + ce[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int VAR, int NB>
static void run(const char* name, int threads, float* out, long long* cyc, long long* h) {
  const int iters = 2000, blocks = 256;
  epi_kernel<VAR, NB><<<blocks, threads>>>(out, cyc, iters);  // warm-up
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  epi_kernel<VAR, NB><<<blocks, threads>>>(out, cyc, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const int nw = blocks * threads / 64;
  hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
  long long mx = 0;
  double avg = 0;
  for (int i = 0; i < nw; ++i) {
    mx = h[i] > mx ? h[i] : mx;
    avg += h[i];
  }
  avg /= nw;
  const int wps = threads / 256;  // waves per SIMD
  // cycles per sample block (4 labels x 2 branches per lane) per SIMD:
  // the SIMD runs wps waves x iters x NB blocks in the slowest wave's time
  printf("%-34s waves/SIMD %d: %7.1f cyc/block/SIMD (max wave), %7.1f (avg), %.3f ms\n", name, wps,
         (double)mx / (iters * NB * wps), avg / (iters * NB * wps), ms);
}

int main() {
  float* out;
  long long *cyc, *h = new long long[256 * 8];
  hipMalloc(&out, sizeof(float) * 256 * 512);
  hipMalloc(&cyc, sizeof(long long) * 256 * 8);
  for (int threads : {256, 512}) {
    run<0, 1>("full (as the epilogue)", threads, out, cyc, h);
    run<1, 1>("no transcendentals", threads, out, cyc, h);
    run<2, 1>("no ranking exp", threads, out, cyc, h);
    run<4, 1>("no BCE log", threads, out, cyc, h);
    run<0, 2>("full, 2 blocks interleaved", threads, out, cyc, h);
    run<1, 2>("no transcendentals, 2 blocks", threads, out, cyc, h);
  }
  hipFree(out);
  hipFree(cyc);
  return 0;
}
