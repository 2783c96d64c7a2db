// Shared device helpers for the MPVAE probit-ELBO kernels (gfx950 / CDNA4).
//
// Wave size is 64 everywhere.  Reductions inside a 16-lane MFMA row use DPP
// row shifts (no LDS round trip); cross-row / cross-wave reductions go
// through __shfl_xor (ds_bpermute) or LDS.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpvae_hip.h"

#define MPV_DEV __device__ __forceinline__

namespace mpv {

// ---- constants of the reference ELBO (mpvae.py:156,177,180,118,148) -------
// eps1 = tensor([1e-6]).float(); E = cdf*(1-eps1) + eps1*0.5 evaluated in fp32
constexpr float kEps1 = 1e-6f;
constexpr float kC1 = 1.0f - kEps1;        // (1 - eps1) rounded to fp32
constexpr float kC0 = kEps1 * 0.5f;        // eps1 * 0.5
constexpr float kInvSqrt2 = 0.70710678118654752440f;
constexpr float kInvSqrt2Pi = 0.39894228040143267794f;
constexpr float kKlEps = 1e-6f;
constexpr float kKlWeight = 1.1f;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Probit probability of reference mpvae.py:171-180 (torch Normal.cdf) with the
// ocml erf: E = 0.5 (1 + erf(u/sqrt2)) (1-1e-6) + 0.5e-6.  Reference-exact
// formula, ~40 VALU ops with the piecewise erf; kept for A/B checks.
MPV_DEV float probit_prob_erf(float u) {
  float cdf = 0.5f * (1.0f + erff(u * kInvSqrt2));
  return cdf * kC1 + kC0;
}

// Hardware transcendentals (v_exp_f32 / v_log_f32 are base 2).
MPV_DEV float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
MPV_DEV float fast_log(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }
MPV_DEV float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// E of reference mpvae.py:171-180 with a branch-free erf: erfc(z), z = |u|/sqrt2,
// from the Chebyshev fit of Numerical Recipes' erfcc, t exp(-z^2 + P(t)),
// t = 1/(1 + z/2), relative error < 1.2e-7 for all z >= 0 (~20 VALU ops
// against ~40 for the piecewise ocml erff).  erf = +-(1 - erfc) and
// E = 0.5 (1 + erf) (1 - 1e-6) + 0.5e-6 are then formed with IEEE fp32 ops in
// the reference's order, so E carries the reference's own quantisation: near
// saturation 1 + erf(x) rounds E to multiples of 2^-25, and the gradient's 1/E
// and 1/(1-E) factors see the same E as the reference does.  Also returns the
// normal density phi(u) = exp(-z^2)/sqrt(2 pi) for the backward.
MPV_DEV float probit_eval(float u, float& phi) {
  const float z = fabsf(u) * kInvSqrt2;
  const float t = fast_rcp(fmaf(0.5f, z, 1.0f));
  float p = fmaf(t, 0.17087277f, -0.82215223f);
  p = fmaf(t, p, 1.48851587f);
  p = fmaf(t, p, -1.13520398f);
  p = fmaf(t, p, 0.27886807f);
  p = fmaf(t, p, -0.18628806f);
  p = fmaf(t, p, 0.09678418f);
  p = fmaf(t, p, 0.37409196f);
  p = fmaf(t, p, 1.00002368f);
  p = fmaf(t, p, -1.26551223f);
  const float ez = fast_exp(-z * z);
  phi = ez * kInvSqrt2Pi;
  const float erfc_z = t * ez * fast_exp(p);
  const float erf_u = u < 0.0f ? __fsub_rn(erfc_z, 1.0f) : __fsub_rn(1.0f, erfc_z);
  const float cdf = __fmul_rn(0.5f, __fadd_rn(1.0f, erf_u));
  return __fadd_rn(__fmul_rn(cdf, kC1), kC0);
}

MPV_DEV float probit_prob(float u) {
  float phi;
  return probit_eval(u, phi);
}

// ---- packed fp32 (v_pk_fma/mul/add_f32: two lanes' worth per issue) -------
typedef float f32x2 __attribute__((ext_vector_type(2)));

MPV_DEV f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
MPV_DEV f32x2 splat2(float v) { return f32x2{v, v}; }

// probit_eval of the label and feature branches at once (every step is the
// same for both), bit-identical to two probit_eval calls: the fused steps are
// explicit fmas and the reference-order steps stay separately rounded.
MPV_DEV f32x2 probit_eval2(f32x2 u, f32x2& phi) {
#pragma clang fp contract(off)
  const f32x2 z = f32x2{fabsf(u.x), fabsf(u.y)} * kInvSqrt2;
  const f32x2 den = pk_fma(splat2(0.5f), z, splat2(1.0f));
  const f32x2 t = f32x2{fast_rcp(den.x), fast_rcp(den.y)};
  f32x2 p = pk_fma(t, splat2(0.17087277f), splat2(-0.82215223f));
  p = pk_fma(t, p, splat2(1.48851587f));
  p = pk_fma(t, p, splat2(-1.13520398f));
  p = pk_fma(t, p, splat2(0.27886807f));
  p = pk_fma(t, p, splat2(-0.18628806f));
  p = pk_fma(t, p, splat2(0.09678418f));
  p = pk_fma(t, p, splat2(0.37409196f));
  p = pk_fma(t, p, splat2(1.00002368f));
  p = pk_fma(t, p, splat2(-1.26551223f));
  // fast_exp(x) = exp2(x * log2 e), as in probit_eval
  const f32x2 az = (-z * z) * 1.4426950408889634f;
  const f32x2 ap = p * 1.4426950408889634f;
  const f32x2 ez = f32x2{__builtin_amdgcn_exp2f(az.x), __builtin_amdgcn_exp2f(az.y)};
  const f32x2 ep = f32x2{__builtin_amdgcn_exp2f(ap.x), __builtin_amdgcn_exp2f(ap.y)};
  phi = ez * kInvSqrt2Pi;
  const f32x2 erfc_z = (t * ez) * ep;
  const f32x2 om = splat2(1.0f) - erfc_z;  // 1 - erfc, rounded once
  // erf(u) = +-(1 - erfc): erfc - 1 is exactly -(1 - erfc)
  const f32x2 erf_u = f32x2{u.x < 0.0f ? -om.x : om.x, u.y < 0.0f ? -om.y : om.y};
  const f32x2 cdf = splat2(0.5f) * (splat2(1.0f) + erf_u);
  return cdf * kC1 + splat2(kC0);
}

// probit_eval2 on N independent pairs in lockstep (step-major): dependent
// packed ops need a wait state between them, and N interleaved chains hide it.
// Bit-identical to N probit_eval2 calls.
template <int N>
MPV_DEV void probit_eval2xN(const f32x2 (&u)[N], f32x2 (&E)[N], f32x2 (&phi)[N]) {
#pragma clang fp contract(off)
  f32x2 z[N], t[N], p[N];
#pragma unroll
  for (int j = 0; j < N; ++j) z[j] = f32x2{fabsf(u[j].x), fabsf(u[j].y)} * kInvSqrt2;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 den = pk_fma(splat2(0.5f), z[j], splat2(1.0f));
    t[j] = f32x2{fast_rcp(den.x), fast_rcp(den.y)};
  }
  constexpr float c[10] = {0.17087277f, -0.82215223f, 1.48851587f, -1.13520398f, 0.27886807f,
                           -0.18628806f, 0.09678418f, 0.37409196f, 1.00002368f, -1.26551223f};
#pragma unroll
  for (int j = 0; j < N; ++j) p[j] = pk_fma(t[j], splat2(c[0]), splat2(c[1]));
#pragma unroll
  for (int k = 2; k < 10; ++k)
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = pk_fma(t[j], p[j], splat2(c[k]));
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 az = (-z[j] * z[j]) * 1.4426950408889634f;
    const f32x2 ap = p[j] * 1.4426950408889634f;
    const f32x2 ez = f32x2{__builtin_amdgcn_exp2f(az.x), __builtin_amdgcn_exp2f(az.y)};
    const f32x2 ep = f32x2{__builtin_amdgcn_exp2f(ap.x), __builtin_amdgcn_exp2f(ap.y)};
    phi[j] = ez * kInvSqrt2Pi;
    z[j] = (t[j] * ez) * ep;  // erfc
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 om = splat2(1.0f) - z[j];
    const f32x2 erf_u = f32x2{u[j].x < 0.0f ? -om.x : om.x, u[j].y < 0.0f ? -om.y : om.y};
    const f32x2 cdf = splat2(0.5f) * (splat2(1.0f) + erf_u);
    E[j] = cdf * kC1 + splat2(kC0);
  }
}

// Forward-only probit (no phi) on N pairs in lockstep: the erfcc form with a
// single exponential, erfc(z) = t * exp(P(t) - z^2), as Numerical Recipes
// writes it.  log2(e) is folded into the variable (zq = z * sqrt(log2 e)) and
// into the coefficients, so the exponent is one fma feeding v_exp_f32; the
// sign of erf follows u by copysign, and 0.5 * C1 is one exact constant.
// Agrees with probit_eval2 to a few ulps of E.
//
// The callers work on w = 1 + erf(u / sqrt 2) = 2 Phi(u): E = kEh w + C0 is
// one fma that a caller folds into its own affine use of E (q = qa E + qb,
// the ranking exponent sg E, the column sums), so E is rarely formed at all.
// 1 + erf is exact for u < 0 (Sterbenz), so a small E keeps its relative
// precision; folding a rounded 0.5 C1 + C0 into one constant would not.
constexpr float kEh = 0.5f * kC1;
constexpr float kPhiK = kC1 * kInvSqrt2Pi;  // dE/du = kPhiK exp(-u^2/2)
//
// P(t) here is a degree-6 minimax fit of log(erfc(z) / t) + z^2 over
// t >= 0.38 (|u| <= 4.6; tools/fit_erfc.py) in place of the degree-9
// Numerical Recipes fit over all t: below t = 0.38 its error grows, but there
// erfc(z) < 6e-6 and E = C0 + C1 Phi(u) is soon C0-dominated.  Emulated in
// fp32 over |u| <= 40, E's maximum relative error is 2.6e-6 against NR's
// 2.46e-6; both are set by the fp32 rounding of zq^2 near |u| ~ 5, not by P.
// Three fewer packed fmas per element pair.
//
// zq = u sqrt(log2 e) / sqrt 2 is the caller's: it keeps u's sign (used only
// squared, through |zq| as an fma abs source modifier, and for erf's sign),
// and a caller with u = t + base forms it as one fma(t, kZq, base kZq).
// 1 - erfc as one fma of the unrounded product (erfc is never formed): one
// packed op fewer per element pair in the forward epilogue and the element
// pass (forward -0.7 %, element pass -1.7 %, round 6), and the probit sweep's
// per-band bounds unchanged (tests/test_gpu_probit_ulp.py)
#ifndef MPV_OM_FMA
#define MPV_OM_FMA 1
#endif
constexpr int kErfcDeg = 6;
constexpr float kSqL2e = 1.2011224087864498f;  // sqrt(log2 e)
constexpr float kZq = kInvSqrt2 * kSqL2e;
template <int N>
MPV_DEV void probit_w2xN_zq(const f32x2 (&zq)[N], f32x2 (&w)[N]) {
#pragma clang fp contract(off)
  constexpr float kL2e = 1.4426950408889634f;  // log2 e
  constexpr float c[kErfcDeg + 1] = {
      -0.139353514f * kL2e, 0.777093824f * kL2e, -1.58356997f * kL2e, 1.19629222f * kL2e,
      -0.0702797193f * kL2e, 1.09342452f * kL2e, -1.27360696f * kL2e};
  f32x2 t[N], p[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    t[j] = f32x2{fast_rcp(fmaf(0.5f / kSqL2e, fabsf(zq[j].x), 1.0f)),
                 fast_rcp(fmaf(0.5f / kSqL2e, fabsf(zq[j].y), 1.0f))};
  }
#pragma unroll
  for (int j = 0; j < N; ++j) p[j] = pk_fma(t[j], splat2(c[0]), splat2(c[1]));
#pragma unroll
  for (int k = 2; k <= kErfcDeg; ++k)
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = pk_fma(t[j], p[j], splat2(c[k]));
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 a = pk_fma(-zq[j], zq[j], p[j]);
    const f32x2 e = f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
#if MPV_OM_FMA
    const f32x2 om = pk_fma(-t[j], e, splat2(1.0f));  // 1 - erfc, erfc = t e unrounded
#else
    const f32x2 om = splat2(1.0f) - t[j] * e;
#endif
    w[j] = splat2(1.0f) +
           f32x2{__builtin_copysignf(om.x, zq[j].x), __builtin_copysignf(om.y, zq[j].y)};
  }
}

template <int N>
MPV_DEV void probit_prob2xN(const f32x2 (&u)[N], f32x2 (&E)[N]) {
  f32x2 zq[N];
#pragma unroll
  for (int j = 0; j < N; ++j) zq[j] = u[j] * kZq;
  probit_w2xN_zq<N>(zq, E);
#pragma unroll
  for (int j = 0; j < N; ++j) E[j] = pk_fma(E[j], splat2(kEh), splat2(kC0));
}

// probit_w2xN_zq for the backward: w (E = kEh w + C0) and ez = exp(-u^2/2),
// which times kPhiK = (1 - 1e-6)/sqrt(2 pi) is the factor dE/du needs (the
// element pass folds kPhiK into its row and column coefficients, so the
// product is one multiply per element, not two).  exp(-z^2) gives phi, so erfc
// is taken as t exp(-z^2) Q(t) with Q a degree-6 minimax fit of
// erfcx(z) / t over t >= 0.38 (relative; tools/fit_erfc.py, form q) instead
// of a second exponential of P(t).  fp32-emulated E error over |u| <= 40:
// max 2.4e-6 (the forward's P form 2.6e-6, NR 2.46e-6).
constexpr int kErfcxDeg = 6;
constexpr float kErfcxC1 = -0.359859836f;  // c[1] below
// qc1: c[1] as a caller-held register pair (a loop keeps it live instead of
// re-copying the constant into a VGPR every row), or null.
template <int N>
MPV_DEV void probit_dw2xN_zq(const f32x2 (&zq)[N], f32x2 (&w)[N], f32x2 (&ezo)[N],
                             const f32x2* qc1 = nullptr) {
#pragma clang fp contract(off)
  constexpr float c[kErfcxDeg + 1] = {0.0899837102f, -0.359859836f, 0.38748431f,
                                      0.0453561664f, 0.275197459f,  0.279788422f,
                                      0.282049996f};
  static_assert(c[1] == kErfcxC1, "qc1 callers hold c[1]");
  f32x2 t[N], q[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    t[j] = f32x2{fast_rcp(fmaf(0.5f / kSqL2e, fabsf(zq[j].x), 1.0f)),
                 fast_rcp(fmaf(0.5f / kSqL2e, fabsf(zq[j].y), 1.0f))};
  }
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], splat2(c[0]), qc1 ? *qc1 : splat2(c[1]));
#pragma unroll
  for (int k = 2; k <= kErfcxDeg; ++k)
#pragma unroll
    for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(c[k]));
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 az = -zq[j] * zq[j];
    const f32x2 ez = f32x2{__builtin_amdgcn_exp2f(az.x), __builtin_amdgcn_exp2f(az.y)};
    ezo[j] = ez;
#if MPV_OM_FMA
    const f32x2 om = pk_fma(-(t[j] * ez), q[j], splat2(1.0f));
#else
    const f32x2 om = splat2(1.0f) - (t[j] * ez) * q[j];
#endif
    w[j] = splat2(1.0f) +
           f32x2{__builtin_copysignf(om.x, zq[j].x), __builtin_copysignf(om.y, zq[j].y)};
  }
}

// Scalar lockstep version (N independent evaluations, no packed ops):
// bit-identical to N probit_eval calls (phi omitted).
template <int N>
MPV_DEV void probit_probN(const float (&u)[N], float (&E)[N]) {
  float z[N], t[N], p[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    z[j] = fabsf(u[j]) * kInvSqrt2;
    t[j] = fast_rcp(fmaf(0.5f, z[j], 1.0f));
  }
  constexpr float c[10] = {0.17087277f, -0.82215223f, 1.48851587f, -1.13520398f, 0.27886807f,
                           -0.18628806f, 0.09678418f, 0.37409196f, 1.00002368f, -1.26551223f};
#pragma unroll
  for (int j = 0; j < N; ++j) p[j] = fmaf(t[j], c[0], c[1]);
#pragma unroll
  for (int k = 2; k < 10; ++k)
#pragma unroll
    for (int j = 0; j < N; ++j) p[j] = fmaf(t[j], p[j], c[k]);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float ez = fast_exp(-z[j] * z[j]);
    const float erfc_z = t[j] * ez * fast_exp(p[j]);
    const float erf_u = u[j] < 0.0f ? __fsub_rn(erfc_z, 1.0f) : __fsub_rn(1.0f, erfc_z);
    const float cdf = __fmul_rn(0.5f, __fadd_rn(1.0f, erf_u));
    E[j] = __fadd_rn(__fmul_rn(cdf, kC1), kC0);
  }
}

// ---- DPP row (16-lane) reductions ------------------------------------------
// row_shr:n = 0x110 + n.  After the 4 steps lane 15 of every 16-lane row holds
// the row's sum (bound_ctrl: lanes shifted in from outside the row read 0).
template <int CTRL>
MPV_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
MPV_DEV float row16_sum_to_lane15(float v) {
  v += dpp_f<0x111>(v);   // row_shr:1
  v += dpp_f<0x112>(v);   // row_shr:2
  v += dpp_f<0x114>(v);   // row_shr:4
  v += dpp_f<0x118>(v);   // row_shr:8
  return v;
}

// row16_sum_to_lane15 of N values step-major: the N independent chains fill
// each other's DPP wait states (no s_nop), and with the permuted operand as
// src0 the add and the row shift fuse into one v_add_f32_dpp.
template <int N>
MPV_DEV void row16_sum_to_lane15_n(float (&v)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = dpp_f<0x111>(v[j]) + v[j];
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = dpp_f<0x112>(v[j]) + v[j];
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = dpp_f<0x114>(v[j]) + v[j];
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = dpp_f<0x118>(v[j]) + v[j];
}

// Sum over the four 16-lane rows of the wave (lanes l, l^16, l^32, l^48) by
// the gfx950 row-swap permutes (VALU, no LDS): every lane gets the total.
MPV_DEV float sum_lanegroups(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(c[0]) + __uint_as_float(c[1]);
}

// sum_lanegroups of N values step-major (independent chains between the
// permutes instead of wait states).
template <int N>
MPV_DEV void sum_lanegroups_n(float (&v)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[j]), __float_as_uint(v[j]),
                                                    false, false);
    v[j] = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j]), __float_as_uint(v[j]),
                                                    false, false);
    v[j] = __uint_as_float(c[0]) + __uint_as_float(c[1]);
  }
}

MPV_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MPV_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block reduction over up to 1024 threads; `red` must hold >= 16 floats.
// Every thread returns the total.
template <bool IS_MAX>
MPV_DEV float block_reduce(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = IS_MAX ? wave_max(v) : wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = IS_MAX ? -INFINITY : 0.0f;
  for (int i = 0; i < nw; ++i) r = IS_MAX ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

// N block reductions of the same kind with one barrier pair (`red` >= 16 N
// floats); each value is combined in the same order as by block_reduce.
template <int N, bool IS_MAX>
MPV_DEV void block_reduce_n(float (&v)[N], float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = IS_MAX ? wave_max(v[k]) : wave_sum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) red[k * 16 + wid] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    float r = IS_MAX ? -INFINITY : 0.0f;
    for (int i = 0; i < nw; ++i) r = IS_MAX ? fmaxf(r, red[k * 16 + i]) : r + red[k * 16 + i];
    v[k] = r;
  }
}

// Two block reductions of the same kind at the cost of one (`red` >= 32
// floats); each value is combined in the same order as by block_reduce.
template <bool IS_MAX>
MPV_DEV void block_reduce2(float& a, float& b, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  a = IS_MAX ? wave_max(a) : wave_sum(a);
  b = IS_MAX ? wave_max(b) : wave_sum(b);
  __syncthreads();
  if (lane == 0) red[wid] = a, red[16 + wid] = b;
  __syncthreads();
  float ra = IS_MAX ? -INFINITY : 0.0f, rb = ra;
  for (int i = 0; i < nw; ++i) {
    ra = IS_MAX ? fmaxf(ra, red[i]) : ra + red[i];
    rb = IS_MAX ? fmaxf(rb, red[16 + i]) : rb + red[16 + i];
  }
  a = ra, b = rb;
}

// d KL / d (mu, logvar) of mpvae.py:147-148, scaled by the upstream gradient
// g = gscal[KL] + 1.1 * gscal[TOTAL], for elements i0, i0 + stride, ...
// (mpv_kl_bwd's kernel, and the extra workgroups of the backward's bwd_coef).
template <typename KlArgs>
MPV_DEV void kl_bwd_range(const KlArgs& a, int64_t i0, int64_t stride) {
  const int64_t n = a.B * a.d;
  // a slot not live is not read (mpv_kl_bwd_args.live): its gradient is 0
  const float gk = (a.live & MPV_LIVE(MPV_G_KL)) ? a.gscal[MPV_G_KL] : 0.0f;
  const float gt = (a.live & MPV_LIVE(MPV_G_TOTAL)) ? a.gscal[MPV_G_TOTAL] : 0.0f;
  const float g = gk + kKlWeight * gt;
  const float s = 0.5f * g / (float)a.B;
  for (int64_t i = i0; i < n; i += stride) {
    const float lve = a.fe_logvar[i], lvx = a.fx_logvar[i];
    const float dm = a.fx_mu[i] - a.fe_mu[i];
    const float ex = expf(lvx);
    const float den = ex + kKlEps;
    const float r = expf(lve - lvx);
    const float gm = s * 2.0f * dm / den;
    a.g_fe_mu[i] = -gm;
    a.g_fx_mu[i] = gm;
    a.g_fe_logvar[i] = s * (r - 1.0f);
    a.g_fx_logvar[i] = s * (1.0f - r - dm * dm * ex / (den * den));
  }
}

// ---- 3xf16 split operands ---------------------------------------------------
// x*s = hi + lo with hi = fp16(x*s), lo = fp16(x*s - hi); the power-of-two
// scale s keeps max|x*s| <= 2^15 so both halves stay in the fp16 normal range
// for every element that matters.  A product is evaluated as
// hi*hi + hi*lo + lo*hi on the f16 matrix cores with fp32 accumulation
// (the dropped lo*lo term is <= 2^-22 relative).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

MPV_DEV void split_f16(float x, float s, uint16_t& hi, uint16_t& lo) {
  const float xs = x * s;
  const _Float16 h = (_Float16)xs;
  const _Float16 l = (_Float16)(xs - (float)h);
  hi = __builtin_bit_cast(uint16_t, h);
  lo = __builtin_bit_cast(uint16_t, l);
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// split_f16 of two values at once, x0 in bits 0-15 and x1 in bits 16-31 of
// the hi and lo words, bit for bit: v_fma_mix rounds fma(s, x, -0) = x*s
// (exact: s is a power of two; the -0 addend keeps a -0's sign) and then
// fma(s, x, -hi) = x*s - hi (exact in fp32) once to fp16, four instructions
// where the plain form takes a multiply, a convert, a convert back and a
// subtract per value.
MPV_DEV void split2_f16(float x0, float x1, float s, uint32_t& hi, uint32_t& lo) {
  const float nz = -0.0f;
  uint32_t h, l;
  asm("v_fma_mixlo_f16 %0, %2, %3, %5\n\t"
      "v_fma_mixhi_f16 %0, %2, %4, %5\n\t"
      "v_fma_mixlo_f16 %1, %2, %3, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %2, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(l)
      : "s"(s), "v"(x0), "v"(x1), "v"(nz));
  hi = h;
  lo = l;
}

// one v_add_f32 (the SLP vectoriser would pack such sums through moves)
MPV_DEV float add_f32(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Power-of-two scale mapping max|x| to (2^13, 2^14]; 1 for 0 / non-finite.
MPV_DEV float pow2_scale(float maxabs) {
  if (!(maxabs > 0.0f) || !isfinite(maxabs)) return 1.0f;
  int e;
  frexpf(maxabs, &e);           // maxabs = m * 2^e, m in [0.5, 1)
  return ldexpf(1.0f, 14 - e);  // maxabs * s in [2^13, 2^14)
}

// Exact combine of row b of per-shard statistics gathered as (R, 6, B):
// M = max m_r, Z = sum Z_r exp(m_r - M), the ranking sums add
// (mpv_bstat_combine, and the sharded finalize in the same order).
MPV_DEV void bstat_combine_row(const float* __restrict__ g, int64_t R, int64_t B, int64_t b,
                               float (&v)[6]) {
#pragma unroll
  for (int br = 0; br < 2; ++br) {
    const int mi = 2 * br, zi = 2 * br + 1;
    float M = -INFINITY;
    for (int64_t r = 0; r < R; ++r) M = fmaxf(M, g[(r * 6 + mi) * B + b]);
    float Z = 0.0f;
    for (int64_t r = 0; r < R; ++r) Z += g[(r * 6 + zi) * B + b] * expf(g[(r * 6 + mi) * B + b] - M);
    v[mi] = M;
    v[zi] = Z;
  }
  for (int k = 4; k < 6; ++k) {
    float acc = 0.0f;
    for (int64_t r = 0; r < R; ++r) acc += g[(r * 6 + k) * B + b];
    v[k] = acc;
  }
}

// pow2_scale of max(bound[0..n)), computed by one wave (every lane active): the
// same bits in every wave of every kernel that needs it (a max is exact in any
// order), so the G planes' scale needs no launch of its own (round 6).
MPV_DEV float wave_pow2_scale(const float* __restrict__ bound, int n) {
  float m = 0.0f;
  for (int i = threadIdx.x & 63; i < n; i += 64) m = fmaxf(m, bound[i]);
  return pow2_scale(wave_max(m));
}

MPV_DEV f16x8 as_f16x8(s16x8 v) { return __builtin_bit_cast(f16x8, v); }

// Chunked split layout (include/mpvae_hip.h mpv_split16): index of the hi half
// of column c in row r; the lo half is kLoOff further.
constexpr int kLoOff = 32;
__host__ __device__ inline int64_t chunked_index(int64_t r, int64_t ld, int64_t c) {
  return r * ld + ((c >> 5) << 6) + (c & 31);
}

// ---- LDS-DMA pipelines: raw barrier + counted vmcnt ------------------------
// __syncthreads() would make hipcc drain every in-flight LDS-DMA (vmcnt(0));
// the rings use a raw s_barrier and wait for exactly the stages they read.
MPV_DEV void barrier_raw() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Barrier for LDS traffic only: this wave's LDS reads/writes are complete,
// then every wave meets.  Unlike __syncthreads() it does not drain LDS-DMA.
MPV_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  barrier_raw();
}

template <int N>
MPV_DEV void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS address (byte offset in the workgroup's LDS) of a __shared__ pointer.
MPV_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4, saddr form): lane i's 16 B
// at saddr + voff land at LDS byte lds + 16*i.  Issued through inline asm so
// that hipcc's waitcnt pass does not see an LDS store: it otherwise puts an
// s_waitcnt vmcnt(0) before every later ds_read (it cannot tell the stage
// images of a ring apart), which exposes the whole DMA latency at every stage.
// Callers order it themselves: counted s_waitcnt vmcnt + a barrier before a
// stage is read, and a barrier after its last read before it is refilled.
MPV_DEV void lds_dma16(const void* saddr, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(saddr), "s"(lds)
      : "memory");
}

// Row stride (floats) of T and of the fp32 G written over it: L rounded up to
// 4, so every row starts 16-B aligned and the element pass reads whole float4
// (ABI v5; include/mpvae_hip.h).
__host__ __device__ inline int64_t t_cols(int64_t L) { return (L + 3) & ~int64_t(3); }

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate must be a constant).
MPV_DEV void wait_vmcnt_dyn(int n) {
#define MPV_VMC(k) \
  case k:          \
    wait_vmcnt<k>(); \
    break;
  switch (n) {
    MPV_VMC(0) MPV_VMC(1) MPV_VMC(2) MPV_VMC(3) MPV_VMC(4) MPV_VMC(5) MPV_VMC(6) MPV_VMC(7)
    MPV_VMC(8) MPV_VMC(9) MPV_VMC(10) MPV_VMC(11) MPV_VMC(12) MPV_VMC(13) MPV_VMC(14)
    MPV_VMC(15) MPV_VMC(16) MPV_VMC(17) MPV_VMC(18) MPV_VMC(19) MPV_VMC(20) MPV_VMC(21)
    MPV_VMC(22) MPV_VMC(23) MPV_VMC(24)
    default:
      wait_vmcnt<0>();
      break;
  }
#undef MPV_VMC
}

// ---- Philox4x32-10 (Salmon et al. SC'11) ------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

MPV_DEV u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product (lo and hi words together)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    // a ^ b ^ k as one v_bitop3_b32 (truth table 0x96); the compiler emits two
    // v_xor_b32 for the plain expression
    c = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
              (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Box-Muller on one word pair (see oracle/philox.py for the exact map), on the
// hardware transcendentals: v_log_f32 (log2), v_sqrt_f32, and v_sin_f32 /
// v_cos_f32, which take their argument in revolutions -- exactly v in [0, 1).
MPV_DEV void box_muller(uint32_t we, uint32_t wo, float& n0, float& n1) {
  const float u = ((float)(we >> 8) + 0.5f) * 5.9604644775390625e-8f;   // 2^-24
  const float v = (float)(wo >> 8) * 5.9604644775390625e-8f;
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u));  // -2 ln 2
  n0 = r * __builtin_amdgcn_cosf(v);
  n1 = r * __builtin_amdgcn_sinf(v);
}

// Compute units of the current device (host side; 256 when it cannot be
// queried, e.g. in a build container without a GPU).  Queried once per
// process (a function-local static: thread-safe initialisation).  The
// forward's s-chunk count and the dR GEMM's split-K chunk count derive from
// it, so the order in which partial sums are added -- and with it the last
// bits of the results -- is fixed per CU count (MI355X: 256), not across
// devices with different CU counts.
inline int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace mpv
