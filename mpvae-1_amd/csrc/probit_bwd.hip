// Backward of the MPVAE probit ELBO for one S-shard: the gradients PyTorch
// autograd takes through reference mpvae.py:165-210, written out analytically.
//
//   bwd_coef_kernel  per (s,b): alpha = -g_nll * softmax_s(logp)/B and the
//                    ranking coefficients betaP = g_c N/(n S B), betaN = g_c P/(n S B)
//                    (NaN for a degenerate row whose ranking term is live,
//                    reproducing the 0/0 of mpvae.py:118 under autograd); per
//                    batch row also an upper bound of |G| (3xf16 scale).
//   bwd_elem_kernel  streams T once: recomputes E, E_x, forms
//                    dE = alpha (y/E - (1-y)/(1-E)) - [y=1] betaP e^{-5E}
//                         + [y=0] betaN e^{5E} + g_indiv/S,
//                    du = dE (1-1e-6) phi(u); column sums over s give d fe_out /
//                    d fx_out; writes G = du + du_x (fp32 over T, or 3xf16 planes).
//   dR16_kernel      dR[l][k] = sum_{s,b} G[s,b,l] eps[s,b,k], 3xf16 operands on
//                    the f16 matrix cores; the rows (the K axis) are the LDS
//                    rows, fragments come from ds_read_b64_tr_b16 transposed
//                    reads; split-K over the S*B rows into slabs reduced in a
//                    fixed order (deterministic).
//   dR_gemm_kernel   the same on exact fp32 MFMA (MPV_GEMM_F32).
#include "abi_util.h"
#include "mpv_common.h"


namespace mpv {

int launch_sum_slabs(const float* in, int64_t nslab, int64_t n, void* out, int out_dtype,
                     hipStream_t s);
int launch_sum_slabs_pair(const float* in0, int64_t nslab0, int64_t n0, void* out0,
                          int out0_dtype, const float* in1, int64_t nslab1, int64_t n1,
                          void* out1, int out1_dtype, hipStream_t s);

// Upper bounds used for the G scale (3xf16): for E = Phi(u)(1-1e-6)+0.5e-6,
// sup_u phi(u) |y/E - (1-y)/(1-E)| < 4.5 (inverse Mills ratio capped by the
// 0.5e-6 floor), phi(u) e^{-5E} <= 0.4, phi(u) e^{5E} <= 0.4 e^5 < 60.  Only the
// order of magnitude matters: the split keeps full precision for anything
// within 2^10 of the bound.
constexpr float kBoundDl = 4.5f, kBoundPos = 0.4f, kBoundNeg = 60.0f, kBoundInd = 0.4f;

// --------------------------------------------------------------- coefficients
// bwd_coef: one workgroup per batch row of 512 threads (1024: C2 +1.3 us, C3
// +-0, round 6; 256: C2 +1.7, C3 +2, C4 +3 us against 512, round 3)
#ifndef MPV_COEF_THREADS
#define MPV_COEF_THREADS 512
#endif
constexpr int kCoefThreads = MPV_COEF_THREADS;

__global__ __launch_bounds__(kCoefThreads) void bwd_coef_kernel(
    const float* __restrict__ y, const float* __restrict__ rowstat, const float* __restrict__ bstat,
    const float* __restrict__ gscal, const float* __restrict__ gI, const float* __restrict__ gIL,
    float* __restrict__ coef, float* __restrict__ gbound, int S, int B, int L, float S_total,
    float nll_coeff, float c_coeff, int live, mpv_kl_bwd_args kl, int kl_blocks) {
  __shared__ float red[48];
  if ((int)blockIdx.x >= B) {  // the extra workgroups: the KL backward (mpv_bwd_args.kl)
    kl_bwd_range(kl, (int64_t)(blockIdx.x - B) * blockDim.x + threadIdx.x,
                 (int64_t)kl_blocks * blockDim.x);
    return;
  }
  const int b = blockIdx.x, tid = threadIdx.x;
  float np = 0.f, nn = 0.f, gi = 0.f;
  for (int l = tid; l < L; l += blockDim.x) {
    const int64_t o = (int64_t)b * L + l;
    const float v = y[o];
    np += (v == 1.0f) ? 1.0f : 0.0f;
    nn += (v == 0.0f) ? 1.0f : 0.0f;
    gi = fmaxf(gi, (gI ? fabsf(gI[o]) : 0.0f) + (gIL ? fabsf(gIL[o]) : 0.0f));
  }
  {  // the two counts and the max with one barrier pair (block_reduce's orders)
    const int lane = tid & 63, wid = tid >> 6, nw = (blockDim.x + 63) >> 6;
    np = wave_sum(np);
    nn = wave_sum(nn);
    gi = wave_max(gi);
    __syncthreads();
    if (lane == 0) red[wid] = np, red[16 + wid] = nn, red[32 + wid] = gi;
    __syncthreads();
    np = nn = 0.0f;
    gi = -INFINITY;
    for (int i = 0; i < nw; ++i) {
      np += red[i];
      nn += red[16 + i];
      gi = fmaxf(gi, red[32 + i]);
    }
  }
  const float nrm = np * nn;
  // only live slots are read (gscal may hold just the TOTAL slot)
  auto gs = [&](int k) { return (live & MPV_LIVE(k)) ? gscal[k] : 0.0f; };
  const float gt = gs(MPV_G_TOTAL);
  const float gn[2] = {gs(MPV_G_NLL) + nll_coeff * gt, gs(MPV_G_NLL_X) + nll_coeff * gt};
  const float gc[2] = {gs(MPV_G_C) + c_coeff * gt, gs(MPV_G_C_X) + c_coeff * gt};
  const bool clive[2] = {(live & (MPV_LIVE(MPV_G_TOTAL) | MPV_LIVE(MPV_G_C))) != 0,
                         (live & (MPV_LIVE(MPV_G_TOTAL) | MPV_LIVE(MPV_G_C_X))) != 0};
  const float inv_B = 1.0f / (float)B;
  float bound = kBoundInd * gi / S_total;
  float bmaxb[2];
#pragma unroll
  for (int br = 0; br < 2; ++br) {
    const float M = bstat[(2 * br) * B + b], Z = bstat[(2 * br + 1) * B + b];
    const bool dead = !(nrm > 0.0f) && clive[br];
    const float cs = gc[br] / (nrm * S_total * (float)B);
    float bmax = 0.0f;
    // one sample's coefficients (stored times dE/du's constant kPhiK: the
    // element pass then multiplies by exp(-u^2/2) alone)
    auto one = [&](float lp, float P, float N, float& ca, float& cp, float& cn) {
      float alpha = -gn[br] * (expf(lp - M) / Z) * inv_B;
      float bP = nrm > 0.0f ? cs * N : 0.0f;
      float bN = nrm > 0.0f ? cs * P : 0.0f;
      bmax = fmaxf(bmax, kBoundDl * fabsf(alpha) + kBoundPos * fabsf(bP) + kBoundNeg * fabsf(bN));
      if (dead) alpha = bP = bN = __builtin_nanf("");
      ca = alpha * kPhiK;
      cp = bP * kPhiK;
      cn = bN * kPhiK;
    };
    const float* rl = rowstat + ((int64_t)br * B + b) * S;
    const float* rp = rowstat + ((int64_t)(2 + 2 * br) * B + b) * S;
    const float* rn = rowstat + ((int64_t)(3 + 2 * br) * B + b) * S;
    float* ca = coef + ((int64_t)(3 * br + 0) * B + b) * S;
    float* cp = coef + ((int64_t)(3 * br + 1) * B + b) * S;
    float* cn = coef + ((int64_t)(3 * br + 2) * B + b) * S;
    if ((S & 3) == 0) {  // four consecutive samples per thread, 16-B accesses (same values)
      for (int s = 4 * tid; s < S; s += 4 * (int)blockDim.x) {
        const f32x4 lp = *reinterpret_cast<const f32x4*>(rl + s);
        const f32x4 P = *reinterpret_cast<const f32x4*>(rp + s);
        const f32x4 N = *reinterpret_cast<const f32x4*>(rn + s);
        float a[4], p[4], n[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) one(lp[j], P[j], N[j], a[j], p[j], n[j]);
        *reinterpret_cast<f32x4*>(ca + s) = f32x4{a[0], a[1], a[2], a[3]};
        *reinterpret_cast<f32x4*>(cp + s) = f32x4{p[0], p[1], p[2], p[3]};
        *reinterpret_cast<f32x4*>(cn + s) = f32x4{n[0], n[1], n[2], n[3]};
      }
    } else {
      for (int s = tid; s < S; s += blockDim.x) one(rl[s], rp[s], rn[s], ca[s], cp[s], cn[s]);
    }
    bmaxb[br] = bmax;
  }
  block_reduce2<true>(bmaxb[0], bmaxb[1], red);
  bound += bmaxb[0];
  bound += bmaxb[1];
  if (tid == 0 && gbound) gbound[b] = bound;
}

// ------------------------------------------------------------ element pass
struct ElemParams {
  const float* y;
  const float* fe;
  const float* fx;
  const float* gI;   // (B,L) grad of indiv_prob (feature branch) or NULL
  const float* gIL;  // (B,L) grad of indiv_prob_label (label branch) or NULL
  const float* coef;
  float* T;          // (B*S, ldT)
  uint16_t* g;       // chunked 3xf16 output planes (B*S rows of gld halves), or NULL: fp32 G over T
  const float* g_bound;  // (B) per-row bounds of |G|: the planes' scale (wave_pow2_scale)
  int64_t gld;
  float* colpart;  // [nSc][2][B][L]
  int S, B, L, Lc;  // Lc: columns covered (L rounded up to 4 for planes: pads get G = 0)
  int ldT;          // t_cols(L)
  int TPR, RPI, rows_per_chunk;
  float inv_S;
};

// dL/dt of one element for the label (.x) and feature (.y) branches at once
// (packed fp32): u = t + base, E = probit(u),
//   dE = alpha (y/E - (1-y)/(1-E)) + [y=1](-betaP) e^{-5E} + [y=0] betaN e^{5E} + g_ind
// (mpvae.py:110-117, 184-185 differentiated), dL/dt = dE (1-1e-6) phi(u).
// Per-column constants of the element pass (the lane's four label columns).
struct ElemCol {
  f32x2 base[4];  // fe_out, fx_out, in the probit's argument units (x kZq)
  f32x2 gind[4];  // g(indiv_prob_label), g(indiv_prob), / S_total, x kPhiK
  float y[4];
  bool soft[4];
  float qm[4];  // d = E + qm: E - 1 for y = 0 (the sign of d logp/dE folded in), E otherwise
  float sga[4];   // e^{-5E} (y = 1) or e^{5E} as exp2(sga w) e^{-+5 C0}
  float wp[4], wn[4];  // [y = 1], [y = 0] (1 or 0)
  bool pos[4];         // y = 1
  float kp, kn;        // e^{-5 C0}, e^{5 C0}: the row's ranking coefficients
                       // rkp = kp (-bP), rkn = kn bN carry them
};

// Four elements (columns) of one row at once, step-major so that the
// dependent packed ops of one element interleave with the others'.
// SOFT: the block may hold soft (non 0/1) labels (a per-column branch; false:
// no branch at all, so the four columns' chains interleave in one basic
// block).  NANCHK: poison the row here when bP is NaN (false: the caller does
// it with a wave-uniform test).  SOFT_RCP: a soft label's y/E - (1-y)/(1-E)
// by hardware reciprocals (1 ulp) instead of IEEE divisions, whose
// registers would spill the LDS-ring kernel.
// rkp, rkn: the row's ranking coefficients of a positive / negative label,
// kp (-betaP) and kn betaN (a binary block picks one per column instead of
// forming wn rkn + wp rkp; elem_rank_coefs).
// rkq: the four columns' ranking coefficients already picked (the LDS-ring
// loop reads each from its own address), or null.
template <bool SOFT = true, bool NANCHK = true, bool SOFT_RCP = false>
MPV_DEV void d_elem2x4(const float (&t)[4], const ElemCol& c, f32x2 alpha, f32x2 rkp, f32x2 rkn,
                       f32x2 (&out)[4], const f32x2* rkq = nullptr, const f32x2* qc1 = nullptr) {
  f32x2 zq[4], w[4], ez[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) zq[q] = pk_fma(splat2(t[q]), splat2(kZq), c.base[q]);
  probit_dw2xN_zq<4>(zq, w, ez, qc1);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // E in the reference's rounding order (mpvae.py:171-180: cdf = 0.5 (1 +
    // erf) exact from w = 1 + erf, then cdf (1 - eps1) and + eps1/2 each
    // rounded in fp32), so that near E -> 1, where one fp32 ulp of E is ~6 %
    // of 1 - E and 1/(1 - E) weights the gradient, E is the reference's E
    // bit for bit whenever w is (a single fma(w, kEh, C0) rounds once and
    // moved such gradients by ~1e-3: DESIGN.md section 4, "Full C4")
    f32x2 E;
    {
#pragma clang fp contract(off)
      E = w[q] * kEh + splat2(kC0);
    }
    // d logp / dE = y/E - (1-y)/(1-E): one reciprocal of E (y = 1) or of
    // E - 1 (y = 0, the sign folded in; exact for E >= 0.5)
    const f32x2 d = E + splat2(c.qm[q]);
    const f32x2 r = f32x2{fast_rcp(d.x), fast_rcp(d.y)};
    f32x2 dE;
    if (SOFT && c.soft[q]) {
      const f32x2 omE = splat2(1.0f) - E;
      const f32x2 dl = SOFT_RCP ? splat2(c.y[q]) * f32x2{fast_rcp(E.x), fast_rcp(E.y)} -
                                      splat2(1.0f - c.y[q]) * f32x2{fast_rcp(omE.x), fast_rcp(omE.y)}
                                : splat2(c.y[q]) / E - splat2(1.0f - c.y[q]) / omE;
      dE = pk_fma(alpha, dl, c.gind[q]);
    } else {
      dE = pk_fma(alpha, r, c.gind[q]);
    }
    // ranking term: pos -> -betaP e^{-5E}, neg -> +betaN e^{5E}
    const f32x2 rk = rkq   ? rkq[q]
                     : SOFT ? pk_fma(splat2(c.wn[q]), rkn, splat2(c.wp[q]) * rkp)
                            : (c.pos[q] ? rkp : rkn);
    const f32x2 a = w[q] * c.sga[q];
    dE = pk_fma(rk, f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)}, dE);
    out[q] = dE * ez[q];  // the coefficients carry kPhiK
  }
  // a degenerate row poisons every label, whatever its value (reference autograd)
  // (rkp is NaN exactly when betaP is)
  if (NANCHK && (rkp.x != rkp.x || rkp.y != rkp.y)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (rkp.x != rkp.x) out[q].x = rkp.x;
      if (rkp.y != rkp.y) out[q].y = rkp.y;
    }
  }
}

// The ranking coefficients of one row from its betaP, betaN (label, feature).
MPV_DEV void elem_rank_coefs(const ElemCol& c, f32x2 bP, f32x2 bN, f32x2& rkp, f32x2& rkn) {
  rkp = splat2(c.kp) * -bP;
  rkn = splat2(c.kn) * bN;
}

// Inputs of one row s of the element pass: its six coefficients (label .x,
// feature .y) and the lane's four t values.
struct ElemRow {
  f32x2 alpha, bP, bN;
  float t[4];
};

template <bool VEC>
MPV_DEV void elem_row_load(ElemRow& r, const ElemParams& p, int b, int s, int c0,
                           const bool (&ok)[4]) {
  const int64_t cb = (int64_t)b * p.S + s;
  const int64_t BS = (int64_t)p.B * p.S;
  r.alpha = f32x2{p.coef[0 * BS + cb], p.coef[3 * BS + cb]};
  r.bP = f32x2{p.coef[1 * BS + cb], p.coef[4 * BS + cb]};
  r.bN = f32x2{p.coef[2 * BS + cb], p.coef[5 * BS + cb]};
  const float* row = p.T + cb * p.ldT;
  if (VEC && c0 < p.L) {  // t_cols rows: the pad columns are readable
    // nontemporal T loads and G-plane stores: element pass -5 %
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(row + c0));
    r.t[0] = v[0]; r.t[1] = v[1]; r.t[2] = v[2]; r.t[3] = v[3];
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) r.t[q] = ok[q] ? row[c0 + q] : 0.0f;
  }
}

// The lane's four label columns c0 .. c0+3 of batch row b: validity and the
// per-column constants of the element math (ElemCol).
MPV_DEV void elem_col_setup(const ElemParams& p, int b, int c0, bool active, bool (&ok)[4],
                            ElemCol& ec) {
  const int L = p.L;
  ec.kp = exp2f((-5.0f * 1.4426950408889634f) * kC0);
  ec.kn = exp2f((5.0f * 1.4426950408889634f) * kC0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + q;
    ok[q] = active && c < L;
    const int64_t o = (int64_t)b * L + (ok[q] ? c : 0);
    const float yv = ok[q] ? p.y[o] : 0.0f;
    const float fe = ok[q] ? p.fe[o] : 0.0f;
    const float fx = ok[q] ? p.fx[o] : 0.0f;
    const float gi = (ok[q] && p.gI) ? p.gI[o] * p.inv_S : 0.0f;
    const float gil = (ok[q] && p.gIL) ? p.gIL[o] * p.inv_S : 0.0f;
    ec.base[q] = f32x2{fe, fx} * kZq;
    ec.gind[q] = f32x2{gil, gi} * kPhiK;
    ec.y[q] = yv;
    ec.soft[q] = !(yv == 0.0f || yv == 1.0f);
    ec.qm[q] = yv == 0.0f ? -1.0f : 0.0f;  // E - 1 = -(1 - E), or E
    const float sgx = (yv == 1.0f ? -5.0f : 5.0f) * 1.4426950408889634f;
    ec.sga[q] = sgx * kEh;
    // the constant factor e^{-+5 C0} of e^{-+5E} rides on the label weights
    ec.wp[q] = yv == 1.0f ? 1.0f : 0.0f;
    ec.wn[q] = yv == 0.0f ? 1.0f : 0.0f;
    ec.pos[q] = yv == 1.0f;
  }
}

// Rows of T in flight per thread beyond the one computing (kElemLookahead),
// and ONE: a block row covers all its columns (RPI == 1), so the row index and
// the six per-row coefficients are wave-uniform (scalar loads, no VGPRs).
// Otherwise (L < 1024: C2, C3) they are per-lane, 12 more VGPRs than fit in
// 128: those instantiations run at 3 waves per SIMD instead of spilling.
#ifndef MPV_ELEM_LA
#define MPV_ELEM_LA 1
#endif
constexpr int kElemLookahead = MPV_ELEM_LA;  // 2, 3: C3 element pass 0.111 -> 0.120 ms (r06_la_ab.json)
#ifndef MPV_ELEM_MIN_ROWS
#define MPV_ELEM_MIN_ROWS 16
#endif
constexpr int kElemMinRows = MPV_ELEM_MIN_ROWS;  // minimum T rows per thread (C2 -6 %)
#ifndef MPV_ELEM_OCC4
#define MPV_ELEM_OCC4 0  // 4 waves per SIMD for per-lane rows too: slower (r06_elem_occ4_ab.json)
#endif
template <bool VEC, bool PLANES, bool ONE>
__global__ __launch_bounds__(256, (ONE || MPV_ELEM_OCC4) ? 4 : 3) void bwd_elem_kernel(ElemParams p) {
  constexpr int LA = kElemLookahead;
  __shared__ float cred[256 * 8];
  const int b = blockIdx.x, sc = blockIdx.y;
  const int tid = threadIdx.x;
  const int rsub = ONE ? 0 : tid / p.TPR, cq = ONE ? tid : tid % p.TPR;
  const bool active = rsub < p.RPI;
  const int c0 = blockIdx.z * 1024 + cq * 4;
  const int S = p.S, B = p.B, L = p.L;
  const float gs = PLANES ? wave_pow2_scale(p.g_bound, p.B) : 1.0f;

  bool ok[4];
  ElemCol ec;
  elem_col_setup(p, b, c0, active, ok, ec);
  f32x2 sg2[4] = {splat2(0.f), splat2(0.f), splat2(0.f), splat2(0.f)};  // (label, feature)
  const int s_begin = sc * p.rows_per_chunk;
  const int s_end = min(S, s_begin + p.rows_per_chunk);
  if (active && c0 < p.Lc) {
    // LA rows of lookahead: rows s+RPI .. s+LA*RPI are in flight while row s
    // computes (the element math and the T stream overlap)
    const int s0 = s_begin + rsub, R = ONE ? 1 : p.RPI;
    ElemRow buf[LA + 1];
#pragma unroll
    for (int j = 0; j < LA; ++j)
      if (s0 + j * R < s_end) elem_row_load<VEC>(buf[j], p, b, s0 + j * R, c0, ok);
    for (int s = s0; s < s_end; s += R) {
      if (s + LA * R < s_end) elem_row_load<VEC>(buf[LA], p, b, s + LA * R, c0, ok);
      const ElemRow& cur = buf[0];
      const int64_t cb = (int64_t)b * S + s;
      float G[4];
      f32x2 g2[4];
      f32x2 rkp, rkn;
      elem_rank_coefs(ec, cur.bP, cur.bN, rkp, rkn);
      d_elem2x4(cur.t, ec, cur.alpha, rkp, rkn, g2);
      // column sums: pad columns (finite, never published) need no mask
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sg2[q] = sg2[q] + g2[q];
        G[q] = ok[q] ? g2[q].x + g2[q].y : 0.0f;
      }
      if (PLANES) {
        // (split2_f16 / add_f32 here, as in elem_ring_rows: C3 element pass
        // +4 %, the per-column branches leave the asm blocks unscheduled)
        uint16_t h[4], l[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split_f16(G[q], gs, h[q], l[q]);
        // rows b*S + s (the noise planes' row order), chunked like mpv_split16
        const int64_t o = chunked_index(cb, p.gld, c0);
        const s16x4 hv{(short)h[0], (short)h[1], (short)h[2], (short)h[3]};
        const s16x4 lv{(short)l[0], (short)l[1], (short)l[2], (short)l[3]};
        __builtin_nontemporal_store(hv, reinterpret_cast<s16x4*>(p.g + o));
        __builtin_nontemporal_store(lv, reinterpret_cast<s16x4*>(p.g + o + kLoOff));
      } else {
        float* row = p.T + cb * p.ldT;
        if (VEC && c0 < L) {  // pad columns get G = 0
          *reinterpret_cast<f32x4*>(row + c0) = f32x4{G[0], G[1], G[2], G[3]};
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (ok[q]) row[c0 + q] = G[q];
        }
      }
#pragma unroll
      for (int j = 0; j < LA; ++j) buf[j] = buf[j + 1];
    }
  }
  // column sums over this block's rows: reduce the RPI row-lanes per column
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    cred[tid * 8 + q] = sg2[q].x;
    cred[tid * 8 + 4 + q] = sg2[q].y;
  }
  __syncthreads();
  for (int j = tid; j < p.TPR * 4; j += blockDim.x) {
    const int cqq = j >> 2, q = j & 3;
    const int c = blockIdx.z * 1024 + j;
    if (c < L) {
      float e = 0.f, x = 0.f;
      for (int r = 0; r < p.RPI; ++r) {
        e += cred[(r * p.TPR + cqq) * 8 + q];
        x += cred[(r * p.TPR + cqq) * 8 + 4 + q];
      }
      p.colpart[(((int64_t)sc * 2 + 0) * B + b) * L + c] = e;
      p.colpart[(((int64_t)sc * 2 + 1) * B + b) * L + c] = x;
    }
  }
}

// The element pass for 3xf16 planes when one thread row of a block covers a
// whole label row (plan_bwd: TPR = cdiv(Lc, 4), so Lc > 512: C4, C5 and any
// 512 < L < 1024, whose surplus waves are masked).  T rows stream through a per-wave LDS ring by LDS-DMA
// (global_load_lds_dwordx4: a wave moves the 1 KB of a row its own 256
// columns need, so no wave reads another's slot and the ring needs no
// barrier); the row's six coefficients come from an LDS copy of the block's
// chunk.  The loop then issues no register load that hipcc must wait for --
// its only vector-memory ops are the DMA (counted here, lds_dma16) and the two
// G-plane stores per row -- and with SOFT false it has no divergent branch,
// so the four columns' element math interleaves in one basic block.  (The
// register-lookahead kernel above serialises each column's dependent packed
// ops behind s_nop: its per-column soft-label branches split the row into
// basic blocks the scheduler cannot interleave across, and without them hipcc
// drains its lookahead loads every row: DESIGN.md section 3.)
constexpr int kElemRing = 8;       // T rows in flight per wave (1 KB each; 8: 3 waves per SIMD)
constexpr int kElemRingRows = 256;  // rows per sub-chunk (the coefficient copy)
constexpr int kElemRingMinRows = 128;  // rows per block at least (plan_bwd; 64: +0.3 % at S 512)
#ifndef MPV_ELEM_SEL
#define MPV_ELEM_SEL 1  // per-lane ranking-coefficient addresses, scalar-base stores
#endif
// The rows of one sub-chunk [sb, sb + nrows) for one wave; SOFT: the block
// holds soft labels (block-uniform, so either loop is one basic block).
// MASK: some lane of the wave has columns past L or past the planes (their G is
// zeroed, their stores skipped).  NANCHK: some row of the sub-chunk is
// degenerate (its NaN poisons every label of that row).  The loop is bound by
// VALU issue (~95 % busy at C4, profiles/r05_elem_valu_pmc.json), so the row
// sums and the f16 split are one instruction each (asm: hipcc's SLP
// vectoriser otherwise packs the sums through register moves and splits by
// convert / convert back / subtract), the coefficients sit in LDS as the
// (label, feature) pairs the packed math takes, and the checks that do not
// apply to a wave or a sub-chunk are compiled out.
template <bool SOFT, bool MASK, bool NANCHK>
MPV_DEV void elem_ring_rows(const ElemParams& p, const ElemCol& ec, const bool (&ok)[4], bool live,
                            int b, int sb, int nrows, int c0, float gs, uint32_t voff,
                            float* myring, const float (*cf)[8], f32x2 (&sg2)[4]) {
  constexpr int NR = kElemRing;
  const int lane = threadIdx.x & 63;
  const int64_t rowb = (int64_t)b * p.S + sb;
  const char* tbase = reinterpret_cast<const char*>(p.T + rowb * p.ldT);
  const int64_t rstride = (int64_t)p.ldT * 4;
  auto issue = [&](int r) {  // LDS-DMA of row r (sub-chunk-relative) into its slot
    lds_dma16(tbase + r * rstride, voff, lds_addr(myring + (r % NR) * 256));
  };
  const int pro = min(NR, nrows);
  for (int r = 0; r < pro; ++r) issue(r);
#if MPV_ELEM_SEL
  // each column's ranking coefficient read from its own cf address (rkp at
  // byte 0 of a row, rkn at 16; alpha at 8 and 24, so 8 past either): no
  // per-row select
  uint32_t rsel[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) rsel[q] = ec.pos[q] ? 0u : 16u;
  // the lane's plane offset in a row (bytes); the row base is wave-uniform
  const uint32_t loffb = live ? 2u * (uint32_t)(((c0 >> 5) << 6) + (c0 & 31)) : 0u;
  f32x2 qc1 = splat2(kErfcxC1);
  asm volatile("" : "+v"(qc1));
#endif
  auto row = [&](int r) {
    const f32x4 tv = *reinterpret_cast<const f32x4*>(myring + (r % NR) * 256 + lane * 4);
    const float t[4] = {tv[0], tv[1], tv[2], tv[3]};
    f32x2 g2[4];
#if MPV_ELEM_SEL
    // (the row offset opaque: a scalar, so each address is one add)
    const char* crow =
        reinterpret_cast<const char*>(&cf[0][0]) + __builtin_amdgcn_readfirstlane(r * 32);
    const f32x2 rkp = *reinterpret_cast<const f32x2*>(crow);
    const f32x2 rkn = *reinterpret_cast<const f32x2*>(crow + 16);
    if (SOFT) {
      const f32x2 alpha = *reinterpret_cast<const f32x2*>(crow + 8);
      d_elem2x4<SOFT, false, true>(t, ec, alpha, rkp, rkn, g2);
    } else {
      f32x2 rkq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) rkq[q] = *reinterpret_cast<const f32x2*>(crow + rsel[q]);
      const f32x2 alpha = *reinterpret_cast<const f32x2*>(crow + rsel[0] + 8);
      d_elem2x4<SOFT, false, true>(t, ec, alpha, rkp, rkn, g2, rkq, &qc1);
    }
#else
    const f32x4 ca = *reinterpret_cast<const f32x4*>(&cf[r][0]);
    const f32x2 rkn = *reinterpret_cast<const f32x2*>(&cf[r][4]);
    const f32x2 alpha = f32x2{ca[0], ca[1]}, rkp = f32x2{ca[2], ca[3]};
    d_elem2x4<SOFT, false, true>(t, ec, alpha, rkp, rkn, g2);
#endif
    // a degenerate row poisons every label (the row's rkp is wave-uniform)
    if (NANCHK && __builtin_amdgcn_readfirstlane((rkp.x != rkp.x || rkp.y != rkp.y) ? 1 : 0)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (rkp.x != rkp.x) g2[q].x = rkp.x;
        if (rkp.y != rkp.y) g2[q].y = rkp.y;
      }
    }
    float G[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sg2[q] = sg2[q] + g2[q];
      G[q] = add_f32(g2[q].x, g2[q].y);
      if (MASK && !ok[q]) G[q] = 0.0f;
    }
    uint32_t hv[2], lv[2];
    split2_f16(G[0], G[1], gs, hv[0], lv[0]);
    split2_f16(G[2], G[3], gs, hv[1], lv[1]);
#if MPV_ELEM_SEL
    // the row base made opaque so it stays a scalar base (saddr stores with a
    // 32-bit lane offset, no 64-bit address add per row)
    const uint64_t ga = reinterpret_cast<uint64_t>(p.g + (rowb + r) * p.gld);
    // (readfirstlane returns int: each half zero-extended through uint32_t)
    const uint64_t grow =
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(ga >> 32)) << 32) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ga);
    if (!MASK || live) {  // nontemporal plane stores (the element pass -2 %, round 2)
      // (asm: hipcc forms a 64-bit lane address per row otherwise; the ring's
      // vmcnt arithmetic counts these two stores as before)
      asm volatile("global_store_dwordx2 %0, %1, %2 nt\n\t"
                   "global_store_dwordx2 %0, %3, %2 offset:%4 nt"
                   :
                   : "v"(loffb), "v"(u32x2{hv[0], hv[1]}), "s"(grow), "v"(u32x2{lv[0], lv[1]}),
                     "i"(2 * kLoOff));
    }
#else
    const int64_t o = chunked_index(rowb + r, p.gld, live ? c0 : 0);
    if (!MASK || live) {  // nontemporal plane stores (the element pass -2 %, round 2)
      __builtin_nontemporal_store(u32x2{hv[0], hv[1]}, reinterpret_cast<u32x2*>(p.g + o));
      __builtin_nontemporal_store(u32x2{lv[0], lv[1]}, reinterpret_cast<u32x2*>(p.g + o + kLoOff));
    }
#endif
    if (r + NR < nrows) issue(r + NR);  // into the slot row r was just read from
  };
  // Before row r is read, the ops issued after its DMA are the DMAs of rows
  // r+1 .. min(r+NR-1, last) and the two plane stores of each row
  // max(0, r-NR+1) .. r-1 (vector memory ops retire in issue order).  Rows
  // NR-1 .. nrows-NR wait for a constant count; the ramps use the run-time
  // count (an s_waitcnt takes an immediate: a compare ladder).  Only the
  // common loop (binary labels, full waves, no degenerate row) is peeled.
  int r = 0;
  if (!SOFT && !MASK && !NANCHK) {
    for (; r < min(NR - 1, nrows); ++r) {
      wait_vmcnt_dyn(min(NR - 1, nrows - 1 - r) + 2 * r);
      row(r);
    }
    for (; r <= nrows - NR; ++r) {
      wait_vmcnt<3 * (NR - 1)>();
      row(r);
    }
  }
  for (; r < nrows; ++r) {
    wait_vmcnt_dyn(min(NR - 1, nrows - 1 - r) + 2 * min(r, NR - 1));
    row(r);
  }
}

__global__ __launch_bounds__(256, 3) void bwd_elem_ring_kernel(ElemParams p) {
  constexpr int NR = kElemRing, CR = kElemRingRows;
  __shared__ __attribute__((aligned(16))) float ring[4][NR][256];  // [wave][slot][1 KB]
  __shared__ __attribute__((aligned(16))) float cf[CR][8];  // alpha, bP, bN (label, feature)
  const int b = blockIdx.x, sc = blockIdx.y, tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.z * 1024 + tid * 4;
  const int S = p.S, B = p.B, L = p.L;
  const float gs = wave_pow2_scale(p.g_bound, B);
  bool ok[4];
  ElemCol ec;
  elem_col_setup(p, b, c0, true, ok, ec);
  bool my_soft = false;
#pragma unroll
  for (int q = 0; q < 4; ++q) my_soft |= ok[q] && ec.soft[q];
  const bool soft_any = __syncthreads_or(my_soft) != 0;
  // a wave whose first lane is past the planes' columns writes nothing and
  // streams nothing (its lane 0 has the wave's smallest c0); in a live wave
  // every store instruction has a live lane, so it issues (the vmcnt
  // arithmetic of elem_ring_rows counts on that)
  const bool wave_live = (int)(blockIdx.z * 1024 + wid * 256) < p.Lc;
  // every lane's four columns are labels (< L) and in the planes (< Lc)
  const bool wave_full = (int)(blockIdx.z * 1024 + wid * 256 + 256) <= min(L, p.Lc);
  const bool live = c0 < p.Lc;
  const int s_begin = sc * p.rows_per_chunk;
  const int s_end = min(S, s_begin + p.rows_per_chunk);
  const int64_t BS = (int64_t)B * S;
  // lanes past the row's end (L % 1024 != 0) re-read column 0 and are masked
  const uint32_t voff = (uint32_t)((c0 < L ? c0 : 0) * 4);
  f32x2 sg2[4] = {splat2(0.f), splat2(0.f), splat2(0.f), splat2(0.f)};
  for (int sb = s_begin; sb < s_end; sb += CR) {  // sub-chunks of <= CR rows
    const int nrows = min(CR, s_end - sb);
    __syncthreads();  // the previous sub-chunk's cf reads are done
    // coef is [k][b][s]: cf[row] = alpha, rkp, rkn as (label, feature) pairs
    bool nan_row = false;
    for (int r = tid; r < nrows; r += 256) {
      const int64_t o = (int64_t)b * S + sb + r;
      const f32x2 alpha{p.coef[o], p.coef[3 * BS + o]};
      const f32x2 bP{p.coef[BS + o], p.coef[4 * BS + o]};
      const f32x2 bN{p.coef[2 * BS + o], p.coef[5 * BS + o]};
      f32x2 rkp, rkn;
      elem_rank_coefs(ec, bP, bN, rkp, rkn);
      nan_row |= bP.x != bP.x || bP.y != bP.y;
#if MPV_ELEM_SEL
      *reinterpret_cast<f32x4*>(&cf[r][0]) = f32x4{rkp.x, rkp.y, alpha.x, alpha.y};
      *reinterpret_cast<f32x4*>(&cf[r][4]) = f32x4{rkn.x, rkn.y, alpha.x, alpha.y};
#else
      *reinterpret_cast<f32x4*>(&cf[r][0]) = f32x4{alpha.x, alpha.y, rkp.x, rkp.y};
      *reinterpret_cast<f32x2*>(&cf[r][4]) = rkn;
#endif
    }
    const bool nan_any = __syncthreads_or(nan_row) != 0;
    if (!wave_live) continue;
    float* myring = &ring[wid][0][0];
    if (soft_any || !wave_full || nan_any) {
      if (soft_any)
        elem_ring_rows<true, true, true>(p, ec, ok, live, b, sb, nrows, c0, gs, voff, myring, cf, sg2);
      else
        elem_ring_rows<false, true, true>(p, ec, ok, live, b, sb, nrows, c0, gs, voff, myring, cf, sg2);
    } else {
      elem_ring_rows<false, false, false>(p, ec, ok, live, b, sb, nrows, c0, gs, voff, myring, cf,
                                          sg2);
    }
  }
  // column sums of the block's rows -> colpart (the ring is free now)
  __syncthreads();
  float* cred = &ring[0][0][0];  // 256 x 8 floats (8 KB, within the ring)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    cred[tid * 8 + q] = sg2[q].x;
    cred[tid * 8 + 4 + q] = sg2[q].y;
  }
  __syncthreads();
  for (int j = tid; j < 1024; j += 256) {
    const int c = blockIdx.z * 1024 + j;
    if (c < L) {
      p.colpart[(((int64_t)sc * 2 + 0) * B + b) * L + c] = cred[(j >> 2) * 8 + (j & 3)];
      p.colpart[(((int64_t)sc * 2 + 1) * B + b) * L + c] = cred[(j >> 2) * 8 + 4 + (j & 3)];
    }
  }
}

// ------------------------------------------------------------ 3xf16 dR GEMM
// K axis = the S*B sample rows q = b*S + s: the noise planes' own row order, in
// which the element pass also writes the G planes, so a K row is one address
// for both operands.  The rows stream in stages of 32 through a ring of LDS
// stage images (LDS-DMA, one barrier per stage).  Both operands are chunked
// (mpv_split16), so the 128 columns of a tile are 512 contiguous bytes per row
// holding hi and lo; a stage image is [G rows | E rows], 32 rows x 512 B each,
// and one DMA wave-instruction moves two whole rows.  The 32-B unit U of row r
// (units 4k, 4k+1: hi of columns 32k..32k+31; 4k+2, 4k+3: their lo) sits at
// position U ^ (r & 7).  An MFMA fragment (8 K rows of one column per lane) is
// two ds_read_b64_tr_b16; lane group g reads rows 4g..4g+3 and 16+4g..16+4g+3,
// so a 32-lane half of one transposed read touches rows 8j..8j+7 at 8 distinct
// positions mod 256 B, all 64 banks once: conflict-free (checked).
// Element j of lane group g holds K row (j < 4 ? 4g + j : 16 + 4g + j - 4), the
// same for A and B.
struct Dr16Params {
  const uint16_t* g;    // chunked G planes, rows b*S + s, gld halves per row
  const float* g_bound;  // (B) per-row bounds of |G|: the planes' scale (wave_pow2_scale)
  int64_t gld;
  mpv_split16 eps16;    // rows b*S + s
  float* slab;          // [nKc][L][z]
  int S, B, L, z;
  int nLt, nZt, nKc, rows_per_chunk, rows_pad;
};

constexpr int kDrKR = 32;     // K rows per stage (one MFMA k-step)

MPV_DEV s16x4 tr_read(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + off));
}

// block id -> (kc, tile): all tiles of one K chunk share rows -> ids equal mod 8
MPV_DEV void decode_kc_tile(int id, int K, int nT, int& kc, int& tile) {
  const int full = (K / 8) * 8 * nT;
  if (id < full) {
    const int q = id / (8 * nT), r = id % (8 * nT);
    tile = r / 8;
    kc = q * 8 + (r % 8);
  } else {
    const int r = id - full, Kr = K % 8;
    tile = r / Kr;
    kc = (K / 8) * 8 + (r % Kr);
  }
}

// One stage's LDS-DMA for this wave: PER_WAVE 1-KB pieces of RPP whole rows.
// Wave w moves pieces w*PER_WAVE ..; the first PIECES/2 are G rows, the rest E.
// The global base address is the piece's first row (wave-uniform: it goes in
// an SGPR pair); with RPP > 1 a lane's row within the piece is in its offset.
template <int PER_WAVE, int PIECES, int RPP>
MPV_DEV void dr_issue(const Dr16Params& p, char* dst, int q0, int rows, int wid,
                      const int (&dma_off)[PER_WAVE]) {
  const int lrow = RPP == 1 ? 0 : (int)(threadIdx.x & 63) / (64 / RPP);
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int pc = wid * PER_WAVE + i;
    const int q = q0 + (pc % (PIECES / 2)) * RPP;
    const uint16_t* src;
    int off = dma_off[i];
    if (pc < PIECES / 2) {  // G rows >= rows are zero
      src = p.g + (int64_t)q * p.gld;
      off += lrow * p.gld * 2;
    } else {  // E rows >= rows: repeat the last real row (finite, times a zero G row)
      const int qb = min(q, rows - 1);
      src = p.eps16.data + (int64_t)qb * p.eps16.ld;
      off += (min(q + lrow, rows - 1) - qb) * (int)p.eps16.ld * 2;
    }
    lds_dma16(src, (uint32_t)off, lds_addr(dst + pc * 1024));
  }
}

template <int WM, int WN, int TM, int TN, int kDrStages>
__global__ __launch_bounds__(WM* WN * 64, 1) void dR16_kernel(Dr16Params p) {
  constexpr int NW = WM * WN;
  constexpr int BL = WM * TM * 16, BZ = WN * TN * 16;
  static_assert(BL == BZ, "square tile: one LDS row layout for both operands");
  constexpr int ROWB = BL * 4;          // bytes per LDS row: BL columns, hi + lo
  constexpr int IMG = kDrKR * ROWB;     // per operand
  constexpr int STAGE = 2 * IMG;
  constexpr int PIECES = STAGE / 1024;  // 1-KB wave-instructions per stage
  constexpr int RPP = 1024 / ROWB;      // rows per piece
  static_assert(PIECES % NW == 0, "DMA pieces must split over waves");
  constexpr int PER_WAVE = PIECES / NW;
  constexpr int P = kDrStages - 1;
  __shared__ __attribute__((aligned(1024))) char smem[kDrStages * STAGE];

  int kc, tile;
  decode_kc_tile(blockIdx.x, p.nKc, p.nLt * p.nZt, kc, tile);
  const int l0 = (tile / p.nZt) * BL, z0 = (tile % p.nZt) * BZ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int rows = p.B * p.S;
  const int q_begin = kc * p.rows_per_chunk;
  const int q_end = min(p.rows_pad, q_begin + p.rows_per_chunk);
  // DMA lane mapping: RPP rows per 1-KB wave-instruction; wave w moves pieces
  // w*PER_WAVE ..; the first PIECES/2 are G rows, the rest E rows.  Per-lane
  // byte offsets (without the stage's first row) of my pieces:
  int dma_off[PER_WAVE];
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int pc = wid * PER_WAVE + i;
    const int pr = pc % (PIECES / 2);
    const int lrow = lane / (64 / RPP), lpos = lane % (64 / RPP);  // 16-B slot within the row
    const int r = pr * RPP + lrow;  // K row within the stage
    const int u_lds = lpos >> 1, half = lpos & 1;
    const int u_src = u_lds ^ (r & 7);
    dma_off[i] = 4 * (pc < PIECES / 2 ? l0 : z0) + u_src * 32 + half * 16;  // chunked: 4 B/column
  }
  // transposed-read lane mapping: lane 4q+p of its 16-lane group
  const int tq = lr >> 2, tp = lr & 3;
  const int r0 = lg * 4 + tq, r1 = r0 + 16, sw = r0 & 7;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (q_end - q_begin + kDrKR - 1) / kDrKR;
  for (int j = 0; j < P && j < nst; ++j)
    dr_issue<PER_WAVE, PIECES, RPP>(p, smem + j * STAGE, q_begin + j * kDrKR, rows, wid, dma_off);
  for (int ci = 0; ci < nst; ++ci) {
    if (P == 1)
      wait_vmcnt<0>();
    else
      wait_vmcnt_dyn(min(P - 1, nst - 1 - ci) * PER_WAVE);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_raw();  // stage ci landed for every wave; all waves are done reading ci-1
    if (ci + P < nst)
      dr_issue<PER_WAVE, PIECES, RPP>(p, smem + ((ci + P) % kDrStages) * STAGE,
                                 q_begin + (ci + P) * kDrKR, rows, wid, dma_off);
    const char* base = smem + (ci % kDrStages) * STAGE;
    s16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
    for (int m = 0; m < TM; ++m) {
      const int t = wm * TM + m, uh = (t >> 1) * 4 + (t & 1);
      const int ch = ((uh ^ sw) << 5) + tp * 8, cl = (((uh + 2) ^ sw) << 5) + tp * 8;
      ah[m] = __builtin_shufflevector(tr_read(base, r0 * ROWB + ch),
                                      tr_read(base, r1 * ROWB + ch), 0, 1, 2, 3, 4, 5, 6, 7);
      al[m] = __builtin_shufflevector(tr_read(base, r0 * ROWB + cl),
                                      tr_read(base, r1 * ROWB + cl), 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int t = wn * TN + n, uh = (t >> 1) * 4 + (t & 1);
      const int ch = ((uh ^ sw) << 5) + tp * 8, cl = (((uh + 2) ^ sw) << 5) + tp * 8;
      bh[n] = __builtin_shufflevector(tr_read(base + IMG, r0 * ROWB + ch),
                                      tr_read(base + IMG, r1 * ROWB + ch), 0, 1, 2, 3, 4, 5, 6, 7);
      bl[n] = __builtin_shufflevector(tr_read(base + IMG, r0 * ROWB + cl),
                                      tr_read(base + IMG, r1 * ROWB + cl), 0, 1, 2, 3, 4, 5, 6, 7);
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
  const float inv = 1.0f / (wave_pow2_scale(p.g_bound, p.B) * *p.eps16.scale);
  // D[i = l][j = z]: row = lg*4 + reg, col = lr
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int l = l0 + (wm * TM + m) * 16 + lg * 4 + i;
        const int zc = z0 + (wn * TN + n) * 16 + lr;
        if (l < p.L && zc < p.z) p.slab[((int64_t)kc * p.L + l) * p.z + zc] = acc[m][n][i] * inv;
      }
}

// Fragments of one dR stage (per wave: TM A tiles and TN B tiles, hi and lo).
template <int TM, int TN>
struct DrFrag {
  s16x8 ah[TM], al[TM], bh[TN], bl[TN];
};

template <int TM, int TN, int ROWB, int IMG>
MPV_DEV void dr_read(DrFrag<TM, TN>& f, const char* base, int wm, int wn, int r0, int r1, int sw,
                     int tp) {
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const int t = wm * TM + m, uh = (t >> 1) * 4 + (t & 1);
    const int ch = ((uh ^ sw) << 5) + tp * 8, cl = (((uh + 2) ^ sw) << 5) + tp * 8;
    f.ah[m] = __builtin_shufflevector(tr_read(base, r0 * ROWB + ch), tr_read(base, r1 * ROWB + ch),
                                      0, 1, 2, 3, 4, 5, 6, 7);
    f.al[m] = __builtin_shufflevector(tr_read(base, r0 * ROWB + cl), tr_read(base, r1 * ROWB + cl),
                                      0, 1, 2, 3, 4, 5, 6, 7);
  }
#pragma unroll
  for (int n = 0; n < TN; ++n) {
    const int t = wn * TN + n, uh = (t >> 1) * 4 + (t & 1);
    const int ch = ((uh ^ sw) << 5) + tp * 8, cl = (((uh + 2) ^ sw) << 5) + tp * 8;
    f.bh[n] = __builtin_shufflevector(tr_read(base + IMG, r0 * ROWB + ch),
                                      tr_read(base + IMG, r1 * ROWB + ch), 0, 1, 2, 3, 4, 5, 6, 7);
    f.bl[n] = __builtin_shufflevector(tr_read(base + IMG, r0 * ROWB + cl),
                                      tr_read(base + IMG, r1 * ROWB + cl), 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// dr_read with a group-0 wave's share of the next stage's LDS-DMA woven in:
// one or two 1-KB pieces after each tile's four transposed reads, so the
// CU's load path (the DMA) and the LDS (the reads) work side by side instead
// of the reads queueing behind the whole DMA burst (tools/studies/dr_stamps.py: DMA
// issue 1060 + reads 960 ticks, serial, against 1650 for the other group's
// MFMAs).  Noise rows past the last real one (a padded last stage) repeat
// that row, as drs_issue_range clamps them.
template <int TM, int TN, int ROWB, int IMG, int PER_WAVE, class Dma>
MPV_DEV void dr_read_dma(DrFrag<TM, TN>& f, const char* base, int wm, int wn, int r0, int r1,
                         int sw, int tp, Dma& dma, char* dst, int rows, int lane_u, int lane_h) {
  constexpr int STEPS = TM + TN;
  // the per-piece source swizzle is recomputed next to its DMA, not hoisted
  // out of the stage loop (8 more live VGPRs spill the accumulators)
  int lu = lane_u;
  asm volatile("" : "+v"(lu));
  const char* sp = dma.src;
  int nvalid = PER_WAVE;
  if (!dma.is_g) {
    const int over = dma.q - (rows - 1);
    if (over > 0) sp -= over * dma.row_b;
    nvalid = max(1, min(PER_WAVE, rows - dma.q));
  }
#pragma unroll
  for (int k = 0; k < STEPS; ++k) {
    const bool is_a = k < TM;
    const int t = is_a ? wm * TM + k : wn * TN + (k - TM), uh = (t >> 1) * 4 + (t & 1);
    const int ch = ((uh ^ sw) << 5) + tp * 8, cl = (((uh + 2) ^ sw) << 5) + tp * 8;
    const char* img = is_a ? base : base + IMG;
    const s16x8 hi = __builtin_shufflevector(tr_read(img, r0 * ROWB + ch), tr_read(img, r1 * ROWB + ch),
                                             0, 1, 2, 3, 4, 5, 6, 7);
    const s16x8 lo = __builtin_shufflevector(tr_read(img, r0 * ROWB + cl), tr_read(img, r1 * ROWB + cl),
                                             0, 1, 2, 3, 4, 5, 6, 7);
    if (is_a) {
      f.ah[k] = hi;
      f.al[k] = lo;
    } else {
      f.bh[k - TM] = hi;
      f.bl[k - TM] = lo;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = k * PER_WAVE / STEPS; i < (k + 1) * PER_WAVE / STEPS; ++i) {
      lds_dma16(sp, (uint32_t)(((lu ^ (i & 7)) << 5) + lane_h), lds_addr(dst + (dma.pc0 + i) * 1024));
      sp += (i + 1 < nvalid) ? dma.row_b : 0;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  dma.end();
}

template <int TM, int TN>
MPV_DEV void dr_mfma(f32x4 (&acc)[TM][TN], const DrFrag<TM, TN>& f) {
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

// Pieces pc0 .. pc0+COUNT-1 of one stage's LDS-DMA (one row each: the first
// PIECES/2 are G rows, the rest E rows).
template <int COUNT, int PIECES>
MPV_DEV void drs_issue_range(const Dr16Params& p, char* dst, int q0, int rows, int pc0, int l0,
                             int z0, int lane_u, int lane_h) {
#pragma unroll
  for (int i = 0; i < COUNT; ++i) {
    const int pc = pc0 + i;  // wave-uniform
    const bool is_g = pc < PIECES / 2;
    const int r = is_g ? pc : pc - PIECES / 2;
    const int q = q0 + r;
    const char* src = is_g ? reinterpret_cast<const char*>(p.g + (int64_t)q * p.gld + 2 * l0)
                           : reinterpret_cast<const char*>(p.eps16.data +
                                                           (int64_t)min(q, rows - 1) * p.eps16.ld +
                                                           2 * z0);
    lds_dma16(src, (uint32_t)(((lane_u ^ (r & 7)) << 5) + lane_h), lds_addr(dst + pc * 1024));
  }
}

// Timing study (MPV_DR_STAMPS=1 builds only, tools/studies/dr_stamps.py): s_memtime
// at the slot boundaries of workgroup 0's waves over its first kDrStampStages
// stages, stored by lane 0 with vector stores; read back through
// mpv_study_dr_stamps.
#ifndef MPV_DR_STAMPS
#define MPV_DR_STAMPS 0
#endif
[[maybe_unused]] constexpr int kDrStampStages = 64, kDrStampPts = 6;
#if MPV_DR_STAMPS
__device__ unsigned long long mpv_dr_stamps[8][kDrStampStages][kDrStampPts];
#define DR_STAMP(i, k)                                                                           \
  do {                                                                                           \
    if (blockIdx.x == 0 && (i) < kDrStampStages) {                                               \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                \
      if (lane == 0) mpv_dr_stamps[wid][(i)][(k)] = t_;                                         \
    }                                                                                            \
  } while (0)
#else
#define DR_STAMP(i, k) \
  do {                 \
  } while (0)
#endif

// A group-0 wave's share of every stage's LDS-DMA: PER_WAVE consecutive rows
// of one operand (the first WN/2 waves G rows, the others noise rows), walked
// by 64-bit pointer increments -- two SALU per row instead of the ~14 of a
// row * ld product and clamp per piece (round 5: the stage's DMA block 325 ->
// 139 instructions, dR -1.5 %, profiles/r05_dr_dma_ab.json).
template <int PER_WAVE, int PIECES, int WN>
struct DrsDma {
  const char* src;  // first row of this wave's share of the next stage
  int64_t row_b;    // bytes per source row
  int q;            // its row index
  int pc0;          // first piece (1-KB LDS row) of the share
  bool is_g;
  MPV_DEV void init(const Dr16Params& p, int q_first, int wn, int l0, int z0) {
    static_assert(PIECES / 2 == (WN / 2) * PER_WAVE, "G rows on the first half of the waves");
    static_assert(PER_WAVE % 8 == 0, "the source swizzle (row & 7) restarts with every share");
    const int pc = wn * PER_WAVE;
    is_g = pc < PIECES / 2;
    pc0 = pc;
    q = q_first + (is_g ? pc : pc - PIECES / 2);
    row_b = is_g ? p.gld * 2 : p.eps16.ld * 2;
    src = is_g ? reinterpret_cast<const char*>(p.g + (int64_t)q * p.gld + 2 * l0)
               : reinterpret_cast<const char*>(p.eps16.data + (int64_t)q * p.eps16.ld + 2 * z0);
  }
  MPV_DEV void end() {  // on to the next stage
    src += kDrKR * row_b;
    q += kDrKR;
  }
};

// Staggered schedule: the waves of row wm = 0 (group 0) and wm = 1 (group 1)
// share the SIMDs pairwise and run one phase apart, so on every SIMD one wave
// issues MFMAs while the other streams/reads.  Time is cut into slots ended by
// one barrier each; group 0 does mem(i) in slot 2i and mma(i) in slot 2i+1,
// group 1 does mem(i) in slot 2i+1 and mma(i) in slot 2i+2.
//   mem(i): fragment reads of stage i; group 0 weaves the LDS-DMA of stage i+1
//           into image (i+1)%2 (read by group 1 in slot 2i-1, so free) into
//           them (dr_read_dma).
//   mma(i): 96 MFMAs; group 0 then waits for its stage i+1 DMA, so stage i+1
//           is visible to both groups after the slot's barrier.
// Two 64-KB stage images; DMA latency budget = one slot pair.  Round 5
// (tools/studies/dr_stamps.py, profiles/r05_dr_ab.json): with the DMA as a burst ahead
// of the reads, group 0's mem slot (1060 + 960 ticks) outlasted the other
// group's MFMAs (1650) every slot; woven, dR -4.2 %.  Measured slower: group 1
// issuing the stream between its own MFMAs (+2.3 %), half of it in each
// group's read slot (+12 % woven, +0.8 % with group 1's half ahead of its
// reads).
template <int WM, int WN, int TM, int TN>
__global__ __launch_bounds__(WM* WN * 64, 1) void dR16s_kernel(Dr16Params p) {
  static_assert(WM == 2, "two wave groups");
  constexpr int BL = WM * TM * 16, BZ = WN * TN * 16;
  static_assert(BL == BZ, "square tile: one LDS row layout for both operands");
  constexpr int ROWB = BL * 4;          // bytes per LDS row: BL columns, hi + lo
  constexpr int IMG = kDrKR * ROWB;     // per operand
  constexpr int STAGE = 2 * IMG;
  constexpr int PIECES = STAGE / 1024;  // 1-KB wave-instructions per stage
  constexpr int RPP = 1024 / ROWB;      // rows per piece
  constexpr int PER_WAVE = PIECES / WN;  // pieces per group-0 wave (group 1 issues none)
  static_assert(PIECES % WN == 0, "DMA pieces must split over the waves");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  int kc, tile;
  decode_kc_tile(blockIdx.x, p.nKc, p.nLt * p.nZt, kc, tile);
  const int l0 = (tile / p.nZt) * BL, z0 = (tile % p.nZt) * BZ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int grp = wm;
  const int lr = lane & 15, lg = lane >> 4;
  const int rows = p.B * p.S;
  const int q_begin = kc * p.rows_per_chunk;
  const int q_end = min(p.rows_pad, q_begin + p.rows_per_chunk);
  static_assert(RPP == 1, "one 1-KB row per DMA piece");
  // per-lane part of a piece's source offset: 16-B slot `lane` of the row
  // (32-B unit lane/2, swizzled by the row's r & 7, which cycles with the piece)
  const int lane_u = lane >> 1, lane_h = (lane & 1) * 16;
  const int tq = lr >> 2, tp = lr & 3;
  const int r0 = lg * 4 + tq, r1 = r0 + 16, sw = r0 & 7;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (q_end - q_begin + kDrKR - 1) / kDrKR;
  if (grp == 0 && nst > 0) {
    drs_issue_range<PIECES / WN, PIECES>(p, smem, q_begin, rows, wn * (PIECES / WN), l0, z0, lane_u,
                                         lane_h);
    wait_vmcnt<0>();
  }
  DrFrag<TM, TN> f;
  DrsDma<PER_WAVE, PIECES, WN> dma;
  if (grp == 0) dma.init(p, q_begin + kDrKR, wn, l0, z0);
  barrier_raw();
  // the two groups run the same number of barriers: 2*nst + 1
  if (grp == 0) {
    // slot 2i: read stage i with stage i+1's DMA woven in; slot 2i+1: MFMAs
    // of stage i, then stage i+1 landed before the closing barrier
    int i = 0;
    for (; i + 1 < nst; ++i) {
      DR_STAMP(i, 0);
      dr_read_dma<TM, TN, ROWB, IMG, PER_WAVE>(f, smem + (i & 1) * STAGE, wm, wn, r0, r1, sw, tp,
                                               dma, smem + (1 - (i & 1)) * STAGE, rows, lane_u,
                                               lane_h);
      lds_barrier();
      DR_STAMP(i, 2);
      __builtin_amdgcn_s_setprio(1);
      dr_mfma<TM, TN>(acc, f);
      __builtin_amdgcn_s_setprio(0);
      DR_STAMP(i, 3);
      wait_vmcnt<0>();
      DR_STAMP(i, 4);
      barrier_raw();
      DR_STAMP(i, 5);
    }
    for (; i < nst; ++i) {  // the last stage: nothing to stream
      dr_read<TM, TN, ROWB, IMG>(f, smem + (i & 1) * STAGE, wm, wn, r0, r1, sw, tp);
      lds_barrier();
      __builtin_amdgcn_s_setprio(1);
      dr_mfma<TM, TN>(acc, f);
      __builtin_amdgcn_s_setprio(0);
      barrier_raw();
    }
    barrier_raw();
  } else {
    barrier_raw();
    // slot 2i+1: read stage i; slot 2i+2: MFMAs of stage i
    for (int i = 0; i < nst; ++i) {
      DR_STAMP(i, 0);
      dr_read<TM, TN, ROWB, IMG>(f, smem + (i & 1) * STAGE, wm, wn, r0, r1, sw, tp);
      lds_barrier();
      DR_STAMP(i, 2);
      __builtin_amdgcn_s_setprio(1);
      dr_mfma<TM, TN>(acc, f);
      __builtin_amdgcn_s_setprio(0);
      DR_STAMP(i, 3);
      barrier_raw();
      DR_STAMP(i, 5);
    }
  }
  const float inv = 1.0f / (wave_pow2_scale(p.g_bound, p.B) * *p.eps16.scale);
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int l = l0 + (wm * TM + m) * 16 + lg * 4 + i;
        const int zc = z0 + (wn * TN + n) * 16 + lr;
        if (l < p.L && zc < p.z) p.slab[((int64_t)kc * p.L + l) * p.z + zc] = acc[m][n][i] * inv;
      }
}

// ---------------------------------------------------------------- dR GEMM
struct DrParams {
  const float* G;    // (B*S, ldG): row q = b*S + s  (the T buffer)
  const float* eps;  // (S, B, z)
  float* slab;       // [nKc][L][z]
  int S, B, L, z;
  int ldG;  // t_cols(L)
  int nLt, nZt, nKc, rows_per_chunk;
};

constexpr int kDrBK = 32;

template <int TM, int TN>
__global__ __launch_bounds__(256) void dR_gemm_kernel(DrParams p) {
  constexpr int WM = 2, WN = 2;
  constexpr int BM = WM * TM * 16;  // l tile
  constexpr int BN = WN * TN * 16;  // z tile
  constexpr int LDG = BM + 16, LDE = BN + 16;  // conflict-free ds_read_b32 (stride = 16 mod 32)
  constexpr int G4 = kDrBK * BM / 4, E4 = kDrBK * BN / 4;
  constexpr int GV = (G4 + 255) / 256, EV = (E4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[kDrBK * (LDG + LDE)];
  float* Gs = smem;
  float* Es = smem + kDrBK * LDG;

  // block -> (kc, tile); all tiles of one kc share eps/G rows: same id mod 8
  const int nT = p.nLt * p.nZt;
  int kc, tile;
  {
    const int id = blockIdx.x, K = p.nKc;
    const int full = (K / 8) * 8 * nT;
    if (id < full) {
      const int q = id / (8 * nT), r = id % (8 * nT);
      tile = r / 8;
      kc = q * 8 + (r % 8);
    } else {
      const int r = id - full, Kr = K % 8;
      tile = r / Kr;
      kc = (K / 8) * 8 + (r % Kr);
    }
  }
  const int l0 = (tile / p.nZt) * BM, z0 = (tile % p.nZt) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int lr = lane & 15, lg = lane >> 4;
  const int S = p.S, B = p.B, L = p.L, z = p.z;
  const int rows = B * S;
  const int q_begin = kc * p.rows_per_chunk;
  const int q_end = min(rows, q_begin + p.rows_per_chunk);
  const bool gvec = true, evec = (z & 3) == 0;  // G rows: t_cols stride

  f32x4 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 rg[GV], re[EV];
  auto load = [&](int q0) {
#pragma unroll
    for (int v = 0; v < GV; ++v) {
      const int idx = tid + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (idx < G4) {
        const int r = idx / (BM / 4), c = l0 + (idx % (BM / 4)) * 4;
        const int q = q0 + r;
        if (q < q_end) {
          const float* src = p.G + (int64_t)q * p.ldG;
          if (gvec && c < L) x = *reinterpret_cast<const f32x4*>(src + c);  // pads hold G = 0
          else {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = (c + k < L) ? src[c + k] : 0.0f;
          }
        }
      }
      rg[v] = x;
    }
#pragma unroll
    for (int v = 0; v < EV; ++v) {
      const int idx = tid + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (idx < E4) {
        const int r = idx / (BN / 4), c = z0 + (idx % (BN / 4)) * 4;
        const int q = q0 + r;
        if (q < q_end) {
          const int bb = q / S, s = q - bb * S;
          const float* src = p.eps + ((int64_t)s * B + bb) * z;
          if (evec && c + 3 < z) x = *reinterpret_cast<const f32x4*>(src + c);
          else {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = (c + k < z) ? src[c + k] : 0.0f;
          }
        }
      }
      re[v] = x;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int v = 0; v < GV; ++v) {
      const int idx = tid + v * 256;
      if (idx < G4)
        *reinterpret_cast<f32x4*>(&Gs[(idx / (BM / 4)) * LDG + (idx % (BM / 4)) * 4]) = rg[v];
    }
#pragma unroll
    for (int v = 0; v < EV; ++v) {
      const int idx = tid + v * 256;
      if (idx < E4)
        *reinterpret_cast<f32x4*>(&Es[(idx / (BN / 4)) * LDE + (idx % (BN / 4)) * 4]) = re[v];
    }
  };

  if (q_begin < q_end) {
    load(q_begin);
    store();
    __syncthreads();
    for (int q0 = q_begin; q0 < q_end; q0 += kDrBK) {
      const bool more = q0 + kDrBK < q_end;
      if (more) load(q0 + kDrBK);
#pragma unroll
      for (int j = 0; j < kDrBK / 4; ++j) {
        float a[TM], bb[TN];
#pragma unroll
        for (int m = 0; m < TM; ++m) a[m] = Gs[(j * 4 + lg) * LDG + wm * TM * 16 + m * 16 + lr];
#pragma unroll
        for (int n = 0; n < TN; ++n) bb[n] = Es[(j * 4 + lg) * LDE + wn * TN * 16 + n * 16 + lr];
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int n = 0; n < TN; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bb[n], acc[m][n], 0, 0, 0);
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
  }
  // D[i = l][j = z]: row = lg*4 + reg, col = lr
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int l = l0 + wm * TM * 16 + m * 16 + lg * 4 + i;
        const int zc = z0 + wn * TN * 16 + n * 16 + lr;
        if (l < L && zc < z) p.slab[((int64_t)kc * L + l) * z + zc] = acc[m][n][i];
      }
}

// ------------------------------------------------------------------- plans
struct BwdPlan {
  int dr_tile;                                  // dR output tile edge
  int TPR, RPI, nLc, nSc, rows_per_chunk, Lc;   // element pass
  int nLt, nZt, nKc, dr_rows_per_chunk, rows_pad;  // dR GEMM
  int64_t ldg;                                  // G plane columns (3xf16, padded)
  size_t coef_bytes, colpart_bytes, slab_bytes, bound_bytes, planes_bytes;
};

constexpr int kDr16Tile = 256;  // 3xf16 dR tile: 256 x 256, 8 waves of 128 x 64
// Small label / latent dims (both <= 128, e.g. mirflickr 38, nuswide 81): a
// 128 x 128 tile (4 waves of 64 x 64, two workgroups per CU), so the G and
// noise planes are padded to 128 columns instead of 256
constexpr int kDr16TileSmall = 128;

// Both <= 64 (mirflickr 38, the fairsoft adult-like 25 x 10): a 64 x 64 tile
// (4 waves of 32 x 32), planes padded to 64 columns: half the G-plane and
// noise-plane bytes of the 128 tile at L = z = 38
constexpr int kDr16TileTiny = 64;

constexpr int kDrSmallChunksPerCu = 2;  // K chunks per CU for the 128 tile
constexpr int kDrTinyChunksPerCu = 2;   // and for the 64 tile (4 and 8 measure the same at C2)
constexpr int64_t kDrMaxChunkRows = 131072;  // longest split-K chunk (sample rows)

static int dr16_tile(int64_t L, int64_t z) {
  if (L <= kDr16TileTiny && z <= kDr16TileTiny) return kDr16TileTiny;
  return (L <= kDr16TileSmall && z <= kDr16TileSmall) ? kDr16TileSmall : kDr16Tile;
}

static BwdPlan plan_bwd(const mpv_shape* s, int gemm) {
  BwdPlan pl;
  const int64_t L = s->L, S = s->S_local, B = s->B, z = s->z;
  const bool planes = gemm == MPV_GEMM_F16X3;
  const int64_t dr_tile = planes ? dr16_tile(L, z) : 128;  // dR output tile edge
  pl.dr_tile = (int)dr_tile;
  pl.ldg = cdiv(L, dr_tile) * dr_tile;
  // columns the element pass covers: L rounded up to whole 4-column lane
  // groups (the pad columns get G = 0).  The G planes' columns beyond are
  // never written: in the dR GEMM a G column l meets only output row l, and
  // rows >= L are not stored (round 5 wrote zeros up to the 32-wide chunk:
  // L = 38 covered 64 columns, 40 now -- C2's element pass does 38 % less)
  const int64_t Lc = planes ? std::min<int64_t>(pl.ldg, cdiv(L, 4) * 4) : L;
  pl.Lc = (int)Lc;
  pl.nLc = (int)cdiv(Lc, 1024);
  pl.TPR = (int)(Lc >= 1024 ? 256 : cdiv(Lc, 4));
  pl.RPI = 256 / pl.TPR;
  // s-chunks: enough blocks for several rounds of resident blocks (short tail)
  int64_t want = cdiv(8192, B * pl.nLc);
  // but at least kElemMinRows rows per thread (block setup amortised; the
  // LDS-ring kernel, with its coefficient staging and ring prologue per block,
  // kElemRingMinRows, which matters at small n_sample: the strong-scaling share)
  const int64_t min_rows = (planes && pl.RPI == 1) ? kElemRingMinRows : kElemMinRows;
  want = std::min<int64_t>(want, cdiv(S, (int64_t)pl.RPI * min_rows));
  // but two blocks per CU at least when a thread still gets kElemMinRows / 2
  // rows (C2: 384 blocks, 1.5 per CU, left half the CUs with one wave per
  // SIMD: element pass 24.9 -> 22.3 us with 512; C3 has 2816 either way)
  const int64_t even = cdiv(2 * (int64_t)num_cus(), B * pl.nLc);
  if (want < even && cdiv(S, even * pl.RPI) >= kElemMinRows / 2) want = even;
  if (want < 1) want = 1;
  const int64_t max_chunks = cdiv(S, pl.RPI);
  if (want > max_chunks) want = max_chunks;
  pl.rows_per_chunk = (int)cdiv(S, want);
  pl.nSc = (int)cdiv(S, pl.rows_per_chunk);
  pl.nLt = (int)cdiv(L, dr_tile);
  pl.nZt = (int)cdiv(z, dr_tile);
  const int64_t rows = B * S;
  const int64_t tiles = (int64_t)pl.nLt * pl.nZt;
  const int64_t kr = 32;  // K rows per stage of either GEMM
  pl.rows_pad = (int)(cdiv(rows, kr) * kr);
  // split-K chunks: the 3xf16 kernel (1 workgroup per CU) gets one workgroup
  // per CU in a single wave of equal chunks; the fp32 kernel several per CU
  const int cpc = dr_tile == kDr16Tile ? 1 : (dr_tile == kDr16TileTiny ? kDrTinyChunksPerCu
                                                                      : kDrSmallChunksPerCu);
  int64_t kc = planes ? cdiv(cpc * (int64_t)num_cus(), tiles)
                      : cdiv(1536, tiles);
  // but no K chunk longer than kDrMaxChunkRows: one fp32 accumulator per output
  // over 4.2 M rows (C5 on one GPU: 256 tiles, so one chunk each) drifted 1e-4
  // (normwise) between two shardings of the same sum; chunks of <= 128 K rows
  // keep it at the C4 level (< 1e-5), the chunks summed in a fixed order
  kc = std::max<int64_t>(kc, cdiv(rows, kDrMaxChunkRows));
  const int64_t kc_max = cdiv(rows, 256);
  if (kc > kc_max) kc = kc_max;
  if (kc < 1) kc = 1;
  pl.dr_rows_per_chunk = (int)(cdiv(cdiv(rows, kc), kr) * kr);
  pl.nKc = (int)cdiv(rows, pl.dr_rows_per_chunk);
  pl.coef_bytes = align_up(sizeof(float) * 6 * (size_t)B * S, 256);
  pl.colpart_bytes = align_up(sizeof(float) * (size_t)pl.nSc * 2 * B * L, 256);
  pl.slab_bytes = align_up(sizeof(float) * (size_t)pl.nKc * L * z, 256);
  pl.bound_bytes = align_up(sizeof(float) * ((size_t)B + 64), 256);
  pl.planes_bytes = planes ? align_up(2 * sizeof(uint16_t) * (size_t)pl.rows_pad * pl.ldg, 256) : 0;
  return pl;
}

}  // namespace mpv

using namespace mpv;

extern "C" {

int64_t mpv_noise_plane_cols(const mpv_shape* shape) {
  if (check_shape(shape) != MPV_OK) return 0;
  const int64_t t = dr16_tile(shape->L, shape->z);
  return cdiv(shape->z, t) * t;
}

size_t mpv_bwd_workspace_bytes(const mpv_shape* shape, int gemm) {
  if (check_shape(shape) != MPV_OK) return 0;
  const BwdPlan pl = plan_bwd(shape, gemm);
  return pl.coef_bytes + pl.colpart_bytes + pl.slab_bytes + pl.bound_bytes + pl.planes_bytes;
}

int mpv_probit_bwd(const mpv_shape* shape, const mpv_bwd_args* a, void* stream) {
  if (int rc = check_shape(shape)) return rc;
  MPV_REQUIRE(a && a->y && a->fe_out && a->fx_out && a->T && a->rowstat && a->bstat &&
                  a->gscal && a->dfe_dfx && a->workspace,
              "NULL pointer in mpv_bwd_args");
  MPV_REQUIRE(a->gemm == MPV_GEMM_F32 || a->gemm == MPV_GEMM_F16X3, "unknown gemm mode %d",
              a->gemm);
  const bool planes = a->gemm == MPV_GEMM_F16X3;
  const BwdPlan pl = plan_bwd(shape, a->gemm);
  MPV_REQUIRE(!(a->dR32 && a->dR64), "dR32 or dR64, not both");
  void* const dR_out = a->dR64 ? (void*)a->dR64 : (void*)a->dR32;
  const int dR_dtype = a->dR64 ? MPV_F64 : MPV_F32;
  if (a->kl) {
    MPV_REQUIRE(a->kl->fe_mu && a->kl->fe_logvar && a->kl->fx_mu && a->kl->fx_logvar &&
                    a->kl->gscal && a->kl->g_fe_mu && a->kl->g_fe_logvar && a->kl->g_fx_mu &&
                    a->kl->g_fx_logvar && a->kl->B > 0 && a->kl->d > 0,
                "bad kl arguments");
  }
  if (dR_out) {
    if (planes) {
      MPV_REQUIRE(a->eps16.data && a->eps16.scale, "eps16 planes are NULL");
      MPV_REQUIRE(a->eps16.ld >= 2 * (int64_t)pl.nZt * pl.dr_tile && a->eps16.ld % 64 == 0 &&
                      a->eps16.rows_pad >= shape->S_local * shape->B,
                  "eps16 planes too small (ld %lld < %lld: mpv_noise_plane_cols)",
                  (long long)a->eps16.ld, 2 * (long long)pl.nZt * pl.dr_tile);
    } else {
      MPV_REQUIRE(a->eps != nullptr, "MPV_GEMM_F32 needs eps");
    }
  }
  const size_t need = pl.coef_bytes + pl.colpart_bytes + pl.slab_bytes + pl.bound_bytes +
                      pl.planes_bytes;
  MPV_REQUIRE(a->workspace_bytes >= need, "workspace too small: %zu < %zu", a->workspace_bytes,
              need);
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(a->workspace);
  float* coef = reinterpret_cast<float*>(ws);
  float* colpart = reinterpret_cast<float*>(ws + pl.coef_bytes);
  float* slab = reinterpret_cast<float*>(ws + pl.coef_bytes + pl.colpart_bytes);
  float* gbound = reinterpret_cast<float*>(ws + pl.coef_bytes + pl.colpart_bytes + pl.slab_bytes);
  // G planes, chunked: rows_pad rows of gld = 2 * ldg halves
  uint16_t* g16 = reinterpret_cast<uint16_t*>(ws + pl.coef_bytes + pl.colpart_bytes +
                                              pl.slab_bytes + pl.bound_bytes);
  const int64_t gld = 2 * pl.ldg;
  const int S = (int)shape->S_local, B = (int)shape->B, L = (int)shape->L, z = (int)shape->z;
  const bool want_planes = planes && dR_out != nullptr;

  mpv_kl_bwd_args kl{};
  int kl_blocks = 0;
  if (a->kl) {
    kl = *a->kl;
    kl_blocks = (int)std::min<int64_t>(cdiv(kl.B * kl.d, kCoefThreads), 256);
  }
  MPV_LAUNCH("bwd_coef", bwd_coef_kernel, dim3(B + kl_blocks), dim3(kCoefThreads), 0, st, a->y, a->rowstat,
             a->bstat, a->gscal, a->g_indiv, a->g_indiv_label, coef,
             want_planes ? gbound : nullptr, S, B, L, (float)shape->S_total, a->nll_coeff,
             a->c_coeff, a->live, kl, kl_blocks);
  if (int rc = check_launch("bwd_coef")) return rc;
  if (want_planes) {
    const int64_t pad_rows = (int64_t)pl.rows_pad - (int64_t)B * S;
    if (pad_rows > 0) {
      const size_t off = (size_t)B * S * gld, n = (size_t)pad_rows * gld * sizeof(uint16_t);
      if (hipMemsetAsync(g16 + off, 0, n, st) != hipSuccess)
        return fail(MPV_ELAUNCH, "memset of G pad rows failed");
    }
  }

  ElemParams ep;
  ep.y = a->y;
  ep.fe = a->fe_out;
  ep.fx = a->fx_out;
  ep.gI = a->g_indiv;
  ep.gIL = a->g_indiv_label;
  ep.coef = coef;
  ep.T = a->T;
  ep.g = want_planes ? g16 : nullptr;
  ep.g_bound = gbound;
  ep.gld = gld;
  ep.colpart = colpart;
  ep.S = S;
  ep.B = B;
  ep.L = L;
  ep.ldT = (int)t_cols(L);
  ep.Lc = want_planes ? pl.Lc : L;
  ep.TPR = pl.TPR;
  ep.RPI = pl.RPI;
  ep.rows_per_chunk = pl.rows_per_chunk;
  ep.inv_S = 1.0f / (float)shape->S_total;
  const dim3 eg(B, pl.nSc, pl.nLc);
  // t_cols rows: 16-B aligned, whole float4 reads (VEC)
  if (want_planes && pl.RPI == 1)  // L >= 1024: the LDS-ring element pass
    MPV_LAUNCH("bwd_elem", bwd_elem_ring_kernel, eg, dim3(256), 0, st, ep);
  else if (want_planes)
    MPV_LAUNCH("bwd_elem", (bwd_elem_kernel<true, true, false>), eg, dim3(256), 0, st, ep);
  else
    MPV_LAUNCH("bwd_elem", (bwd_elem_kernel<true, false, false>), eg, dim3(256), 0, st, ep);
  if (int rc = check_launch("bwd_elem")) return rc;
  if (!dR_out) {
    if (int rc = launch_sum_slabs(colpart, pl.nSc, 2 * (int64_t)B * L, a->dfe_dfx, MPV_F32, st))
      return rc;
  }

  if (dR_out) {
    const int64_t blocks = (int64_t)pl.nLt * pl.nZt * pl.nKc;
    if (planes) {
      Dr16Params dp;
      dp.g = g16;
      dp.g_bound = gbound;
      dp.gld = gld;
      dp.eps16 = a->eps16;
      dp.slab = slab;
      dp.S = S;
      dp.B = B;
      dp.L = L;
      dp.z = z;
      dp.nLt = pl.nLt;
      dp.nZt = pl.nZt;
      dp.nKc = pl.nKc;
      dp.rows_per_chunk = pl.dr_rows_per_chunk;
      dp.rows_pad = pl.rows_pad;
      // 256 x 256 tile, 8 waves of 128 x 64, 2-stage ring (128 KB LDS)
      static_assert(kDr16Tile == 256 && kDr16TileSmall == 128 && kDr16TileTiny == 64,
                    "launch configs below");
      if (pl.dr_tile == kDr16TileTiny)  // 64 x 64, 4 waves of 32 x 32, 2 x 16 KB stages
        MPV_LAUNCH("dR_gemm", (dR16_kernel<2, 2, 2, 2, 2>), dim3((unsigned)blocks), dim3(256), 0, st, dp);
      else if (pl.dr_tile == kDr16TileSmall)  // 128 x 128, 4 waves of 64 x 64, 2 x 32 KB stages
        MPV_LAUNCH("dR_gemm", (dR16_kernel<2, 2, 4, 4, 2>), dim3((unsigned)blocks), dim3(256), 0, st, dp);
      else  // 256 x 256, two wave groups one phase apart (dR16s)
        MPV_LAUNCH("dR_gemm", (dR16s_kernel<2, 4, 8, 4>), dim3((unsigned)blocks), dim3(512), 0, st, dp);
    } else {
      DrParams dp;
      dp.G = a->T;
      dp.eps = a->eps;
      dp.slab = slab;
      dp.S = S;
      dp.B = B;
      dp.L = L;
      dp.ldG = (int)t_cols(L);
      dp.z = z;
      dp.nLt = pl.nLt;
      dp.nZt = pl.nZt;
      dp.nKc = pl.nKc;
      dp.rows_per_chunk = pl.dr_rows_per_chunk;
      MPV_LAUNCH("dR_gemm", (dR_gemm_kernel<4, 4>), dim3((unsigned)blocks), dim3(256), 0, st, dp);
    }
    if (int rc = check_launch("dR_gemm")) return rc;
    // the column partials (d fe_out, d fx_out) and the dR slabs in one launch
    if (int rc = launch_sum_slabs_pair(colpart, pl.nSc, 2 * (int64_t)B * L, a->dfe_dfx, MPV_F32,
                                       slab, pl.nKc, (int64_t)L * z, dR_out, dR_dtype, st))
      return rc;
  }
  return MPV_OK;
}

#if MPV_DR_STAMPS
// study builds only: copy workgroup 0's slot stamps (8 x 64 x 6 u64) to host
int mpv_study_dr_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mpv_dr_stamps), sizeof(mpv_dr_stamps), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif
}  // extern "C"
