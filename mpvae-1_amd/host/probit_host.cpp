// libmpvae_host.so: the probit-ELBO hot path on host memory (include/mpvae_host.h).
//
// The product's CPU backend for CPU tensors (the reference's CPU runs, BASELINE
// configs[0]); the GPU path is libmpvae_hip.so.  The same algorithm as the HIP
// kernels -- factorised ranking loss, exact log-sum-exp, analytic backward --
// written for cores instead of wavefronts: one batch row per OpenMP task (its
// S samples in order, so the column sums and the row statistics need no
// cross-thread reduction), dR one output row per task.  Every sum has a fixed
// order: results do not depend on the thread count.
//
// Built with -ffp-contract=off: E is formed op by op in fp32 exactly as the
// reference's torch ops round it (mpvae.py:171-180).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include <omp.h>

#include "mpvae_host.h"

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return MPV_EINVAL;
}

#define REQ(cond, ...)               \
  do {                               \
    if (!(cond)) return fail(__VA_ARGS__); \
  } while (0)

constexpr float kEps1 = 1e-6f;
constexpr float kC1 = 1.0f - kEps1;  // (1 - eps1) in fp32 (mpvae.py:156,177)
constexpr float kC0 = kEps1 * 0.5f;  // eps1 * 0.5
constexpr double kInvSqrt2Pi = 0.3989422804014327;
constexpr double kKlEps = 1e-6;      // mpvae.py:148
constexpr double kKlWeight = 1.1;    // mpvae.py:208

// E = Normal(0,1).cdf(u) (1 - eps1) + eps1 / 2 in fp32, the reference's op
// order: x = u / sqrt(2) as an fp32 division (torch divides by the Python
// float, rounded to fp32), erf rounded to fp32, cdf = 0.5 (1 + erf), then
// cdf (1 - eps1) and + eps1 / 2, each rounded.
inline float probit_E(float u) {
  const float x = u / 1.41421356237309515f;
  const float e = static_cast<float>(std::erf(static_cast<double>(x)));
  const float cdf = 0.5f * (1.0f + e);
  return cdf * kC1 + kC0;
}

int check_shape(const mpv_shape* s) {
  REQ(s != nullptr, "shape is NULL");
  REQ(s->S_local > 0 && s->S_total >= s->S_local && s->s_offset >= 0 && s->B > 0 && s->L > 0 &&
          s->z > 0,
      "bad shape (S_local %lld, S_total %lld, B %lld, L %lld, z %lld)", (long long)s->S_local,
      (long long)s->S_total, (long long)s->B, (long long)s->L, (long long)s->z);
  return MPV_OK;
}

// R.float() (mpvae.py:165) as fp64 values, (L, z)
std::vector<double> r_as_f32(const void* R, int dt, int64_t n) {
  std::vector<double> out(n);
  if (dt == MPV_F64) {
    const double* r = static_cast<const double*>(R);
    for (int64_t i = 0; i < n; ++i) out[i] = static_cast<double>(static_cast<float>(r[i]));
  } else {
    const float* r = static_cast<const float*>(R);
    for (int64_t i = 0; i < n; ++i) out[i] = static_cast<double>(r[i]);
  }
  return out;
}

// t = eps[s, b, :] . R^T, accumulated in fp64, rounded once (the HIP kernels'
// t is at least this accurate: tests/test_gpu_parity.py _t_accuracy)
inline void noise_product(const float* e, const double* Rd, int64_t L, int64_t z, float* t) {
  for (int64_t l = 0; l < L; ++l) {
    const double* r = Rd + l * z;
    double acc = 0.0;
    for (int64_t k = 0; k < z; ++k) acc += static_cast<double>(e[k]) * r[k];
    t[l] = static_cast<float>(acc);
  }
}

// |pos| * |neg| of a label row (mpvae.py:115-117)
inline double row_norm(const float* y, int64_t L) {
  double np = 0.0, nn = 0.0;
  for (int64_t l = 0; l < L; ++l) {
    np += y[l] == 1.0f ? 1.0 : 0.0;
    nn += y[l] == 0.0f ? 1.0 : 0.0;
  }
  return np * nn;
}

}  // namespace

extern "C" {

int mpvh_abi_version(void) { return MPVH_ABI_VERSION; }

const char* mpvh_last_error(void) { return g_err.c_str(); }

int mpvh_set_threads(int n) {
  REQ(n >= 0, "thread count %d < 0", n);
  omp_set_num_threads(n > 0 ? n : omp_get_num_procs());
  return MPV_OK;
}

int mpvh_probit_fwd(const mpv_shape* shape, const mpvh_fwd_args* a) {
  if (int rc = check_shape(shape)) return rc;
  REQ(a && a->y && a->fe_out && a->fx_out && a->R && a->eps && a->rowstat && a->bstat &&
          a->colsum,
      "NULL pointer in mpvh_fwd_args");
  REQ(a->R_dtype == MPV_F32 || a->R_dtype == MPV_F64, "unsupported R dtype %d", a->R_dtype);
  const int64_t S = shape->S_local, B = shape->B, L = shape->L, z = shape->z;
  const std::vector<double> Rd = r_as_f32(a->R, a->R_dtype, L * z);
#pragma omp parallel
  {
    std::vector<float> t(L);
    std::vector<double> cs(2 * L);
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
      const float* y = a->y + b * L;
      const double n = row_norm(y, L);
      std::fill(cs.begin(), cs.end(), 0.0);
      double m[2] = {-INFINITY, -INFINITY}, csum[2] = {0.0, 0.0};
      for (int64_t s = 0; s < S; ++s) {
        noise_product(a->eps + (s * B + b) * z, Rd.data(), L, z, t.data());
        if (a->T) std::copy(t.begin(), t.end(), a->T + (s * B + b) * L);
        for (int br = 0; br < 2; ++br) {
          const float* base = (br == 0 ? a->fe_out : a->fx_out) + b * L;
          double logp = 0.0, P = 0.0, N = 0.0;
          for (int64_t l = 0; l < L; ++l) {
            const double E = probit_E(t[l] + base[l]);  // u = t + fe_out in fp32 (mpvae.py:168)
            const double yv = y[l];
            // BCE log-probability (mpvae.py:184-185); ranking factors
            // P = sum_pos e^{-5E}, N = sum_neg e^{5E} (mpvae.py:110-114 factorised)
            logp += yv * std::log(E) + (1.0 - yv) * std::log(1.0 - E);
            if (y[l] == 1.0f) P += std::exp(-5.0 * E);
            if (y[l] == 0.0f) N += std::exp(5.0 * E);
            cs[br * L + l] += E;
          }
          a->rowstat[((int64_t)br * B + b) * S + s] = logp;
          a->rowstat[((int64_t)(2 + 2 * br) * B + b) * S + s] = P;
          a->rowstat[((int64_t)(3 + 2 * br) * B + b) * S + s] = N;
          m[br] = std::max(m[br], logp);
          const double c = P * N / (5.0 * n);  // inf / nan (no pos or neg) -> 0 (mpvae.py:119-121)
          csum[br] += std::isfinite(c) ? c : 0.0;
        }
      }
      for (int br = 0; br < 2; ++br) {
        double Z = 0.0;
        for (int64_t s = 0; s < S; ++s)
          Z += std::exp(a->rowstat[((int64_t)br * B + b) * S + s] - m[br]);
        a->bstat[(2 * br) * B + b] = m[br];
        a->bstat[(2 * br + 1) * B + b] = Z;
        a->bstat[(4 + br) * B + b] = csum[br];
        for (int64_t l = 0; l < L; ++l) a->colsum[((int64_t)br * B + b) * L + l] = cs[br * L + l];
      }
    }
  }
  return MPV_OK;
}

int mpvh_bstat_combine(const double* g, int64_t R, int64_t B, double* out) {
  REQ(g && out && R > 0 && B > 0, "bad bstat_combine arguments");
  for (int64_t b = 0; b < B; ++b) {
    for (int br = 0; br < 2; ++br) {
      const int mi = 2 * br, zi = 2 * br + 1;
      double M = -INFINITY;
      for (int64_t r = 0; r < R; ++r) M = std::max(M, g[(r * 6 + mi) * B + b]);
      double Z = 0.0;
      for (int64_t r = 0; r < R; ++r) Z += g[(r * 6 + zi) * B + b] * std::exp(g[(r * 6 + mi) * B + b] - M);
      out[mi * B + b] = M;
      out[zi * B + b] = Z;
    }
    for (int k = 4; k < 6; ++k) {
      double acc = 0.0;
      for (int64_t r = 0; r < R; ++r) acc += g[(r * 6 + k) * B + b];
      out[k * B + b] = acc;
    }
  }
  return MPV_OK;
}

int mpvh_probit_finalize(const mpv_shape* shape, const mpvh_final_args* a) {
  REQ(shape && shape->B > 0 && shape->L > 0 && shape->S_total > 0, "bad shape");
  REQ(a && a->bstat && a->colsum && a->fe_mu && a->fe_logvar && a->fx_mu && a->fx_logvar &&
          a->out6 && a->indiv_prob && a->indiv_prob_label && a->d > 0,
      "NULL pointer in mpvh_final_args");
  const int64_t B = shape->B, L = shape->L, d = a->d;
  const double S = static_cast<double>(shape->S_total);
  double nll = 0.0, nll_x = 0.0, ce = 0.0, cx = 0.0, kl = 0.0;
  // nll = mean_b(-log(mean_s exp(logp - max)) - max)   (mpvae.py:188-190)
  for (int64_t b = 0; b < B; ++b) {
    nll += -std::log(a->bstat[1 * B + b] / S) - a->bstat[0 * B + b];
    nll_x += -std::log(a->bstat[3 * B + b] / S) - a->bstat[2 * B + b];
    ce += a->bstat[4 * B + b];
    cx += a->bstat[5 * B + b];
  }
  // KL (mpvae.py:147-148)
  for (int64_t b = 0; b < B; ++b) {
    double row = 0.0;
    for (int64_t j = 0; j < d; ++j) {
      const int64_t i = b * d + j;
      const double lve = a->fe_logvar[i], lvx = a->fx_logvar[i];
      const double dm = static_cast<double>(a->fx_mu[i]) - a->fe_mu[i];
      row += (lvx - lve) - 1.0 + std::exp(lve - lvx) + dm * dm / (std::exp(lvx) + kKlEps);
    }
    kl += 0.5 * row;
  }
  nll /= B;
  nll_x /= B;
  const double c = ce / (S * B), c_x = cx / (S * B);
  kl /= B;
  const double total = (nll + nll_x) * a->nll_coeff + (c + c_x) * a->c_coeff + kl * kKlWeight;
  const double v[6] = {total, nll, nll_x, c, c_x, kl};
  for (int k = 0; k < 6; ++k) a->out6[k] = static_cast<float>(v[k]);
  for (int64_t i = 0; i < B * L; ++i) {  // mpvae.py:203-204
    a->indiv_prob_label[i] = static_cast<float>(a->colsum[i] / S);
    a->indiv_prob[i] = static_cast<float>(a->colsum[B * L + i] / S);
  }
  return MPV_OK;
}

int mpvh_probit_bwd(const mpv_shape* shape, const mpvh_bwd_args* a) {
  if (int rc = check_shape(shape)) return rc;
  REQ(a && a->y && a->fe_out && a->fx_out && a->eps && a->T && a->rowstat && a->bstat &&
          a->gscal && a->dfe_dfx,
      "NULL pointer in mpvh_bwd_args");
  const int64_t S = shape->S_local, B = shape->B, L = shape->L, z = shape->z;
  const double St = static_cast<double>(shape->S_total);
  const int live = a->live;
  auto gs = [&](int k) { return (live & MPV_LIVE(k)) ? static_cast<double>(a->gscal[k]) : 0.0; };
  const bool tl = live & MPV_LIVE(MPV_G_TOTAL);
  // the components' upstream gradients; a component is live when any gradient
  // reaches it (that is what makes a degenerate row NaN, mpvae.py:118)
  const double gt = gs(MPV_G_TOTAL);
  const bool nlive[2] = {tl || (live & MPV_LIVE(MPV_G_NLL)), tl || (live & MPV_LIVE(MPV_G_NLL_X))};
  const bool clive[2] = {tl || (live & MPV_LIVE(MPV_G_C)), tl || (live & MPV_LIVE(MPV_G_C_X))};
  const double gn[2] = {gs(MPV_G_NLL) + a->nll_coeff * gt, gs(MPV_G_NLL_X) + a->nll_coeff * gt};
  const double gc[2] = {gs(MPV_G_C) + a->c_coeff * gt, gs(MPV_G_C_X) + a->c_coeff * gt};
  std::vector<double> G(a->dR ? S * B * L : 0);
#pragma omp parallel
  {
    std::vector<double> acc(2 * L);
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
      const float* y = a->y + b * L;
      const double n = row_norm(y, L);
      std::fill(acc.begin(), acc.end(), 0.0);
      for (int64_t s = 0; s < S; ++s) {
        const float* t = a->T + (s * B + b) * L;
        for (int br = 0; br < 2; ++br) {
          const float* base = (br == 0 ? a->fe_out : a->fx_out) + b * L;
          const float* gind = br == 0 ? a->g_indiv_label : a->g_indiv;
          // row coefficients: alpha = -g_nll softmax_s(logp) / B, and the
          // ranking betaP = g_c N / (n S B), betaN = g_c P / (n S B); a row
          // with no positive or no negative label is NaN when its ranking
          // term is live (the 0/0 of mpvae.py:118 under autograd)
          const double lp = a->rowstat[((int64_t)br * B + b) * S + s];
          const double P = a->rowstat[((int64_t)(2 + 2 * br) * B + b) * S + s];
          const double N = a->rowstat[((int64_t)(3 + 2 * br) * B + b) * S + s];
          const double M = a->bstat[(2 * br) * B + b], Z = a->bstat[(2 * br + 1) * B + b];
          const double alpha = nlive[br] ? -gn[br] * (std::exp(lp - M) / Z) / B : 0.0;
          double bP = 0.0, bN = 0.0;
          if (clive[br]) {
            const double sc = gc[br] / (n * St * B);
            bP = n == 0.0 ? NAN : sc * N;
            bN = n == 0.0 ? NAN : sc * P;
          }
          const bool dead = std::isnan(bP) || std::isnan(bN);
          for (int64_t l = 0; l < L; ++l) {
            const float u32 = t[l] + base[l];
            const double E = probit_E(u32), yv = y[l];
            double gE = alpha * (yv / E - (1.0 - yv) / (1.0 - E));
            if (y[l] == 1.0f) gE -= bP * std::exp(-5.0 * E);
            if (y[l] == 0.0f) gE += bN * std::exp(5.0 * E);
            if (dead) gE = NAN;  // every label of the row, whatever its value
            if (gind) gE += static_cast<double>(gind[b * L + l]) / St;
            const double u = u32;
            const double gu = gE * static_cast<double>(kC1) * kInvSqrt2Pi * std::exp(-0.5 * u * u);
            acc[br * L + l] += gu;
            if (a->dR) {
              double& g = G[(s * B + b) * L + l];
              g = br == 0 ? gu : g + gu;
            }
          }
        }
      }
      for (int br = 0; br < 2; ++br)
        for (int64_t l = 0; l < L; ++l) a->dfe_dfx[((int64_t)br * B + b) * L + l] = acc[br * L + l];
    }
    if (a->dR) {
      // dR[l, k] = sum_{s,b} G[s,b,l] eps[s,b,k], rows (s, b) in order
#pragma omp for schedule(static)
      for (int64_t l = 0; l < L; ++l) {
        double* out = a->dR + l * z;
        std::fill(out, out + z, 0.0);
        for (int64_t r = 0; r < S * B; ++r) {
          const double g = G[r * L + l];
          const float* e = a->eps + r * z;
          for (int64_t k = 0; k < z; ++k) out[k] += g * e[k];
        }
      }
    }
  }
  return MPV_OK;
}

int mpvh_kl_bwd(const float* fe_mu, const float* fe_logvar, const float* fx_mu,
                const float* fx_logvar, int64_t B, int64_t d, const float* gscal, int live,
                float* g_fe_mu, float* g_fe_logvar, float* g_fx_mu, float* g_fx_logvar) {
  REQ(fe_mu && fe_logvar && fx_mu && fx_logvar && gscal && g_fe_mu && g_fe_logvar && g_fx_mu &&
          g_fx_logvar && B > 0 && d > 0,
      "bad kl_bwd arguments");
  const double gk = (live & MPV_LIVE(MPV_G_KL)) ? gscal[MPV_G_KL] : 0.0;
  const double gt = (live & MPV_LIVE(MPV_G_TOTAL)) ? gscal[MPV_G_TOTAL] : 0.0;
  const double s = 0.5 * (gk + kKlWeight * gt) / B;
  for (int64_t i = 0; i < B * d; ++i) {
    const double ex = std::exp(static_cast<double>(fx_logvar[i]));
    const double den = ex + kKlEps;
    const double dm = static_cast<double>(fx_mu[i]) - fe_mu[i];
    const double r = std::exp(static_cast<double>(fe_logvar[i]) - fx_logvar[i]);
    g_fe_mu[i] = static_cast<float>(s * (-2.0 * dm / den));
    g_fx_mu[i] = static_cast<float>(s * (2.0 * dm / den));
    g_fe_logvar[i] = static_cast<float>(s * (-1.0 + r));
    g_fx_logvar[i] = static_cast<float>(s * (1.0 - r - dm * dm * ex / (den * den)));
  }
  return MPV_OK;
}

}  // extern "C"
