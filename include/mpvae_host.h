/* C ABI of libmpvae_host.so: the probit-ELBO hot path on host (CPU) memory.
 *
 * The reference runs its small configurations on the CPU (BASELINE configs[0]:
 * script/run_train_mirflickr.sh on a machine without a GPU;
 * fairsoft_trial.py:157-158 picks the CPU device when CUDA is absent).  This
 * library is the product's CPU backend for CPU tensors -- compute_loss
 * dispatches on the tensors' device, it is not a fallback for a missing GPU
 * library (CUDA tensors without libmpvae_hip.so still raise).  It computes the
 * same per-shard quantities as the HIP entry points of include/mpvae_hip.h
 * (mpv_probit_fwd / mpv_bstat_combine / mpv_probit_finalize / mpv_probit_bwd /
 * mpv_kl_bwd), with the same algorithm: the factorised ranking loss
 * (P * N instead of the (S, B, L, L) tensor of mpvae.py:103-123), the exact
 * log-sum-exp combine, and the analytic backward.  Numerics: t = eps . R^T
 * accumulated in fp64 and rounded once to fp32; E = Phi(u)(1-1e-6)+0.5e-6 in
 * fp32 in the reference's op order (mpvae.py:171-180); everything after E in
 * fp64.  Parallel over (s, b) rows and dR rows with OpenMP; every sum runs in a
 * fixed order (results do not depend on the thread count).
 *
 * Shapes follow include/mpvae_hip.h (mpv_shape: this shard's S_local samples
 * of S_total).  All pointers are host pointers, row-major, contiguous. */
#ifndef MPVAE_HOST_H
#define MPVAE_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "mpvae_hip.h" /* mpv_shape, mpv_status, mpv_dtype, mpv_gslot, MPV_LIVE */

#ifdef __cplusplus
extern "C" {
#endif

#define MPVH_ABI_VERSION 1

int mpvh_abi_version(void);
const char* mpvh_last_error(void);

/* OpenMP threads of the calls below (0: one per core).  The results do not
 * depend on it (every sum runs in a fixed order). */
int mpvh_set_threads(int n);

/* Replaces mpvae.py:165-204 for one S-shard (mpv_probit_fwd's host twin). */
typedef struct mpvh_fwd_args {
  const float* y;       /* (B,L) */
  const float* fe_out;  /* (B,L) */
  const float* fx_out;  /* (B,L) */
  const void* R;        /* (L,z) r_sqrt_sigma, fp32 or fp64 (R_dtype); used as R.float() */
  int R_dtype;          /* mpv_dtype */
  const float* eps;     /* (S_local,B,z) noise */
  float* T;             /* (S_local,B,L) out: t = eps . R^T, for the backward; or NULL */
  double* rowstat;      /* (6,B,S_local) out: logp, logp_x, P, N, P_x, N_x */
  double* bstat;        /* (6,B) out: shard max / sum-exp of logp (two branches), ranking sums */
  double* colsum;       /* (2,B,L) out: sums over s of E and E_x */
} mpvh_fwd_args;

int mpvh_probit_fwd(const mpv_shape* shape, const mpvh_fwd_args* args);

/* Exact combine of per-shard bstat gathered as (nshards,6,B) -> (6,B). */
int mpvh_bstat_combine(const double* gathered, int64_t nshards, int64_t B, double* out);

/* Replaces mpvae.py:147-148 (KL), :188-190, :122, :203-210 from the global
 * statistics.  out6: total, nll, nll_x, c, c_x, kl. */
typedef struct mpvh_final_args {
  const double* bstat;   /* (6,B) global */
  const double* colsum;  /* (2,B,L) global */
  const float* fe_mu;    /* (B,d) */
  const float* fe_logvar;
  const float* fx_mu;
  const float* fx_logvar;
  int64_t d;
  float nll_coeff, c_coeff;
  float* out6;
  float* indiv_prob;        /* (B,L) */
  float* indiv_prob_label;  /* (B,L) */
} mpvh_final_args;

int mpvh_probit_finalize(const mpv_shape* shape, const mpvh_final_args* args);

/* The analytic backward of one shard (mpv_probit_bwd's host twin). */
typedef struct mpvh_bwd_args {
  const float* y;
  const float* fe_out;
  const float* fx_out;
  const float* eps;         /* (S_local,B,z) */
  const float* T;           /* (S_local,B,L) from mpvh_probit_fwd */
  const double* rowstat;    /* (6,B,S_local) from mpvh_probit_fwd */
  const double* bstat;      /* (6,B) GLOBAL */
  const float* gscal;       /* (6) upstream gradients, mpv_gslot order; slots not live unread */
  int live;                 /* MPV_LIVE bits */
  const float* g_indiv;     /* (B,L) grad of indiv_prob, or NULL */
  const float* g_indiv_label; /* (B,L) grad of indiv_prob_label, or NULL */
  float nll_coeff, c_coeff;
  double* dfe_dfx;          /* (2,B,L) out: this shard's d fe_out, d fx_out */
  double* dR;               /* (L,z) out: this shard's d r_sqrt_sigma, or NULL */
} mpvh_bwd_args;

int mpvh_probit_bwd(const mpv_shape* shape, const mpvh_bwd_args* args);

/* d KL / d (mu, logvar) (mpvae.py:147-148) scaled by gscal[KL] + 1.1 gscal[TOTAL]
 * (live slots only); outputs (B,d) fp32. */
int mpvh_kl_bwd(const float* fe_mu, const float* fe_logvar, const float* fx_mu,
                const float* fx_logvar, int64_t B, int64_t d, const float* gscal, int live,
                float* g_fe_mu, float* g_fe_logvar, float* g_fx_mu, float* g_fx_logvar);

#ifdef __cplusplus
}
#endif

#endif /* MPVAE_HOST_H */
