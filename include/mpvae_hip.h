/*
 * mpvae_hip.h -- C ABI of the MI355X (gfx950) MPVAE probit-ELBO hot path.
 *
 * libmpvae_hip.so exports exactly the functions below: plain C types, raw
 * device pointers, sizes, and a hipStream_t passed as `void*`.  Every call is
 * stream-ordered and asynchronous (no host sync, no allocation: scratch comes
 * from a caller-owned workspace); the return value is MPV_OK or an MPV_E*
 * code, with a message in mpv_last_error() (thread-local).
 *
 * The reference (lliutianc/MPVAE-1) is pure PyTorch with no FFI; each entry
 * point names the reference lines whose semantics it implements.  The Python
 * host layer (mpvae-1_amd/mpvae.py) binds them with ctypes behind the
 * reference's own `VAE` / `compute_loss` API.
 *
 * Layouts (row-major, fp32 unless stated):
 *   y, fe_out, fx_out           (B, L)          labels and the two probit means
 *   R                           (L, z)          r_sqrt_sigma (fp64 or fp32)
 *   eps                         (S_local, B, z) probit noise of this S-shard
 *   T                           (B, S_local, L) t = eps . R^T, kept for backward
 *   rowstat                     (6, B, S_local) [logp_e, logp_x, P_e, N_e, P_x, N_x]
 *   bstat                       (6, B)          [m_e, Z_e, m_x, Z_x, csum_e, csum_x]
 *   colsum                      (2, B, L)       [sum_s E, sum_s E_x]
 * "_e" = label branch (E, mpvae.py:177), "_x" = feature branch (E_x, :180).
 */
#ifndef MPVAE_HIP_H
#define MPVAE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPV_ABI_VERSION 10 /* 4: device-memory Philox keys (mpv_noise_philox*_dev);
                              5: T rows padded to roundup(L, 4) floats;
                              6: mpv_linear (the VAE's Linear layers); mpv_bwd_args
                                 dR64 and kl;
                              7: mpv_linear_batch takes up to 4 problems
                              8: mpv_adam_step; mpv_reparam_bwd_args adds
                                 the other consumers' mu / logvar gradients;
                                 mpv_linear_args second reduction segment;
                              9: mpv_adam_step reads the step count without
                                 advancing it (mpv_adam_finish does, with the
                                 update counter and a device StepLR); lr may
                                 live in device memory;
                             10: mpv_probit_finalize_shards (the cross-shard
                                 combine folded into the finalize launch); only
                                 the live slots of gscal are read (mpv_kl_bwd_args
                                 .live); mpv_noise_philox_f16_split;
                                 mpv_final_args.seed_advance */

enum mpv_status { MPV_OK = 0, MPV_EINVAL = 1, MPV_ELAUNCH = 2 };
enum mpv_dtype { MPV_F32 = 0, MPV_F64 = 1 };

/* Upstream-gradient slots of the 6 scalar outputs (gscal[] index) and the
 * matching liveness bits: a slot is live when autograd delivered a gradient
 * for it (even 0) -- that is what makes degenerate label rows NaN, exactly as
 * the reference's 0/0 in build_multi_classification_loss (mpvae.py:118). */
enum mpv_gslot { MPV_G_TOTAL = 0, MPV_G_NLL, MPV_G_NLL_X, MPV_G_C, MPV_G_C_X, MPV_G_KL };
#define MPV_LIVE(slot) (1 << (slot))

typedef struct mpv_shape {
  int64_t S_local;  /* Monte-Carlo samples held by this shard                */
  int64_t S_total;  /* samples over all shards (n_train/n_test_sample)       */
  int64_t s_offset; /* global index of this shard's first sample             */
  int64_t B, L, z;  /* batch, label_dim, z_dim                               */
} mpv_shape;

int mpv_abi_version(void);
const char* mpv_last_error(void);

/* Replaces mpvae.py:162 (noise = torch.normal(0,1,(S,B,z))) in perf mode:
 * counter-based Philox4x32-10 + Box-Muller keyed on the GLOBAL element index
 * ((s_offset+s)*B+b)*z+k, so any S-sharding draws the same noise. */
int mpv_noise_philox(float* eps, const mpv_shape* shape, uint64_t seed, uint64_t offset,
                     void* stream);

/* The same draw with the 64-bit Philox key read from device memory at run
 * time (seed_dev: one uint64 in device memory), so a step captured in a HIP
 * graph draws fresh noise on each replay when the step advances that word,
 * and the sharded path agrees on rank 0's key by a broadcast with no host
 * sync.  Same numbers as mpv_noise_philox with seed = *seed_dev. */
int mpv_noise_philox_dev(float* eps, const mpv_shape* shape, const uint64_t* seed_dev,
                         uint64_t offset, void* stream);

/* Raw Philox4x32-10 words (known-answer tests): out[4*i..4*i+3] =
 * philox(counter = ctr0 + i (as lo,hi,0,0), key = key). */
int mpv_philox_raw(uint32_t* out, int64_t n, uint64_t ctr0, uint64_t key, void* stream);

/* 3xf16 split operand of the noise GEMMs: value = (hi + lo) / *scale, with hi
 * and lo fp16 values, zero padded, and *scale a power of two chosen on the
 * device from max|x| (mpv_split_f16) or fixed (mpv_noise_philox_f16).
 * hi*hi + hi*lo + lo*hi on the f16 matrix cores with fp32 accumulation
 * reproduces an fp32 product to ~2^-22.
 *
 * Chunked layout: row r is ld halves; every 32-column chunk k of the row is
 * 32 hi halves followed by its 32 lo halves, so column c of row r has
 *   hi at data[r*ld + (c/32)*64 + c%32],  lo 32 halves further,
 * and one 128-B line carries both halves of a 32-element K slice (the GEMMs
 * stream whole lines).  Columns 0 .. ld/2-1 are addressable. */
typedef struct mpv_split16 {
  uint16_t* data;
  float* scale;      /* device scalar */
  int64_t rows_pad;  /* allocated rows */
  int64_t ld;        /* halves per row: 2 x padded columns, a multiple of 64 */
} mpv_split16;

enum mpv_gemm { MPV_GEMM_F16X3 = 0, MPV_GEMM_F32 = 1 };

size_t mpv_split_workspace_bytes(void);

/* Columns the 3xf16 noise planes of this shape need (z padded to the dR
 * GEMM's tile: 64 when L and z are both <= 64, 128 when both are <= 128,
 * else 256); the planes' ld is twice this. */
int64_t mpv_noise_plane_cols(const mpv_shape* shape);

/* x (rows, cols) fp32 / fp64 -> split planes.  Used for r_sqrt_sigma
 * (replacing R.T.float(), mpvae.py:165) and for explicit noise, which the
 * caller passes as its (B, S_local, z) transpose (plane row b*S_local + s). */
int mpv_split_f16(const void* x, int x_dtype, int64_t rows, int64_t cols, const mpv_split16* out,
                  void* workspace, void* stream);

/* mpv_noise_philox writing split planes directly: S_local*B rows, plane row
 * b*S_local + s = eps[s, b, :] (the s rows of one batch row contiguous, as the
 * GEMMs stream them); the same numbers as mpv_noise_philox.  Columns z ..
 * roundup(z, 32) - 1 are written as zeros; columns past that (the dR tile's
 * padding, mpv_noise_plane_cols) are not written. */
int mpv_noise_philox_f16(const mpv_shape* shape, uint64_t seed, uint64_t offset,
                         const mpv_split16* out, void* stream);

/* mpv_noise_philox_f16 with the key read from device memory (see
 * mpv_noise_philox_dev). */
int mpv_noise_philox_f16_dev(const mpv_shape* shape, const uint64_t* seed_dev, uint64_t offset,
                             const mpv_split16* out, void* stream);

/* mpv_noise_philox_f16 (seed_dev NULL: the key `seed`) or mpv_noise_philox_f16_dev
 * (the key read from seed_dev), and mpv_split_f16 of a small operand x (rows *
 * cols <= 16384: r_sqrt_sigma at L, z <= 128) into x_out, in ONE launch: the
 * split runs in extra workgroups beside the noise's.  The same outputs as the
 * two calls. */
int mpv_noise_philox_f16_split(const mpv_shape* shape, uint64_t seed, const uint64_t* seed_dev,
                               uint64_t offset, const mpv_split16* out, const void* x,
                               int x_dtype, int64_t rows, int64_t cols,
                               const mpv_split16* x_out, void* stream);

/* Element-wise dtype conversion; replaces r_sqrt_sigma.T.float() (mpvae.py:165)
 * and the fp32 -> fp64 cast of its gradient in autograd. */
int mpv_convert(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n,
                void* stream);

/* ---------------------------------------------------------------- forward */
typedef struct mpv_fwd_args {
  const float* y;
  const float* fe_out;
  const float* fx_out;
  int gemm;             /* mpv_gemm: which operand pair below is used */
  const float* R32;     /* MPV_GEMM_F32:   (L,z) fp32 */
  const float* eps;     /*                 (S_local,B,z) fp32 */
  mpv_split16 R16;      /* MPV_GEMM_F16X3: R planes, rows_pad >= roundup(L,256), ld >= 2*roundup(z,128) */
  mpv_split16 eps16;    /*                 noise planes, row b*S_local + s = eps[s, b, :], ld >= 2*mpv_noise_plane_cols() */
  float* T;             /* (B,S_local,roundup(L,4)): rows 16-B aligned, the pad columns
                           scratch; or NULL when no backward will follow */
  float* rowstat;       /* (6,B,S_local) out */
  float* bstat;         /* (6,B) out: this shard's statistics */
  float* colsum;        /* (2,B,L) out: this shard's sums over s */
  void* workspace;
  size_t workspace_bytes;
} mpv_fwd_args;

size_t mpv_fwd_workspace_bytes(const mpv_shape* shape);

/* Replaces mpvae.py:165-204 for one S-shard: the noise GEMM
 * sample_r(_x) = eps . R^T + fe_out / fx_out (computed once for both
 * branches), the probit decode E = Phi(u)(1-1e-6)+0.5e-6, the per-(s,b) BCE
 * log-probability (:184-185), the ranking-loss factors (:103-123, factorised
 * as P*N), the shard-local log-sum-exp statistics (:188-189) and the sums
 * over s behind indiv_prob / indiv_prob_label (:203-204). */
int mpv_probit_fwd(const mpv_shape* shape, const mpv_fwd_args* args, void* stream);

/* Exact combine of per-shard bstat gathered as (nshards,6,B) -> (6,B):
 * M = max m_r, Z = sum Z_r exp(m_r - M), ranking sums add. */
int mpv_bstat_combine(const float* gathered, int64_t nshards, int64_t B, float* out,
                      void* stream);

typedef struct mpv_final_args {
  const float* bstat;   /* (6,B) global */
  const float* colsum;  /* (2,B,L) global */
  const float* fe_mu;   /* (B,d) */
  const float* fe_logvar;
  const float* fx_mu;
  const float* fx_logvar;
  int64_t d;
  float nll_coeff, c_coeff;
  float* total;  /* 0-d outputs, mpvae.py:210 order */
  float* nll;
  float* nll_x;
  float* c;
  float* c_x;
  float* kl;
  float* indiv_prob;        /* (B,L) = mean_s E_x  (mpvae.py:203) */
  float* indiv_prob_label;  /* (B,L) = mean_s E    (mpvae.py:204) */
  uint64_t* seed_advance;   /* a device Philox key this step's noise has read, advanced by 1
                               in the finalize launch (the next step draws fresh noise
                               with no launch of its own), or NULL */
} mpv_final_args;

/* Replaces mpvae.py:147-148 (KL), :188-190 (log-sum-exp nll), :122 (ranking
 * mean), :203-210 (indiv_prob*, total).  `shape` gives B, L, S_total. */
int mpv_probit_finalize(const mpv_shape* shape, const mpv_final_args* args, void* stream);

/* mpv_bstat_combine + mpv_probit_finalize in one launch (the sample-sharded
 * path): `slots` holds the shards' bstat as (nslots, 6, B) (the all-reduced
 * slot buffer), combined exactly into `bstat_out` (6, B) for the backward;
 * `args->bstat` is ignored, `args->colsum` is the all-reduced (2, B, L). */
int mpv_probit_finalize_shards(const mpv_shape* shape, const float* slots, int64_t nslots,
                               float* bstat_out, const mpv_final_args* args, void* stream);

/* --------------------------------------------------------------- backward */
struct mpv_kl_bwd_args;  /* below */

typedef struct mpv_bwd_args {
  const float* y;
  const float* fe_out;
  const float* fx_out;
  int gemm;                    /* mpv_gemm, as in the forward */
  const float* eps;            /* MPV_GEMM_F32: (S_local,B,z), the forward's noise */
  mpv_split16 eps16;           /* MPV_GEMM_F16X3: the forward's noise planes */
  float* T;                    /* in: forward's T; MPV_GEMM_F32 overwrites it with
                                  d(sample_r)+d(sample_r_x) (F16X3 writes planes in
                                  the workspace instead) */
  const float* rowstat;        /* (6,B,S_local) from the forward */
  const float* bstat;          /* (6,B) GLOBAL statistics */
  const float* gscal;          /* device: upstream grads, mpv_gslot order; a slot whose
                                  MPV_LIVE bit is clear is not read (its gradient is 0),
                                  so (6) floats, or just (1) when only MPV_G_TOTAL is live */
  const float* g_indiv;        /* (B,L) grad of indiv_prob, or NULL */
  const float* g_indiv_label;  /* (B,L) grad of indiv_prob_label, or NULL */
  float nll_coeff, c_coeff;
  int live;                    /* MPV_LIVE bits of gscal */
  float* dfe_dfx;              /* (2,B,L) out: d fe_out, d fx_out (this shard) */
  float* dR32;                 /* (L,z) out fp32 d r_sqrt_sigma (this shard), or NULL */
  void* workspace;
  size_t workspace_bytes;
  double* dR64;                /* (L,z) out fp64 d r_sqrt_sigma instead of dR32, for an fp64
                                  r_sqrt_sigma with no cross-shard sum to follow; or NULL */
  const struct mpv_kl_bwd_args* kl; /* run the KL backward (mpv_kl_bwd) in this call, or NULL */
} mpv_bwd_args;

size_t mpv_bwd_workspace_bytes(const mpv_shape* shape, int gemm);

/* Replaces PyTorch autograd through mpvae.py:165-210 (including the pairwise
 * (S,B,L,L) ranking tensor): d fe_out, d fx_out and d r_sqrt_sigma. */
int mpv_probit_bwd(const mpv_shape* shape, const mpv_bwd_args* args, void* stream);

typedef struct mpv_kl_bwd_args {
  const float* fe_mu;
  const float* fe_logvar;
  const float* fx_mu;
  const float* fx_logvar;
  int64_t B, d;
  const float* gscal;  /* device, mpv_gslot order; uses TOTAL and KL where live */
  float* g_fe_mu;
  float* g_fe_logvar;
  float* g_fx_mu;
  float* g_fx_logvar;
  int live;            /* MPV_LIVE bits of gscal (slots not live are not read) */
} mpv_kl_bwd_args;

/* Replaces autograd through the KL term, mpvae.py:147-148. */
int mpv_kl_bwd(const mpv_kl_bwd_args* args, void* stream);

/* ------------------------------------------------- reparameterisation a3 */
typedef struct mpv_reparam_args {
  const float* mu_e;
  const float* logvar_e;
  const float* eps_e;
  float* z_e;
  int64_t n_e;  /* elements of the label encoder (0 = skip) */
  const float* mu_x;
  const float* logvar_x;
  const float* eps_x;
  float* z_x;
  int64_t n_x;  /* elements of the feature encoder (0 = skip) */
  /* ABI v9, each may be NULL: copies of mu / logvar written in the same pass,
   * so the VAE hands its callers fresh tensors (not aliases of the encoder
   * heads' outputs) at no extra launch */
  float* mu_e_out;
  float* logvar_e_out;
  float* mu_x_out;
  float* logvar_x_out;
} mpv_reparam_args;

/* Replaces label_reparameterize / feat_reparameterize (mpvae.py:66-74):
 * z = mu + eps * exp(0.5 logvar) for BOTH encoders in one launch. */
int mpv_reparam_fwd(const mpv_reparam_args* args, void* stream);

typedef struct mpv_reparam_bwd_args {
  const float* gz_e;  /* NULL = no gradient reached z_e */
  const float* logvar_e;
  const float* eps_e;
  float* gmu_e;
  float* glogvar_e;
  int64_t n_e;
  const float* gz_x;
  const float* logvar_x;
  const float* eps_x;
  float* gmu_x;
  float* glogvar_x;
  int64_t n_x;
  /* ABI v8: gradients of mu / logvar from their other consumers (the KL in
   * compute_loss), added to the outputs (NULL = none) */
  const float* gmu_add_e;
  const float* glogvar_add_e;
  const float* gmu_add_x;
  const float* glogvar_add_x;
} mpv_reparam_bwd_args;

int mpv_reparam_bwd(const mpv_reparam_bwd_args* args, void* stream);

/* ------------------------------------------------- encoder/decoder MLPs a2/a4
 * One fp32 matrix-core GEMM with a fused epilogue (linear.hip):
 *   out[i * out_si + j] = act(alpha * (sum_r A(i, r) B(j, r) + bias[j]))
 *   A(i, r) = a[i * a_si + r * a_sr] * a_scale, zeroed where a_mask (same
 *             strides, optional) is not > 0 (the ReLU backward);
 *   B(j, r) = b[j * b_sj + r * b_sr], or 1 for j == ones_col, whose output
 *             goes to out_col[i] instead (the bias gradient; ones_col must be
 *             N - 1, or -1 for none).
 * act = ReLU when relu != 0 (NaN passes, as torch.relu).  Replaces nn.Linear
 * (+ F.relu, + the `* scale_coeff` of mpvae.py:54-55,63-64) in the forward
 * and the three GEMMs of its backward (mpvae.py:11-38 layers, :51-84 uses).
 * The reduction is split over workgroups when the output is small; the
 * chunk partials (workspace, mpv_linear_workspace_bytes) are summed in a
 * fixed order, so results are deterministic. */
typedef struct mpv_linear_args {
  int64_t M, N, R;
  const float* a;
  int64_t a_si, a_sr;
  const float* a_mask;
  float a_scale;
  const float* b;
  int64_t b_sj, b_sr;
  int64_t ones_col;
  const float* bias; /* (N) or NULL */
  float alpha;
  int relu;
  float* out;
  int64_t out_si;
  float* out_col;    /* (M), with ones_col */
  /* ABI v8: optional second reduction segment -- for r >= R1 the sum reads
   * A = a2 (row stride a2_si, reduction stride a_sr) and B = b2 (B's
   * strides) at index r - R1; a2 = b2 = NULL: one segment.  No a_mask. */
  const float* a2;
  int64_t a2_si;
  const float* b2;
  int64_t R1;
} mpv_linear_args;

size_t mpv_linear_workspace_bytes(int64_t M, int64_t N, int64_t R);
int mpv_linear(const mpv_linear_args* args, void* workspace, size_t workspace_bytes, void* stream);

/* n (1..4) independent mpv_linear problems in one launch pair (a layer's dx
 * and dW + db; two heads and their gradients); the workspace is the sum of
 * the problems' own, in order. */
size_t mpv_linear_batch_workspace_bytes(const mpv_linear_args* args, int n);
int mpv_linear_batch(const mpv_linear_args* args, int n, void* workspace, size_t workspace_bytes,
                     void* stream);

/* ------------------------------------------------------ Adam (TrainStep) */
/* One Adam update over up to MPV_ADAM_MAX_TENSORS parameter tensors, fp32 and
 * fp64 mixed, in one launch; replaces optimizer.step() of
 * torch.optim.Adam(params, lr, betas, eps, weight_decay) (fairsoft_train.py:57,
 * :146; fairsoft_jaccard.py:64-65) inside mpvae_step.TrainStep, with torch's
 * fused-Adam arithmetic (L2 weight decay, no amsgrad / maximize).  `step` is
 * the tensor's device step count BEFORE this update: the bias corrections use
 * step + 1 (the float add torch's capturable protocol performs), and the count
 * itself is advanced afterwards by mpv_adam_finish.  found_inf (may be NULL):
 * when *found_inf == 1 nothing is written.  lr_dev (may be NULL): the learning
 * rate is read from device memory (a StepLR that mpv_adam_finish decays)
 * instead of `lr`. */
#define MPV_ADAM_MAX_TENSORS 32
typedef struct mpv_adam_tensor {
  void* param;
  const void* grad;
  void* exp_avg;
  void* exp_avg_sq;
  const float* step;
  int64_t numel;
  int is_f64;  /* 0: float32 tensors, 1: float64 */
} mpv_adam_tensor;

typedef struct mpv_adam_args {
  int n;
  mpv_adam_tensor t[MPV_ADAM_MAX_TENSORS];
  double lr, beta1, beta2, weight_decay, eps;
  const float* found_inf;
  const double* lr_dev;  /* NULL, or this group's device learning rate */
} mpv_adam_args;

int mpv_adam_step(const mpv_adam_args* args, void* stream);

/* After the mpv_adam_step launches of one optimizer step (one launch, one
 * workgroup): every step count += 1 - found_inf (torch's +1 then -found_inf);
 * the applied-update counter += 1 - found_inf (the reference's
 * succses_updates, fairsoft_train.py:146); and, when n_lr > 0, the
 * scheduler step the reference takes after an applied update only
 * (fairsoft_train.py:142-145) for torch.optim.lr_scheduler.StepLR
 * (fairsoft_jaccard.py:67-68): last_epoch += 1, and if last_epoch is a
 * non-zero multiple of step_size (fmod, as Python's % for a float step_size)
 * every lr[g] *= gamma in double -- the chainable form torch's StepLR.get_lr
 * uses, so the device lr equals torch's bit for bit. */
#define MPV_ADAM_FINISH_MAX 256
typedef struct mpv_adam_finish_args {
  int n_steps;
  float* steps[MPV_ADAM_FINISH_MAX];
  const float* found_inf; /* NULL: the update was applied */
  int64_t* updates;       /* NULL, or the applied-update counter */
  int n_lr;               /* 0: no scheduler */
  double* lr;             /* n_lr device learning rates (one per param group) */
  int64_t* last_epoch;    /* the scheduler's device last_epoch */
  double step_size, gamma;
} mpv_adam_finish_args;

int mpv_adam_finish(const mpv_adam_finish_args* args, void* stream);

/* ------------------------------------------------------------ measurement */
/* When enabled, every kernel launch of the library is bracketed by a pair of
 * HIP events on the launch stream (bench.py's per-kernel roofline timing).
 * Kernel names: noise_philox, probit_fwd, fwd_combine, finalize, bwd_coef,
 * bwd_elem, dR_gemm, sum_slabs, convert, bstat_combine, reparam_fwd,
 * reparam_bwd, kl_bwd, linear, adam, adam_finish.  Query synchronises the recorded events. */
int mpv_timing_enable(int on);
int mpv_timing_reset(void);
int mpv_timing_query(const char* kernel, int64_t* launches, double* total_ms);

/* ---- Consumers of indiv_prob / indiv_prob_label in the training step ------
 * (fairness.hip) */

/* Open-addressing table of 0/1 label patterns -> distance, one per target
 * fair label: replaces label_distances[target].get(''.join(label.astype(str)),
 * 0.) per batch row (fairsoft_train.py:85-93).  Key = the pattern packed
 * 64 labels per word (bit j of word w = label 64w+j), W = ceil(L/64) words;
 * slot = splitmix64-chain hash & (nslots-1), linear probing, used[slot] = 0
 * ends a probe.  Built once on the host (mpvae_fair.LabelDistanceTable). */
typedef struct mpv_label_table {
  const uint64_t* keys; /* nslots * W */
  const double* vals;   /* nslots */
  const int32_t* used;  /* nslots */
  int64_t nslots;       /* a power of two (0: empty table) */
  int64_t W;
} mpv_label_table;

/* w[b] = table value of row b's pattern (0 when absent or not 0/1 after
 * int()); *contributed += #rows with w > 0 (fairsoft_train.py:91-92). */
int mpv_label_weights(const float* y, int64_t B, int64_t L, const mpv_label_table* table,
                      double* w, int32_t* contributed, void* stream);

enum mpv_fair_norm { MPV_FAIR_L1 = 1, MPV_FAIR_L2 = 2 };

/* Fairness regulariser (fairsoft_train.py:95-131), fp64 as in the reference:
 *   W_t = sum_b w[t,b];  m_t = sum_b w[t,b] z[b] / W_t           (if W_t > 0)
 *   per sensitive group k: W_tk, m_tk likewise                      (if W_tk > 0)
 *   out = fair_coeff * sum_{z in label_z, feat_z} sum_t sum_k sum_l f(m_tk - m_t)
 * with f = |.| (l1) or (.)^2 (l2).  Rows are grouped by `gid` (B), `order`
 * (B) lists them group by group, `goff` (G+1) holds the group offsets.  The
 * workspace keeps the backward's tables: pass the same one to mpv_fair_bwd. */
typedef struct mpv_fair_args {
  const float* label_z;  /* (B, L) indiv_prob_label */
  const float* feat_z;   /* (B, L) indiv_prob */
  const double* w;       /* (T, B) */
  const int32_t* order;  /* (B) */
  const int32_t* goff;   /* (G + 1) */
  const int32_t* gid;    /* (B) */
  int64_t B, L, T, G;
  int norm;              /* MPV_FAIR_L1 / MPV_FAIR_L2 (else the penalty is 0) */
  double fair_coeff;
  double* out;           /* device scalar */
} mpv_fair_args;

size_t mpv_fair_workspace_bytes(int64_t L, int64_t T, int64_t G);
int mpv_fair_fwd(const mpv_fair_args* args, void* workspace, size_t workspace_bytes,
                 void* stream);
/* g_label_z, g_feat_z (B, L) = *gout x d out / d label_z, feat_z (sgn(0) = 0). */
int mpv_fair_bwd(const mpv_fair_args* args, const double* gout, float* g_label_z,
                 float* g_feat_z, void* workspace, size_t workspace_bytes, void* stream);

/* evals.compute_metrics(pred, target, threshold, all_metrics=False)
 * (evals.py:178-238) on the device: out[8] = [ACC, HA, ebF1, miF1, maF1,
 * p@1, p@3, p@5].  Top-k ties go to the larger label index. */
size_t mpv_metrics_workspace_bytes(int64_t B, int64_t L);
int mpv_train_metrics(const float* pred, const float* target, int64_t B, int64_t L,
                      float threshold, double* out, void* workspace, size_t workspace_bytes,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPVAE_HIP_H */
