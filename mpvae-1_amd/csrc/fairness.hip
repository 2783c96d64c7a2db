// The two per-step consumers of compute_loss's indiv_prob outputs in the
// reference training loop, on the device:
//
//   label_weights_kernel   per-row weight = label_distances[target].get(
//                          ''.join(label.astype(str)), 0.)  (fairsoft_train.py:
//                          85-93): the row's 0/1 label pattern is packed by
//                          wave ballots and looked up in an open-addressing
//                          table of packed patterns (built once on the host
//                          from the same dict), instead of a Python string join
//                          and dict lookup per row.
//   fair_fwd_kernel        the fairness regulariser (fairsoft_train.py:95-131):
//                          weighted means of indiv_prob_label / indiv_prob over
//                          the batch and over each sensitive group, l1 or l2
//                          distance, summed over target labels and groups.  fp64
//                          throughout.  The reference computes in fp64 when its
//                          distances are numpy float64 (torch.tensor(weights)
//                          is float64 and the products promote) and in fp32
//                          when they are Python floats; the host returns the
//                          loss in that dtype (mpvae_fair.py).  Also stashes
//                          f'(d) / W_tk and sum_k f'(d) / W_t for the backward.
//   fair_bwd_kernel        d penalty / d indiv_prob[_label] (autograd through
//                          the same lines; |x|' = sgn(x), sgn(0) = 0).
//   metric_rows_kernel,    evals.compute_metrics(..., all_metrics=False)
//   metric_cols_kernel,    (evals.py:178-238): ACC, HA, ebF1, miF1, maF1 and
//   metric_final_kernel    p@1/3/5 without copying the batch to the host.
//
// All reductions run in a fixed order: results are deterministic.
#include "abi_util.h"
#include "mpv_common.h"

namespace mpv {

// ------------------------------------------------------------ label weights
// splitmix64 finaliser; the host builder (mpvae_fair.py) uses the same mix
MPV_DEV uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// One wave per batch row.  Bit j of word w is label 64w + j (character
// 64w + j of the reference's key string).  A row with a label value whose
// int() is neither 0 nor 1 has no binary key: weight 0, as a dict miss.
constexpr int kLwWaves = 4;
__global__ __launch_bounds__(64 * kLwWaves) void label_weights_kernel(
    const float* __restrict__ y, int B, int L, mpv_label_table tab, double* __restrict__ w,
    int* __restrict__ contributed) {
  __shared__ uint64_t words[kLwWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x * kLwWaves + wv;
  if (b >= B) return;
  const int W = (int)tab.W;
  bool bad = false;
  uint64_t h = 0x6A09E667F3BCC909ull ^ (uint64_t)W;
  for (int k = 0; k < W; ++k) {
    const int l = k * 64 + lane;
    const float v = l < L ? truncf(y[(int64_t)b * L + l]) : 0.0f;
    bad |= !(v == 0.0f || v == 1.0f);
    const uint64_t bits = __ballot(v == 1.0f);
    if (lane == 0) words[wv][k] = bits;
    h = mix64(h ^ bits);
  }
  bad = __any(bad);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double val = 0.0;
  if (!bad && tab.nslots > 0) {
    const uint64_t mask = (uint64_t)tab.nslots - 1;
    for (uint64_t probe = 0; probe < (uint64_t)tab.nslots; ++probe) {
      const uint64_t slot = (h + probe) & mask;
      if (!tab.used[slot]) break;  // empty slot: not in the table
      bool diff = false;
      for (int k = lane; k < W; k += 64) diff |= tab.keys[slot * W + k] != words[wv][k];
      if (!__any(diff)) {
        val = tab.vals[slot];
        break;
      }
    }
  }
  if (lane == 0) {
    w[b] = val;
    if (val > 0.0) atomicAdd(contributed, 1);  // integer count: order-free
  }
}

// -------------------------------------------------------- fairness penalty
constexpr int kFairThreads = 256;

// Weight sums W_t (index t*(G+1) + G) and W_tk (t*(G+1) + k), one thread per
// (t, k) pair, each a fixed-order loop: deterministic.
__global__ void fair_wsum_kernel(const double* __restrict__ w, const int* __restrict__ order,
                                 const int* __restrict__ goff, int B, int T, int G,
                                 double* __restrict__ wsum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T * (G + 1)) return;
  const int t = i / (G + 1), k = i % (G + 1);
  double s = 0.0;
  if (k == G) {
    for (int b = 0; b < B; ++b) s += w[(int64_t)t * B + b];
  } else {
    for (int j = goff[k]; j < goff[k + 1]; ++j) s += w[(int64_t)t * B + order[j]];
  }
  wsum[i] = s;
}

// One thread per (label l, branch br): br 0 = indiv_prob_label (label_z),
// br 1 = indiv_prob (feat_z).
__global__ __launch_bounds__(kFairThreads) void fair_fwd_kernel(mpv_fair_args a,
                                                                const double* __restrict__ wsum,
                                                                double* __restrict__ dtab,
                                                                double* __restrict__ etab,
                                                                double* __restrict__ part) {
  __shared__ double red[kFairThreads / 64];
  const int L = (int)a.L, B = (int)a.B, T = (int)a.T, G = (int)a.G;
  const int br = blockIdx.y;
  const int l = blockIdx.x * kFairThreads + threadIdx.x;
  const float* z = br == 0 ? a.label_z : a.feat_z;
  double pen = 0.0;
  if (l < L) {
    for (int t = 0; t < T; ++t) {
      const double* wt = a.w + (int64_t)t * B;
      const double Wt = wsum[t * (G + 1) + G];
      double esum = 0.0;
      if (Wt > 0.0) {  // fairsoft_train.py:97 `if weights.sum() > 0`
        double tot = 0.0;
        for (int b = 0; b < B; ++b) tot += (double)z[(int64_t)b * L + l] * wt[b];
        const double mt = tot / Wt;
        for (int k = 0; k < G; ++k) {
          const double Wk = wsum[t * (G + 1) + k];
          double fp = 0.0;
          if (Wk > 0.0) {  // :110 `if weight_sensitive.sum() > 0`
            double s = 0.0;
            for (int j = a.goff[k]; j < a.goff[k + 1]; ++j) {
              const int b = a.order[j];
              s += (double)z[(int64_t)b * L + l] * wt[b];
            }
            const double d = s / Wk - mt;
            if (a.norm == MPV_FAIR_L1) {
              pen += fabs(d);
              fp = d > 0.0 ? 1.0 : (d < 0.0 ? -1.0 : 0.0);
            } else if (a.norm == MPV_FAIR_L2) {
              pen += d * d;
              fp = 2.0 * d;
            }
            esum += fp;
            fp /= Wk;
          }
          dtab[(((int64_t)br * T + t) * G + k) * L + l] = fp;
        }
        esum /= Wt;
      } else {
        for (int k = 0; k < G; ++k) dtab[(((int64_t)br * T + t) * G + k) * L + l] = 0.0;
      }
      etab[((int64_t)br * T + t) * L + l] = esum;
    }
  }
  // block sum of pen (fixed shuffle tree, then the 4 waves in order)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) pen += __shfl_xor(pen, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pen;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < kFairThreads / 64; ++i) s += red[i];
    part[blockIdx.y * gridDim.x + blockIdx.x] = s;
  }
}

__global__ void fair_final_kernel(const double* __restrict__ part, int n, double coeff,
                                  double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += part[i];
  *out = coeff * s;
}

// grad[b, l] = gout * coeff * sum_t w[t,b] (dtab[t, gid[b], l] - etab[t, l])
__global__ __launch_bounds__(kFairThreads) void fair_bwd_kernel(mpv_fair_args a,
                                                                const double* __restrict__ dtab,
                                                                const double* __restrict__ etab,
                                                                const double* __restrict__ gout,
                                                                float* __restrict__ g_label_z,
                                                                float* __restrict__ g_feat_z) {
  const int L = (int)a.L, B = (int)a.B, T = (int)a.T, G = (int)a.G;
  const int64_t i = (int64_t)blockIdx.x * kFairThreads + threadIdx.x;
  const int br = blockIdx.y;
  if (i >= (int64_t)B * L) return;
  const int b = (int)(i / L), l = (int)(i % L), k = a.gid[b];
  double g = 0.0;
  for (int t = 0; t < T; ++t) {
    const double wb = a.w[(int64_t)t * B + b];
    g += wb * (dtab[(((int64_t)br * T + t) * G + k) * L + l] - etab[((int64_t)br * T + t) * L + l]);
  }
  g *= *gout * a.fair_coeff;
  (br == 0 ? g_label_z : g_feat_z)[i] = (float)g;
}

// ------------------------------------------------------------ train metrics
constexpr int kMetThreads = 256;

struct ArgMax {
  float v;
  int i;
};
// larger value wins; on a tie the larger index (= numpy argsort(...)[::-1]
// with a stable sort; numpy's default sort is not stable)
MPV_DEV ArgMax better(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i > a.i)) ? b : a;
}

// One block per batch row: subset accuracy, hamming, example-F1 terms and the
// top-5 hits (evals.py:13-45, 48-83).  rowstat[b] = [eq_all, xor_count,
// tp, sum_true, sum_pred, hit@1, hit@3, hit@5].
__global__ __launch_bounds__(kMetThreads) void metric_rows_kernel(const float* __restrict__ pred,
                                                                  const float* __restrict__ tgt,
                                                                  int B, int L, float thr,
                                                                  double* __restrict__ rowstat) {
  __shared__ float sred[5][kMetThreads / 64];
  __shared__ ArgMax am[kMetThreads / 64];
  __shared__ int chosen[5];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* pr = pred + (int64_t)b * L;
  const float* tr = tgt + (int64_t)b * L;
  float neq = 0.f, nxor = 0.f, tp = 0.f, st = 0.f, sp = 0.f;
  for (int l = tid; l < L; l += kMetThreads) {
    const float p = pr[l] < thr ? 0.0f : 1.0f;  // evals.py:201-202
    const float t = tr[l];
    neq += (t == p) ? 0.f : 1.f;
    nxor += ((t != 0.f) != (p != 0.f)) ? 1.f : 0.f;
    tp += t * p;
    st += t;
    sp += p;
  }
  float v[5] = {neq, nxor, tp, st, sp};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    if (lane == 0) sred[k][wv] = v[k];
  }
  // top-5 by the raw probabilities, one block argmax per rank
  int hits[5];
  for (int r = 0; r < 5; ++r) {
    ArgMax m{-INFINITY, -1};
    for (int l = tid; l < L; l += kMetThreads) {
      bool used = false;
      for (int q = 0; q < r; ++q) used |= chosen[q] == l;
      if (!used) m = better(m, ArgMax{pr[l], l});
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      ArgMax x{__shfl_xor(m.v, o, 64), __shfl_xor(m.i, o, 64)};
      m = better(m, x);
    }
    if (lane == 0) am[wv] = m;
    __syncthreads();
    if (tid == 0) {
      ArgMax best = am[0];
      for (int i = 1; i < kMetThreads / 64; ++i) best = better(best, am[i]);
      chosen[r] = best.i;
    }
    __syncthreads();
    hits[r] = (chosen[r] >= 0 && tr[chosen[r]] == 1.0f) ? 1 : 0;
  }
  if (tid == 0) {
    float s[5];
    for (int k = 0; k < 5; ++k) {
      s[k] = 0.f;
      for (int i = 0; i < kMetThreads / 64; ++i) s[k] += sred[k][i];
    }
    double* o = rowstat + (int64_t)b * 8;
    o[0] = s[0] == 0.f ? 1.0 : 0.0;  // all labels equal
    o[1] = s[1];
    o[2] = s[2];
    o[3] = s[3];
    o[4] = s[4];
    o[5] = hits[0];
    o[6] = hits[0] + hits[1] + hits[2];
    o[7] = hits[0] + hits[1] + hits[2] + hits[3] + hits[4];
  }
}

// One thread per label: tp, fp, fn over the batch (compute_tp_fp_fn axis=0).
__global__ void metric_cols_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                   int B, int L, float thr, float* __restrict__ colstat) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= L) return;
  float tp = 0.f, fp = 0.f, fn = 0.f;
  for (int b = 0; b < B; ++b) {
    const float p = pred[(int64_t)b * L + l] < thr ? 0.0f : 1.0f;
    const float t = tgt[(int64_t)b * L + l];
    tp += t * p;
    fp += (t == 0.f ? 1.f : 0.f) * p;
    fn += t * (p == 0.f ? 1.f : 0.f);
  }
  colstat[l] = tp;
  colstat[L + l] = fp;
  colstat[2 * L + l] = fn;
}

// out = [ACC, HA, ebF1, miF1, maF1, p@1, p@3, p@5] (evals.py:205-237)
__global__ void metric_final_kernel(const double* __restrict__ rowstat,
                                    const float* __restrict__ colstat, int B, int L,
                                    double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double acc = 0, hl = 0, ef = 0, p1 = 0, p3 = 0, p5 = 0;
  int nef = 0;
  for (int b = 0; b < B; ++b) {
    const double* r = rowstat + (int64_t)b * 8;
    acc += r[0];
    hl += r[1] / L;
    const float den = (float)r[3] + (float)r[4];
    if (den != 0.0f) {
      ef += (double)((2.0f * (float)r[2]) / den);
      ++nef;
    }
    p1 += r[5] / 1.0;
    p3 += r[6] / 3.0;
    p5 += r[7] / 5.0;
  }
  double tp = 0, fp = 0, fn = 0, ma = 0;
  int nma = 0;
  for (int l = 0; l < L; ++l) {
    const float a = colstat[l], c = colstat[L + l], d = colstat[2 * L + l];
    tp += a;
    fp += c;
    fn += d;
    const double f = (double)(2.0f * a) / (double)(2.0f * a + c + d + 1e-6f);
    if (isfinite(f)) {
      ma += f;
      ++nma;
    }
  }
  out[0] = acc / B;
  out[1] = 1.0 - hl / B;
  out[2] = nef ? ef / nef : NAN;
  out[3] = (2.0 * tp) / (2.0 * tp + fp + fn);
  out[4] = nma ? ma / nma : NAN;
  out[5] = p1 / B;
  out[6] = p3 / B;
  out[7] = p5 / B;
}

}  // namespace mpv

using namespace mpv;

extern "C" {

int mpv_label_weights(const float* y, int64_t B, int64_t L, const mpv_label_table* tab,
                      double* w, int32_t* contributed, void* stream) {
  MPV_REQUIRE(y && tab && w && contributed && B > 0 && L > 0, "bad label_weights arguments");
  MPV_REQUIRE(tab->W == (L + 63) / 64, "table words %lld != ceil(L/64) = %lld",
              (long long)tab->W, (long long)((L + 63) / 64));
  MPV_REQUIRE(tab->nslots == 0 || (tab->keys && tab->vals && tab->used &&
                                   (tab->nslots & (tab->nslots - 1)) == 0),
              "table slots must be a power of two with keys/vals/used");
  MPV_REQUIRE(tab->W <= 64, "label_dim > 4096 is not supported by the pattern table");
  const int blocks = (int)cdiv(B, kLwWaves);
  MPV_LAUNCH("label_weights", label_weights_kernel, dim3(blocks), dim3(64 * kLwWaves), 0,
             as_stream(stream), y, (int)B, (int)L, *tab, w, contributed);
  return check_launch("label_weights");
}

size_t mpv_fair_workspace_bytes(int64_t L, int64_t T, int64_t G) {
  if (L <= 0 || T <= 0 || G <= 0) return 0;
  const int64_t nlb = cdiv(L, kFairThreads);
  return sizeof(double) * (size_t)(2 * T * G * L + 2 * T * L + T * (G + 1) + 2 * nlb);
}

static void fair_ws(const mpv_fair_args* a, void* ws, double*& dtab, double*& etab, double*& wsum,
                    double*& part) {
  dtab = reinterpret_cast<double*>(ws);
  etab = dtab + 2 * a->T * a->G * a->L;
  wsum = etab + 2 * a->T * a->L;
  part = wsum + a->T * (a->G + 1);
}

int mpv_fair_fwd(const mpv_fair_args* a, void* workspace, size_t workspace_bytes, void* stream) {
  MPV_REQUIRE(a && a->label_z && a->feat_z && a->w && a->order && a->goff && a->gid && a->out,
              "NULL pointer in mpv_fair_args");
  MPV_REQUIRE(a->B > 0 && a->L > 0 && a->T > 0 && a->G > 0, "bad fairness shape");
  MPV_REQUIRE(workspace && workspace_bytes >= mpv_fair_workspace_bytes(a->L, a->T, a->G),
              "fairness workspace too small");
  hipStream_t st = as_stream(stream);
  double *dtab, *etab, *wsum, *part;
  fair_ws(a, workspace, dtab, etab, wsum, part);
  const int npair = (int)(a->T * (a->G + 1));
  MPV_LAUNCH("fair_fwd", fair_wsum_kernel, dim3((unsigned)cdiv(npair, 64)), dim3(64), 0, st, a->w,
             a->order, a->goff, (int)a->B, (int)a->T, (int)a->G, wsum);
  if (int rc = check_launch("fair_wsum")) return rc;
  const int nlb = (int)cdiv(a->L, kFairThreads);
  MPV_LAUNCH("fair_fwd", fair_fwd_kernel, dim3(nlb, 2), dim3(kFairThreads), 0, st, *a, wsum, dtab,
             etab, part);
  if (int rc = check_launch("fair_fwd")) return rc;
  MPV_LAUNCH("fair_fwd", fair_final_kernel, dim3(1), dim3(64), 0, st, part, 2 * nlb, a->fair_coeff,
             a->out);
  return check_launch("fair_final");
}

int mpv_fair_bwd(const mpv_fair_args* a, const double* gout, float* g_label_z, float* g_feat_z,
                 void* workspace, size_t workspace_bytes, void* stream) {
  MPV_REQUIRE(a && gout && g_label_z && g_feat_z && a->w && a->gid, "NULL pointer in fair_bwd");
  MPV_REQUIRE(workspace && workspace_bytes >= mpv_fair_workspace_bytes(a->L, a->T, a->G),
              "fairness workspace too small");
  double *dtab, *etab, *wsum, *part;
  fair_ws(a, workspace, dtab, etab, wsum, part);
  const int64_t n = a->B * a->L;
  MPV_LAUNCH("fair_bwd", fair_bwd_kernel, dim3((unsigned)cdiv(n, kFairThreads), 2),
             dim3(kFairThreads), 0, as_stream(stream), *a, dtab, etab, gout, g_label_z, g_feat_z);
  return check_launch("fair_bwd");
}

size_t mpv_metrics_workspace_bytes(int64_t B, int64_t L) {
  if (B <= 0 || L <= 0) return 0;
  return align_up(sizeof(double) * 8 * (size_t)B, 256) + sizeof(float) * 3 * (size_t)L;
}

int mpv_train_metrics(const float* pred, const float* target, int64_t B, int64_t L,
                      float threshold, double* out, void* workspace, size_t workspace_bytes,
                      void* stream) {
  MPV_REQUIRE(pred && target && out && B > 0 && L > 0, "bad train_metrics arguments");
  MPV_REQUIRE(workspace && workspace_bytes >= mpv_metrics_workspace_bytes(B, L),
              "metrics workspace too small");
  hipStream_t st = as_stream(stream);
  double* rowstat = reinterpret_cast<double*>(workspace);
  float* colstat = reinterpret_cast<float*>((char*)workspace + align_up(sizeof(double) * 8 * B, 256));
  MPV_LAUNCH("metrics", metric_rows_kernel, dim3((unsigned)B), dim3(kMetThreads), 0, st, pred,
             target, (int)B, (int)L, threshold, rowstat);
  if (int rc = check_launch("metric_rows")) return rc;
  MPV_LAUNCH("metrics", metric_cols_kernel, dim3((unsigned)cdiv(L, 256)), dim3(256), 0, st, pred,
             target, (int)B, (int)L, threshold, colstat);
  if (int rc = check_launch("metric_cols")) return rc;
  MPV_LAUNCH("metrics", metric_final_kernel, dim3(1), dim3(64), 0, st, rowstat, colstat, (int)B,
             (int)L, out);
  return check_launch("metric_final");
}

}  // extern "C"
