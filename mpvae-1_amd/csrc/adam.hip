// The Adam update of the drop-in training step (fairsoft_train.py:57,146:
// torch.optim.Adam(model.parameters(), lr, weight_decay) then
// optimizer.step()), for mpvae_step.TrainStep.
//
// torch's fused Adam (capturable) walks the parameter list in chunks of 65536
// elements per workgroup: the VAE's ~1.5 M parameters are ~25 workgroups, so
// the update runs on a tenth of the chip at one CU's bandwidth (42 us at C2 for
// 42 MB of traffic).  Here every parameter tensor of one launch is cut into
// 2048-element blocks (~750 workgroups at the VAE's sizes), fp32 and fp64
// tensors in the same launch.  Per element the arithmetic is torch's own
// (at::native adam_math, ADAM_MODE::ORIGINAL, no amsgrad / maximize / grad
// scale): the same mixed double / opmath expressions in the same order, the
// bias corrections from the device step count + 1 (torch's capturable
// protocol adds the 1 in a launch of its own first), and the whole update
// skipped when *found_inf == 1.  FP contraction is the compiler's default for
// device code (fast), as in torch's ROCm build of the same expressions: the
// parameters and moments equal torch's fused Adam bit for bit
// (tests/test_gpu_vae.py asserts torch.equal).
//
// adam_finish then advances the step counts, the applied-update counter and
// the reference's StepLR (fairsoft_jaccard.py:67-68, stepped after an applied
// update only, fairsoft_train.py:142-145) in one single-workgroup launch: the
// update kernel reads the counts and the lr, so they cannot change inside it.
#include <cmath>

#include "abi_util.h"
#include "mpv_common.h"

namespace mpv {
namespace {

constexpr int kAdamThreads = 256;
constexpr int kAdamPer = 8;  // elements per thread per block
constexpr int kAdamBlock = kAdamThreads * kAdamPer;

struct AdamBatch {
  mpv_adam_tensor t[MPV_ADAM_MAX_TENSORS];
  int64_t boff[MPV_ADAM_MAX_TENSORS + 1];  // first block of each tensor
  int n;
  double lr, beta1, beta2, weight_decay, eps;
  const float* found_inf;
  const double* lr_dev;
};

template <typename T>
MPV_DEV void adam_elem(T& param, T grad, T& exp_avg, T& exp_avg_sq, const AdamBatch& a, double lr,
                       T bc1, T bc2s) {
  // adam_math with opmath_t = T: the double hyper-parameters promote each
  // expression to double, the result is stored back to T
  if (a.weight_decay != 0) grad += param * a.weight_decay;
  exp_avg = a.beta1 * exp_avg + (1 - a.beta1) * grad;
  exp_avg_sq = a.beta2 * exp_avg_sq + (1 - a.beta2) * grad * grad;
  const T step_size = lr / bc1;
  const T denom = (std::sqrt(exp_avg_sq) / bc2s) + a.eps;
  param -= step_size * exp_avg / denom;
}

template <typename T>
MPV_DEV void adam_block(const mpv_adam_tensor& t, int64_t e0, const AdamBatch& a, double lr) {
  // bias corrections in double from the float step count, then to T; the
  // count is this update's (torch's foreach_add of 1.0 in float, done here)
  const float step = *t.step + 1.0f;
  const T bc1 = (T)(1 - ::pow(a.beta1, step));
  const T bc2s = (T)std::sqrt(1 - ::pow(a.beta2, step));
  T* p = reinterpret_cast<T*>(t.param);
  const T* g = reinterpret_cast<const T*>(t.grad);
  T* m = reinterpret_cast<T*>(t.exp_avg);
  T* v = reinterpret_cast<T*>(t.exp_avg_sq);
#pragma unroll
  for (int k = 0; k < kAdamPer; ++k) {
    const int64_t e = e0 + k * kAdamThreads + threadIdx.x;
    if (e < t.numel) {
      T pe = p[e], me = m[e], ve = v[e];
      adam_elem<T>(pe, g[e], me, ve, a, lr, bc1, bc2s);
      p[e] = pe;
      m[e] = me;
      v[e] = ve;
    }
  }
}

__global__ __launch_bounds__(kAdamThreads) void adam_kernel(AdamBatch a) {
  if (a.found_inf != nullptr && *a.found_inf == 1.0f) return;
  const int64_t blk = blockIdx.x;
  const double lr = a.lr_dev != nullptr ? *a.lr_dev : a.lr;
  int q = 0;
  for (int k = 1; k < a.n; ++k)
    if (blk >= a.boff[k]) q = k;
  const mpv_adam_tensor& t = a.t[q];
  const int64_t e0 = (blk - a.boff[q]) * kAdamBlock;
  if (t.is_f64)
    adam_block<double>(t, e0, a, lr);
  else
    adam_block<float>(t, e0, a, lr);
}

struct FinishBatch {
  float* steps[MPV_ADAM_FINISH_MAX];
  int n_steps, n_lr;
  const float* found_inf;
  int64_t* updates;
  double* lr;
  int64_t* last_epoch;
  double step_size, gamma;
};

__global__ __launch_bounds__(MPV_ADAM_FINISH_MAX) void adam_finish_kernel(FinishBatch a) {
  const float f = a.found_inf != nullptr ? *a.found_inf : 0.0f;
  const int i = threadIdx.x;
  // torch: step += 1 (before the update), step -= found_inf (after it)
  if (i < a.n_steps) a.steps[i][0] = (a.steps[i][0] + 1.0f) - f;
  if (i != 0 || f == 1.0f) return;
  if (a.updates != nullptr) a.updates[0] += 1;
  if (a.n_lr == 0) return;
  // StepLR.step() -> get_lr(): chainable form, lr * gamma when last_epoch is
  // a non-zero multiple of step_size (Python's % on a float step_size)
  const int64_t e = ++a.last_epoch[0];
  if (e != 0 && ::fmod((double)e, a.step_size) == 0.0)
    for (int g = 0; g < a.n_lr; ++g) a.lr[g] = a.lr[g] * a.gamma;
}

}  // namespace
}  // namespace mpv

using namespace mpv;

extern "C" int mpv_adam_step(const mpv_adam_args* args, void* stream) {
  MPV_REQUIRE(args != nullptr && args->n >= 0 && args->n <= MPV_ADAM_MAX_TENSORS,
              "adam: 0..%d tensors per launch", MPV_ADAM_MAX_TENSORS);
  AdamBatch a;
  a.n = args->n;
  a.lr = args->lr;
  a.beta1 = args->beta1;
  a.beta2 = args->beta2;
  a.weight_decay = args->weight_decay;
  a.eps = args->eps;
  a.found_inf = args->found_inf;
  a.lr_dev = args->lr_dev;
  a.boff[0] = 0;
  for (int k = 0; k < args->n; ++k) {
    const mpv_adam_tensor& t = args->t[k];
    MPV_REQUIRE(t.numel >= 0, "adam: bad numel (tensor %d)", k);
    MPV_REQUIRE(t.numel == 0 || (t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.step),
                "adam: NULL pointer (tensor %d)", k);
    a.t[k] = t;
    a.boff[k + 1] = a.boff[k] + cdiv(t.numel, (int64_t)kAdamBlock);
  }
  for (int k = args->n; k < MPV_ADAM_MAX_TENSORS; ++k) a.boff[k + 1] = a.boff[k];
  const int64_t blocks = a.boff[args->n];
  MPV_REQUIRE(blocks < (1ll << 31), "adam: too many elements");
  if (blocks == 0) return MPV_OK;
  MPV_LAUNCH("adam", adam_kernel, dim3((unsigned)blocks), dim3(kAdamThreads), 0,
             as_stream(stream), a);
  return check_launch("adam");
}

extern "C" int mpv_adam_finish(const mpv_adam_finish_args* args, void* stream) {
  MPV_REQUIRE(args != nullptr && args->n_steps >= 0 && args->n_steps <= MPV_ADAM_FINISH_MAX,
              "adam_finish: 0..%d step counts per launch", MPV_ADAM_FINISH_MAX);
  MPV_REQUIRE(args->n_lr >= 0, "adam_finish: bad n_lr");
  MPV_REQUIRE(args->n_lr == 0 || (args->lr != nullptr && args->last_epoch != nullptr &&
                                  args->step_size > 0.0),
              "adam_finish: a scheduler needs lr, last_epoch and step_size > 0");
  FinishBatch a;
  a.n_steps = args->n_steps;
  for (int k = 0; k < args->n_steps; ++k) {
    MPV_REQUIRE(args->steps[k] != nullptr, "adam_finish: NULL step count %d", k);
    a.steps[k] = args->steps[k];
  }
  a.found_inf = args->found_inf;
  a.updates = args->updates;
  a.n_lr = args->n_lr;
  a.lr = args->lr;
  a.last_epoch = args->last_epoch;
  a.step_size = args->step_size;
  a.gamma = args->gamma;
  if (a.n_steps == 0 && a.updates == nullptr && a.n_lr == 0) return MPV_OK;
  MPV_LAUNCH("adam_finish", adam_finish_kernel, dim3(1), dim3(MPV_ADAM_FINISH_MAX), 0,
             as_stream(stream), a);
  return check_launch("adam_finish");
}
