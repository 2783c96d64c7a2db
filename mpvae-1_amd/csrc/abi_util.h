// Host-side helpers shared by the C-ABI entry points.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpvae_hip.h"

namespace mpv {

// Record a message for mpv_last_error() and return `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// After a kernel launch: MPV_OK, or MPV_ELAUNCH with the HIP error text.
int check_launch(const char* what);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Shape sanity shared by forward and backward.
int check_shape(const mpv_shape* s);

// Brackets one kernel launch with HIP events when mpv_timing_enable(1) is on
// (no cost otherwise beyond one branch).
class TimedLaunch {
 public:
  TimedLaunch(const char* kernel, hipStream_t s);
  ~TimedLaunch();

 private:
  int slot_ = -1;
  size_t pair_ = 0;
  hipStream_t s_;
};

}  // namespace mpv

// hipLaunchKernelGGL under a TimedLaunch scope named `tag`.
#define MPV_LAUNCH(tag, kernel, grid, block, shm, stream, ...)                  \
  do {                                                                         \
    ::mpv::TimedLaunch mpv_tl_(tag, stream);                                   \
    hipLaunchKernelGGL(kernel, grid, block, shm, stream, __VA_ARGS__);         \
  } while (0)

#define MPV_REQUIRE(cond, ...)                         \
  do {                                                 \
    if (!(cond)) return ::mpv::fail(MPV_EINVAL, __VA_ARGS__); \
  } while (0)
