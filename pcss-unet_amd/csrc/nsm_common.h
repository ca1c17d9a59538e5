// Shared helpers for the MI355X (gfx950) U-Net hot-path kernels.
// Everything here is device/host glue: error plumbing, fast integer division,
// vector types. No allocation, no host synchronisation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>

#include "../../include/nsm.h"

namespace nsm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- error handling: thread-local last error, int return codes ----------
void set_error(const std::string& msg);
int fail(int code, const char* fmt, ...);

#define NSM_CHECK_ARG(cond, ...)                                   \
  do {                                                             \
    if (!(cond)) return ::nsm::fail(NSM_E_ARG, __VA_ARGS__);       \
  } while (0)

#define NSM_LAUNCH_CHECK(what)                                          \
  do {                                                                  \
    hipError_t _e = hipGetLastError();                                  \
    if (_e != hipSuccess)                                               \
      return ::nsm::fail(NSM_E_HIP, "%s: %s", what, hipGetErrorString(_e)); \
  } while (0)

// ---- fast unsigned division by a runtime-invariant divisor ---------------
// q = umulhi(n, mul) >> shr, exact for 0 <= n < 2^31 (d >= 1).
struct FastDiv {
  uint32_t d, mul, shr;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d <= 1) {
    f.mul = 0;
    f.shr = 0;
    return f;
  }
  uint32_t l = 0;
  while ((1u << l) < d) ++l;  // ceil(log2 d)
  uint32_t p = 31 + l;
  f.mul = (uint32_t)(((1ull << p) + d - 1) / d);
  f.shr = p - 32;
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  // d == 1 has mul == 0: umulhi gives 0 and the second term returns n
  // (arithmetic select: no branch around the division).
  return (__umulhi(n, f.mul) >> f.shr) + (f.mul == 0 ? n : 0u);
}

__device__ __forceinline__ float lrelu(float v, float slope) {
  // ATen leaky_relu: x > 0 ? x : x * negval  (Unetmodel.py:23,28)
  return v > 0.f ? v : v * slope;
}

__device__ __forceinline__ float lrelu_grad(float z, float slope) {
  // ATen leaky_relu_backward: self > 0 ? grad : grad * negval
  return z > 0.f ? 1.f : slope;
}

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace nsm
