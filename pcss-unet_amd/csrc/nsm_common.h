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

// Bilinear resize, align_corners=True (ATen upsample_bilinear2d semantics:
// scale=(in-1)/(out-1) in fp32, src=scale*dst, i0=floor, i1=i0+(i0<in-1),
// l1=src-i0, l0=1-l1): the source taps of destination index dst.
__device__ __forceinline__ void lin_idx(float scale, int dst, int in, int& i0, int& i1, float& l0,
                                        float& l1) {
  // keep src rounded to fp32 as ATen does; letting the compiler contract
  // scale*dst - i0 into one FMA shifts lambda by up to ~1e-5.
#pragma clang fp contract(off)
  float src = scale * (float)dst;
  i0 = min((int)src, in - 1);
  l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  l0 = 1.f - l1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
}

static inline float ac_scale(int in, int out) {  // align_corners source step
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
}

// ---- bf16 storage (NSM_BF16 tensors): raw 16-bit words, fp32 arithmetic ------
typedef unsigned short bf16_t;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  bf16x2 v = __builtin_convertvector((f32x2){a, b}, bf16x2);  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float round_bf(float a) { return bf_lo(pack_bf2(a, 0.f)); }

// 4 consecutive elements of a T = float | bf16_t buffer as / from f32x4
__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 ld4(const bf16_t* p) {
  const u32x2 w = *(const u32x2*)p;
  return f32x4{bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)};
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void st4(bf16_t* p, f32x4 v) {
  *(u32x2*)p = u32x2{pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
}
// 8 consecutive elements per lane (16 B of bf16 / 32 B of fp32): the unit of
// the streaming kernels, so a bf16 lane moves a full 16-B vector
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct F8 {
  f32x4 a, b;
};
__device__ __forceinline__ F8 operator+(F8 x, F8 y) { return F8{x.a + y.a, x.b + y.b}; }
__device__ __forceinline__ F8 operator-(F8 x, F8 y) { return F8{x.a - y.a, x.b - y.b}; }
__device__ __forceinline__ F8 operator*(F8 x, F8 y) { return F8{x.a * y.a, x.b * y.b}; }
__device__ __forceinline__ F8 operator*(float s, F8 x) { return F8{s * x.a, s * x.b}; }
__device__ __forceinline__ F8& operator+=(F8& x, F8 y) {
  x.a += y.a;
  x.b += y.b;
  return x;
}
__device__ __forceinline__ F8 f8zero() { return F8{f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}}; }
__device__ __forceinline__ F8 ld8(const float* p) { return F8{*(const f32x4*)p, *(const f32x4*)(p + 4)}; }
__device__ __forceinline__ F8 ld8(const bf16_t* p) {
  const u32x4 w = *(const u32x4*)p;
  return F8{f32x4{bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)},
            f32x4{bf_lo(w.z), bf_hi(w.z), bf_lo(w.w), bf_hi(w.w)}};
}
__device__ __forceinline__ void st8(float* p, F8 v) {
  *(f32x4*)p = v.a;
  *(f32x4*)(p + 4) = v.b;
}
__device__ __forceinline__ void st8(bf16_t* p, F8 v) {
  *(u32x4*)p = u32x4{pack_bf2(v.a.x, v.a.y), pack_bf2(v.a.z, v.a.w), pack_bf2(v.b.x, v.b.y),
                     pack_bf2(v.b.z, v.b.w)};
}
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) { return __uint_as_float((uint32_t)*p << 16); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = (bf16_t)(pack_bf2(v, 0.f) & 0xFFFFu); }

// ---- |x| maxima of f16x2 GEMM operands (nsm_conv_split16.inc) ---------------
// fp32 bit patterns of |x| compare as unsigned (NaN above +Inf). An operand's
// maximum lives in a slot of NSM_AMAX_WORDS uint32 (include/nsm.h): 64 partial
// maxima on separate 128-B lines, so the atomics of thousands of producer
// waves spread over 64 addresses instead of queueing on one. A producer folds
// what it stores into a per-thread max and flushes it once per wave (every
// lane of the wave must reach amax_flush) into the line of its block;
// consumers reduce the 64 lines (amax_read). out == NULL: nothing recorded.
constexpr int AMAX_LINES = 64, AMAX_STRIDE = 32;  // NSM_AMAX_WORDS = 2048
__device__ __forceinline__ void amax_fold(uint32_t& m, float v) {
  m = max(m, __float_as_uint(v) & 0x7fffffffu);
}
__device__ __forceinline__ void amax_fold(uint32_t& m, f32x4 v) {
  amax_fold(m, v.x);
  amax_fold(m, v.y);
  amax_fold(m, v.z);
  amax_fold(m, v.w);
}
__device__ __forceinline__ void amax_flush(uint32_t m, uint32_t* out) {
  if (!out) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  const uint32_t line = (blockIdx.x + 7u * blockIdx.y + 13u * blockIdx.z) & (AMAX_LINES - 1);
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out + line * AMAX_STRIDE, m);
}
// the maximum a slot holds (uniform over the wave; all 64 lanes must call)
__device__ __forceinline__ uint32_t amax_read(const uint32_t* p) {
  uint32_t m = p[(threadIdx.x & 63) * AMAX_STRIDE];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  return m;
}

// ---- the f16x2 split of power-of-two scaled fp32 operands (h2 tensors) ------
// (nsm_conv_split16.inc, nsm_conv_h2.inc): shared by the GEMM TU and the
// elementwise TU, whose producers write h2 operands
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// s = 2^(15 - ceil(log2 m)) from the bits of m = max|X| (0, Inf, NaN -> 1).
// Clamped to [-126, 126] so that s and the epilogue's undo factor 2^-se are
// both normal floats (exp2i(-127) would be the bit pattern 0): an operand
// whose maximum is below 2^-111 is scaled by 2^126 only, i.e. represented with
// fewer significand bits, but never flushed to an all-zero GEMM.
__device__ __forceinline__ int pow2_scale_exp(uint32_t u) {
  if (u == 0u || u >= 0x7f800000u) return 0;
  int e = (int)(u >> 23) - 127;  // floor(log2 m) (subnormal m: -127)
  if (u & 0x7fffffu) e += 1;     // ceil
  int se = 15 - e;
  return se < -126 ? -126 : (se > 126 ? 126 : se);
}
__device__ __forceinline__ float exp2i(int e) { return __int_as_float((e + 127) << 23); }

__device__ __forceinline__ uint32_t pack_h2(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
}
__device__ __forceinline__ f32x2 unpack_h2(uint32_t w) {
  return __builtin_convertvector(__builtin_bit_cast(f16x2, w), f32x2);
}

// f16 Winograd M of the bf16 path (nsm_conv_h2.inc, O16): 15 + ceil log2 K
__device__ __forceinline__ int o16_exp(int K) {
  return 15 + (K > 1 ? 32 - __builtin_clz((unsigned)(K - 1)) : 0);
}
__device__ __forceinline__ u32x2 pack_f16x4(f32x4 v) {
  return u32x2{pack_h2(f32x2{v.x, v.y}), pack_h2(f32x2{v.z, v.w})};
}

// ---- f16 storage (NSM_F16 tensors, the fp16-autocast mode) -----------------
// raw IEEE half words behind a distinct element type, so the elementwise
// templates instantiate for it beside float and bf16_t; RNE conversions
// (values beyond 65504 become +-Inf, as in the reference's fp16 tensors)
struct f16_t {
  unsigned short bits;
};
__device__ __forceinline__ float h_lo(uint32_t w) { return (float)__builtin_bit_cast(f16x2, w).x; }
__device__ __forceinline__ float h_hi(uint32_t w) { return (float)__builtin_bit_cast(f16x2, w).y; }
__device__ __forceinline__ uint32_t pack_hh(float a, float b) { return pack_h2(f32x2{a, b}); }
__device__ __forceinline__ f32x4 ld4(const f16_t* p) {
  const u32x2 w = *(const u32x2*)p;
  return f32x4{h_lo(w.x), h_hi(w.x), h_lo(w.y), h_hi(w.y)};
}
__device__ __forceinline__ void st4(f16_t* p, f32x4 v) {
  *(u32x2*)p = u32x2{pack_hh(v.x, v.y), pack_hh(v.z, v.w)};
}
__device__ __forceinline__ F8 ld8(const f16_t* p) {
  const u32x4 w = *(const u32x4*)p;
  return F8{f32x4{h_lo(w.x), h_hi(w.x), h_lo(w.y), h_hi(w.y)},
            f32x4{h_lo(w.z), h_hi(w.z), h_lo(w.w), h_hi(w.w)}};
}
__device__ __forceinline__ void st8(f16_t* p, F8 v) {
  *(u32x4*)p = u32x4{pack_hh(v.a.x, v.a.y), pack_hh(v.a.z, v.a.w), pack_hh(v.b.x, v.b.y),
                     pack_hh(v.b.z, v.b.w)};
}
__device__ __forceinline__ float ld1(const f16_t* p) { return h_lo((uint32_t)p->bits); }
__device__ __forceinline__ void st1(f16_t* p, float v) {
  p->bits = (unsigned short)(pack_hh(v, 0.f) & 0xFFFFu);
}

__device__ __forceinline__ void split4h(f32x4 v, float s, u32x2& h, u32x2& l) {
  const f32x2 a = f32x2{v.x, v.y} * s, b = f32x2{v.z, v.w} * s;
  h = u32x2{pack_h2(a), pack_h2(b)};
  l = u32x2{pack_h2(a - unpack_h2(h.x)), pack_h2(b - unpack_h2(h.y))};
}

// ---- pre-split (h2) operands: scale source and writers (nsm_conv_h2.inc) ----
struct H2Scale {
  const uint32_t* amax;  // max|source| slot (NSM_AMAX_WORDS)
  float beta;            // max|operand| <= beta * max|source|
};
// beta * max can overflow fp32 for a finite max (beta is 3969 for the F(6x6)
// output-gradient transform): that saturates at FLT_MAX (s = 2^-113, every
// finite operand value fits f16) instead of reading as Inf (s = 1, values
// above 65504 would turn Inf). A non-finite max keeps s = 1 (NaN propagates).
__device__ __forceinline__ int h2_exp(const H2Scale& s) {
  const uint32_t m = amax_read(s.amax);
  uint32_t b = __float_as_uint(__uint_as_float(m) * s.beta);
  if (m < 0x7f800000u && b >= 0x7f800000u) b = 0x7f7fffffu;
  return pow2_scale_exp(b);
}

// 4 consecutive channels c..c+3 (c % 4 == 0) of one lane: h and l as 8-B words
__device__ __forceinline__ void h2_store4(bf16_t* row, int c, f32x4 v, float s) {
  u32x2 h, l;
  split4h(v, s, h, l);
  const int o = 16 * (c >> 3) + (c & 7);
  *(u32x2*)(row + o) = h;
  *(u32x2*)(row + o + 8) = l;
}
// 8 consecutive channels c..c+7 (c % 8 == 0) of one lane: h and l as one
// 16-B word each (row = the h2 row of the pixel)
__device__ __forceinline__ void h2_store8(bf16_t* row, int c, F8 v, float s) {
  u32x2 ha, la, hb, lb;
  split4h(v.a, s, ha, la);
  split4h(v.b, s, hb, lb);
  *(u32x4*)(row + 2 * c) = u32x4{ha.x, ha.y, hb.x, hb.y};
  *(u32x4*)(row + 2 * c + 8) = u32x4{la.x, la.y, lb.x, lb.y};
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace nsm
