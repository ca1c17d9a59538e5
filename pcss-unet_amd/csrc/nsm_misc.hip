// Small boundary kernels of the drop-in surface:
//  * NCHW <-> NHWC layout changes for a standalone DoubleConv call
//    (Unetmodel.py:32-33: `DoubleConv.forward(x)` on an NCHW tensor), tiled
//    through LDS so both the NCHW rows and the NHWC pixel vectors are coalesced;
//  * the output-range assertion of CustomLoss / PerturbationLoss
//    (customLoss.py:131, pert_loss.py:131: min >= 0 and max <= 1, NaN fails)
//    as a sticky device flag, so the check costs no host synchronisation.
#include <algorithm>
#include "nsm_common.h"

namespace nsm {

constexpr int LT_P = 64;  // pixels per tile
constexpr int LT_C = 32;  // channels per tile

// x [B][C][HW] fp32 -> y [B*HW][cp] (T), channels C..cp-1 written as 0.
template <typename T>
__global__ void __launch_bounds__(256) nchw_to_nhwc_kernel(const float* __restrict__ x, int C,
                                                           int HW, int cp, T* __restrict__ y,
                                                           int ldy) {
  __shared__ float tile[LT_C][LT_P + 1];
  const int b = blockIdx.z, c0 = blockIdx.y * LT_C, p0 = blockIdx.x * LT_P;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  for (int cc = ty; cc < LT_C; cc += 4) {
    const int c = c0 + cc, p = p0 + tx;
    float v = 0.f;
    if (c < C && p < HW) v = x[((size_t)b * C + c) * HW + p];
    tile[cc][tx] = v;
  }
  __syncthreads();
  const int lc = threadIdx.x & 31, lp = threadIdx.x >> 5;  // 32 x 8
  for (int pp = lp; pp < LT_P; pp += 8) {
    const int p = p0 + pp, c = c0 + lc;
    if (p < HW && c < cp) st1(y + ((size_t)b * HW + p) * ldy + c, tile[lc][pp]);
  }
}

// z [B*HW][ld] (T) -> x [B][C][HW] fp32 (first C channels)
template <typename T>
__global__ void __launch_bounds__(256) nhwc_to_nchw_kernel(const T* __restrict__ z, int ldz, int C,
                                                           int HW, float* __restrict__ x) {
  __shared__ float tile[LT_C][LT_P + 1];
  const int b = blockIdx.z, c0 = blockIdx.y * LT_C, p0 = blockIdx.x * LT_P;
  const int lc = threadIdx.x & 31, lp = threadIdx.x >> 5;
  for (int pp = lp; pp < LT_P; pp += 8) {
    const int p = p0 + pp, c = c0 + lc;
    tile[lc][pp] = (p < HW && c < C) ? ld1(z + ((size_t)b * HW + p) * ldz + c) : 0.f;
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int cc = ty; cc < LT_C; cc += 4) {
    const int c = c0 + cc, p = p0 + tx;
    if (c < C && p < HW) x[((size_t)b * C + c) * HW + p] = tile[cc][tx];
  }
}

// flag[0] = 1 if any o[i] < lo, o[i] > hi or o[i] is NaN; never written 0
__global__ void __launch_bounds__(256) range_flag_kernel(const float* __restrict__ o, int64_t n,
                                                         float lo, float hi, int* flag) {
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = o[i];
    bad |= !(v >= lo && v <= hi);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) flag[0] = 1;
}

// Dropout2d masks of every block of one forward in ONE launch: job j covers
// rows [B] x channels [cp_j] at offset off_j of `out`; m = (u < keep) / keep
// for c < c_real, 0 in the padded channels; u from a counter-based hash of
// (seed, job, b, c). desc[j] = {offset, c_real, cp, keep (float bits)}.
__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// seed_dev (nsm_dropout_masks_dev): the seed read from device memory, so a
// captured graph draws new masks on every replay (torch's graph-safe generator
// writes it there)
__global__ void __launch_bounds__(256) dropout_masks_kernel(const int* __restrict__ desc, int njobs,
                                                            int B, uint64_t seed,
                                                            float* __restrict__ out,
                                                            const int64_t* __restrict__ seed_dev) {
  const int j = blockIdx.y;
  if (j >= njobs) return;
  if (seed_dev) seed = (uint64_t)seed_dev[0];
  const int off = desc[4 * j], creal = desc[4 * j + 1], cp = desc[4 * j + 2];
  const float keep = __int_as_float(desc[4 * j + 3]);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * cp; i += gridDim.x * blockDim.x) {
    const int c = i % cp, b = i / cp;
    float v = 0.f;
    if (c < creal) {
      const uint32_t h = hash32(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(((uint64_t)j << 40) |
                                                                      ((uint64_t)b << 20) | c));
      const float u = (float)(h >> 8) * (1.f / 16777216.f);  // [0, 1)
      v = u < keep ? 1.f / keep : 0.f;
    }
    out[off + i] = v;
  }
}

// profiling marker (nsm_stage_mark): no work, its grid encodes the stage
__global__ void __launch_bounds__(64) stage_mark_kernel(int code) {}

__global__ void __launch_bounds__(256) zero_u32_kernel(uint32_t* __restrict__ p, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    p[i] = 0u;
}

}  // namespace nsm

using namespace nsm;

extern "C" int nsm_stage_mark(int code, void* stream) {
  NSM_CHECK_ARG(code >= 0 && code < 4096, "stage_mark: bad code");
  hipLaunchKernelGGL(stage_mark_kernel, dim3(code + 1), dim3(64), 0, as_stream(stream), code);
  NSM_LAUNCH_CHECK("stage_mark");
  return 0;
}

extern "C" int nsm_zero_u32(uint32_t* p, int64_t n, void* stream) {
  NSM_CHECK_ARG(p && n > 0, "zero_u32: bad args");
  const long long g = std::min<long long>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(zero_u32_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), p,
                     (long long)n);
  NSM_LAUNCH_CHECK("zero_u32");
  return 0;
}

extern "C" int nsm_dropout_masks(const int* desc, int njobs, int B, uint64_t seed, float* out,
                                 void* stream) {
  NSM_CHECK_ARG(desc && out && njobs > 0 && B > 0, "dropout_masks: bad args");
  hipLaunchKernelGGL(dropout_masks_kernel, dim3(8, njobs), dim3(256), 0, as_stream(stream), desc,
                     njobs, B, seed, out, nullptr);
  NSM_LAUNCH_CHECK("dropout_masks");
  return 0;
}

extern "C" int nsm_dropout_masks_dev(const int* desc, int njobs, int B, const int64_t* seed,
                                     float* out, void* stream) {
  NSM_CHECK_ARG(desc && out && seed && njobs > 0 && B > 0, "dropout_masks_dev: bad args");
  hipLaunchKernelGGL(dropout_masks_kernel, dim3(8, njobs), dim3(256), 0, as_stream(stream), desc,
                     njobs, B, 0ull, out, seed);
  NSM_LAUNCH_CHECK("dropout_masks_dev");
  return 0;
}

extern "C" int nsm_nchw_to_nhwc(const float* x, int B, int C, int H, int W, void* y, int cp,
                                int ldy, int dtype, void* stream) {
  NSM_CHECK_ARG(x && y && B > 0 && C > 0 && cp >= C && ldy >= cp && H * W > 0,
                "nchw_to_nhwc: bad args");
  const int HW = H * W;
  dim3 grid((HW + LT_P - 1) / LT_P, (cp + LT_C - 1) / LT_C, B);
  hipStream_t s = as_stream(stream);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, grid, dim3(256), 0, s, x, C, HW, cp,
                       (bf16_t*)y, ldy);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<f16_t>, grid, dim3(256), 0, s, x, C, HW, cp,
                       (f16_t*)y, ldy);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, grid, dim3(256), 0, s, x, C, HW, cp, (float*)y,
                       ldy);
  NSM_LAUNCH_CHECK("nchw_to_nhwc");
  return 0;
}

extern "C" int nsm_nhwc_to_nchw(const void* z, int ldz, int B, int C, int H, int W, float* x,
                                int dtype, void* stream) {
  NSM_CHECK_ARG(z && x && B > 0 && C > 0 && ldz >= C && H * W > 0, "nhwc_to_nchw: bad args");
  const int HW = H * W;
  dim3 grid((HW + LT_P - 1) / LT_P, (C + LT_C - 1) / LT_C, B);
  hipStream_t s = as_stream(stream);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)z, ldz,
                       C, HW, x);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<f16_t>, grid, dim3(256), 0, s, (const f16_t*)z, ldz,
                       C, HW, x);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, grid, dim3(256), 0, s, (const float*)z, ldz, C,
                       HW, x);
  NSM_LAUNCH_CHECK("nhwc_to_nchw");
  return 0;
}

extern "C" int nsm_range_flag(const float* o, int64_t n, float lo, float hi, int* flag,
                              void* stream) {
  NSM_CHECK_ARG(o && flag && n > 0, "range_flag: bad args");
  long long g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(range_flag_kernel, dim3((int)g), dim3(256), 0, as_stream(stream), o, n, lo, hi,
                     flag);
  NSM_LAUNCH_CHECK("range_flag");
  return 0;
}
