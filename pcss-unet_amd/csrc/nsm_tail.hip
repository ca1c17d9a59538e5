// Train-step tail of main.py:287-423 on the device, with no host
// synchronisation: gradient sanitising (NaN/Inf census, >20 % skip, repair),
// the per-parameter pre-unscale clip to 1000*scale, the per-parameter 1e5 skip /
// 1e3 rescale, clip_grad_norm_(max_norm), the post-clip max-norm > 10 skip, and
// an AdamW step that honours the device skip flag.
//
// The gradient is ONE flat fp32 buffer holding the module's parameters in
// order; `seg_off[nseg+1]` delimits the parameters ("segments"). Work is cut
// into blocks that never straddle a segment (nsm_tail_plan), so every
// per-parameter statistic is a deterministic fixed-order reduction of
// per-block partials. Decisions the reference takes on the host (`.item()`,
// `continue`) become device flags read by the kernels that follow, so the whole
// tail is a fixed launch sequence (hipGraph-capturable).
//
// Rounding follows the reference's fp32 op sequence: grads are multiplied by the
// pre-clip factor, then the 1e3 rescale, then the clip coefficient (three
// separate fp32 products, exactly like the three mul_ calls), and AdamW is
// torch's single-tensor AdamW. FP contraction is off in this file so no FMA
// merges two of those roundings.
#include <cfloat>
#include <math.h>

#include "nsm_common.h"

#pragma clang fp contract(off)

namespace nsm {

constexpr int TAIL_THREADS = 256;
constexpr int64_t TAIL_CHUNK = 8192;  // elements per block (32 per thread)

// workspace layout (all offsets 8-byte aligned)
struct TailWs {
  double* blk_d;    // [nblk][2]  sum, sumsq of finite values (pre-repair)
  int* blk_i;       // [nblk][2]  nan count, inf count
  float* blk_max;   // [nblk]     max |finite|
  double* rep_d;    // [nblk]     sumsq after repair
  int* rep_i;       // [nblk]     non-finite count after repair
  double* seg_d;    // [nseg][4]  mean, std, maxabs, sumsq
  int* seg_i;       // [nseg][2]  invalid count, zeroed
  int* ctl;         // [4]        0: repair needed, 1: severe
};

static inline size_t align8(size_t x) { return (x + 7) & ~(size_t)7; }

static size_t tail_ws_layout(int nseg, int nblk, char* base, TailWs* w) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off = align8(off + bytes);
    return base ? base + o : nullptr;
  };
  char* p;
  p = take(sizeof(double) * 2 * nblk);
  if (w) w->blk_d = (double*)p;
  p = take(sizeof(int) * 2 * nblk);
  if (w) w->blk_i = (int*)p;
  p = take(sizeof(float) * nblk);
  if (w) w->blk_max = (float*)p;
  p = take(sizeof(double) * nblk);
  if (w) w->rep_d = (double*)p;
  p = take(sizeof(int) * nblk);
  if (w) w->rep_i = (int*)p;
  p = take(sizeof(double) * 4 * nseg);
  if (w) w->seg_d = (double*)p;
  p = take(sizeof(int) * 2 * nseg);
  if (w) w->seg_i = (int*)p;
  p = take(sizeof(int) * 4);
  if (w) w->ctl = (int*)p;
  return off;
}

__device__ __forceinline__ bool is_finite_f(float v) { return fabsf(v) <= 3.402823466e38f; }

template <typename T>
__device__ __forceinline__ T wave_red_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_red_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block of 256 threads: sum over the block, result valid in thread 0
template <typename T>
__device__ __forceinline__ T block_red_sum(T v, T* sh) {
  v = wave_red_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  T r = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < TAIL_THREADS / 64; ++k) r += sh[k];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_red_max(float v, float* sh) {
  v = wave_red_max(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < TAIL_THREADS / 64; ++k) r = fmaxf(r, sh[k]);
  __syncthreads();
  return r;
}

// ---- K1: per-block census of the (rank-averaged) gradient --------------------
// main.py:295-312: isnan / isinf counts per parameter; the finite values'
// sum, sum of squares and max |.| feed the repair statistics (:326-346) and the
// per-parameter norm (:365). With inv_world != 1 the DP sum is turned into the
// mean in place first (the tail then sees what a single process would).
__global__ void __launch_bounds__(TAIL_THREADS) tail_stats_kernel(
    float* __restrict__ g, const int64_t* __restrict__ blk_lo, const int64_t* __restrict__ blk_hi,
    float inv_world, TailWs w) {
  __shared__ double shd[4];
  __shared__ int shi[4];
  __shared__ float shf[4];
  const int b = blockIdx.x;
  const int64_t lo = blk_lo[b], hi = blk_hi[b];
  double s = 0.0, s2 = 0.0;
  int nn = 0, ni = 0;
  float mx = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += TAIL_THREADS) {
    float v = g[i];
    if (inv_world != 1.f) {
      v = v * inv_world;
      g[i] = v;
    }
    if (v != v) {
      ++nn;
    } else if (!is_finite_f(v)) {
      ++ni;
    } else {
      s += (double)v;
      s2 += (double)v * (double)v;
      mx = fmaxf(mx, fabsf(v));
    }
  }
  s = block_red_sum(s, shd);
  s2 = block_red_sum(s2, shd);
  nn = block_red_sum(nn, shi);
  ni = block_red_sum(ni, shi);
  mx = block_red_max(mx, shf);
  if (threadIdx.x == 0) {
    w.blk_d[2 * b] = s;
    w.blk_d[2 * b + 1] = s2;
    w.blk_i[2 * b] = nn;
    w.blk_i[2 * b + 1] = ni;
    w.blk_max[b] = mx;
  }
}

// ---- K2: per-parameter statistics + the skip / repair decision ---------------
// One block; wave k reduces segments k, k+16, ... over their blocks in order.
// severe (main.py:305-317): some parameter has (nan+inf)/numel > 0.2 -> skip.
// fixable (:311,320): some parameter has an invalid value -> repair all.
__global__ void __launch_bounds__(1024) tail_decide_kernel(const int64_t* __restrict__ seg_off,
                                                           const int* __restrict__ seg_blk,
                                                           int nseg, TailWs w) {
  __shared__ int sh_sev[16], sh_fix[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int sev = 0, fix = 0;
  for (int sgi = wv; sgi < nseg; sgi += 16) {
    const int b0 = seg_blk[sgi], b1 = seg_blk[sgi + 1];
    double s = 0.0, s2 = 0.0;
    long long nn = 0, ni = 0;
    float mx = 0.f;
    for (int b = b0 + lane; b < b1; b += 64) {
      s += w.blk_d[2 * b];
      s2 += w.blk_d[2 * b + 1];
      nn += w.blk_i[2 * b];
      ni += w.blk_i[2 * b + 1];
      mx = fmaxf(mx, w.blk_max[b]);
    }
    s = wave_red_sum(s);
    s2 = wave_red_sum(s2);
    nn = wave_red_sum(nn);
    ni = wave_red_sum(ni);
    mx = wave_red_max(mx);
    if (lane == 0) {
      const long long numel = seg_off[sgi + 1] - seg_off[sgi];
      const long long bad = nn + ni;
      const long long nv = numel - bad;
      // torch: valid_grads.mean() / .std() (unbiased; 0.01 when one value)
      const double mean = nv > 0 ? s / (double)nv : 0.0;
      double var = nv > 1 ? (s2 - s * mean) / (double)(nv - 1) : 0.0;
      if (var < 0.0) var = 0.0;
      w.seg_d[4 * sgi + 0] = mean;
      w.seg_d[4 * sgi + 1] = nv > 1 ? sqrt(var) : 0.01;
      w.seg_d[4 * sgi + 2] = (double)mx;
      w.seg_d[4 * sgi + 3] = s2;
      w.seg_i[2 * sgi + 0] = (int)(bad < 0x7fffffff ? bad : 0x7fffffff);
      w.seg_i[2 * sgi + 1] = 0;
      if (bad > 0) {
        fix = 1;
        // (nan.sum() + inf.sum()).item() / numel > 0.2, in double as in Python
        if ((double)bad / (double)numel > 0.2) sev = 1;
      }
    }
  }
  if (lane == 0) {
    sh_sev[wv] = sev;
    sh_fix[wv] = fix;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int S = 0, X = 0;
    for (int k = 0; k < 16; ++k) {
      S |= sh_sev[k];
      X |= sh_fix[k];
    }
    w.ctl[0] = (X && !S) ? 1 : 0;  // repair
    w.ctl[1] = S;                  // severe skip
  }
}

// standard normal from (seed, counter): splitmix64 -> two uniforms -> Box-Muller
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float gauss_hash(uint64_t seed, uint64_t ctr) {
  const uint64_t r = mix64(seed ^ mix64(ctr));
  const float u1 = ((float)(uint32_t)(r >> 40) + 1.f) * (1.f / 16777217.f);  // (0, 1]
  const float u2 = (float)(uint32_t)(r & 0xFFFFFFu) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cosf(6.28318530718f * u2);
}

// ---- K3: repair (main.py:320-354), only when K2 decided so -------------------
// NaN -> mean + randn * std * 0.1 ; +-Inf -> sign * max|valid| * 10.
// `noise` (optional, flat like g) supplies the randn values for parity tests;
// otherwise a counter-based generator keyed by (seed, step, index) is used.
__global__ void __launch_bounds__(TAIL_THREADS) tail_repair_kernel(
    float* __restrict__ g, const int* __restrict__ blk_seg, const int64_t* __restrict__ blk_lo,
    const int64_t* __restrict__ blk_hi, const float* __restrict__ noise, uint64_t seed,
    const int* __restrict__ step, TailWs w) {
  __shared__ double shd[4];
  __shared__ int shi[4];
  if (w.ctl[0] == 0) return;  // uniform across the grid
  const int b = blockIdx.x, sgi = blk_seg[b];
  const int64_t lo = blk_lo[b], hi = blk_hi[b];
  const float mean = (float)w.seg_d[4 * sgi + 0];
  const float stdv = (float)w.seg_d[4 * sgi + 1];
  const float mx = (float)w.seg_d[4 * sgi + 2];
  // keyed by the tail-call counter step[1] (advances on every call, skipped
  // steps included), so consecutive repairs draw independent normals
  const uint64_t key = seed ^ ((uint64_t)(uint32_t)step[1] << 40);
  double s2 = 0.0;
  int bad = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += TAIL_THREADS) {
    float v = g[i];
    if (v != v) {
      const float z = noise ? noise[i] : gauss_hash(key, (uint64_t)i);
      v = mean + (z * stdv) * 0.1f;  // valid_mean + randn * valid_std * 0.1
      g[i] = v;
    } else if (!is_finite_f(v)) {
      v = (v > 0.f ? mx : -mx) * 10.f;  // sign * max_valid * 10.0
      g[i] = v;
    }
    if (!is_finite_f(v))
      ++bad;
    else
      s2 += (double)v * (double)v;
  }
  s2 = block_red_sum(s2, shd);
  bad = block_red_sum(bad, shi);
  if (threadIdx.x == 0) {
    w.rep_d[b] = s2;
    w.rep_i[b] = bad;
  }
}

// ---- K4: norms, factors and the step decision (main.py:357-418) --------------
// seg_coef[s] = {f1 (pre-unscale clip), f2 (1e3 rescale), c (clip_grad_norm_),
// zero}; stat = {total norm, clip coef, max_norm, max post-clip norm};
// flags = {skip, repaired, severe, nonfinite, huge (>1e5), postclip (>10),
// n rescaled, n zeroed}; step[0] += !skip.
__global__ void __launch_bounds__(1024) tail_finalize_kernel(
    const int* __restrict__ seg_blk, int nseg, float scale, float max_norm, TailWs w,
    float* __restrict__ seg_coef, float* __restrict__ stat, int* __restrict__ flags,
    int* __restrict__ step) {
  __shared__ double sh_tot[16];
  __shared__ float sh_mx[16];
  __shared__ int sh_f[16][4];
  __shared__ float s_clip;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool repaired = w.ctl[0] != 0;
  double tot = 0.0;  // sum of squared per-parameter norms after f1, f2
  int nonfin = 0, huge = 0, nresc = 0, nzero = 0;
  for (int sgi = wv; sgi < nseg; sgi += 16) {
    double s2 = w.seg_d[4 * sgi + 3];
    int zero = 0;
    if (repaired) {
      const int b0 = seg_blk[sgi], b1 = seg_blk[sgi + 1];
      double r = 0.0;
      long long bad = 0;
      for (int b = b0 + lane; b < b1; b += 64) {
        r += w.rep_d[b];
        bad += w.rep_i[b];
      }
      r = wave_red_sum(r);
      bad = wave_red_sum(bad);
      s2 = r;
      if (bad > 0) {  // main.py:352-354: repair failed -> zero the gradient
        zero = 1;
        s2 = 0.0;
      }
    }
    if (lane == 0) {
      // the fp32 norm: the squares are summed in double and rounded to fp32,
      // except that a sum of squares above FLT_MAX reads +inf, as an fp32
      // accumulation of them does (the reference's device, main.py:95,
      // torch.norm on CUDA; and the CPU kernels of most hosts)
      const float n1 = s2 > (double)FLT_MAX ? __builtin_inff() : (float)sqrt(s2);
      // main.py:365: g *= clamp(1 / max(1, |g| / (1000*scale)), max=1)
      const float t = n1 / (float)(1000.0 * (double)scale);
      float f1 = t > 1.f ? 1.f / t : 1.f;
      f1 = fminf(f1, 1.f);
      // main.py:368 unscale_ (x 1/scale), then :371-397 on the unscaled grad
      const float inv_s = (float)(1.0 / (double)scale);
      float n2 = (n1 * f1) * inv_s;
      // A norm above ~1.8e19 (sum of squares > FLT_MAX) reads +inf (above).
      // Then the reference's factor 1/max(1, inf) = 0 zeroes the gradient,
      // whose norm is 0 and the step goes on (main.py:361-365); inf * 0 is NaN
      // here, so n2 is set to 0 (tests/test_gpu_tail.py::
      // test_large_finite_norm_zeroes_like_fp32_norm).
      if (n1 == __builtin_inff()) n2 = 0.f;
      // a non-finite survivor of the repair (:374-381) is impossible once
      // zeroed; only an infinite norm (overflowed sum of squares) is left
      if (!zero && !(n2 == n2)) ++nonfin;
      float f2 = 1.f;
      if (n2 > 1e3f) {
        if (n2 > 1e5f)
          ++huge;                      // :388-391 skip
        else {
          f2 = fminf(1.f, 1e3f / n2);  // :396-397
          ++nresc;
        }
      }
      const float n3 = n2 * f2;
      tot += (double)n3 * (double)n3;
      nzero += zero;
      seg_coef[4 * sgi + 0] = f1 * inv_s;  // unscale folded into the pre-clip factor
      seg_coef[4 * sgi + 1] = f2;
      seg_coef[4 * sgi + 3] = (float)zero;
      // stash n3 for the post-clip check
      seg_coef[4 * sgi + 2] = n3;
    }
  }
  if (lane == 0) {
    sh_tot[wv] = tot;
    sh_f[wv][0] = nonfin;
    sh_f[wv][1] = huge;
    sh_f[wv][2] = nresc;
    sh_f[wv][3] = nzero;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double T = 0.0;
    for (int k = 0; k < 16; ++k) T += sh_tot[k];
    // clip_grad_norm_: total = ||stack(norms)||, coef = max_norm / (total + 1e-6), clamp 1
    const float total = (float)sqrt(T);
    float c = max_norm / (total + 1e-6f);
    c = fminf(c, 1.f);
    s_clip = c;
    stat[0] = total;
    stat[1] = c;
    stat[2] = max_norm;
  }
  __syncthreads();
  const float c = s_clip;
  float mxn = 0.f;
  for (int sgi = threadIdx.x; sgi < nseg; sgi += blockDim.x) {
    const float n3 = seg_coef[4 * sgi + 2];
    mxn = fmaxf(mxn, n3 * c);
    seg_coef[4 * sgi + 2] = c;
  }
  mxn = wave_red_max(mxn);
  if (lane == 0) sh_mx[wv] = mxn;
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = 0.f;
    int nonfin_t = 0, huge_t = 0, nresc_t = 0, nzero_t = 0;
    for (int k = 0; k < 16; ++k) {
      M = fmaxf(M, sh_mx[k]);
      nonfin_t += sh_f[k][0];
      huge_t += sh_f[k][1];
      nresc_t += sh_f[k][2];
      nzero_t += sh_f[k][3];
    }
    stat[3] = M;
    const int severe = w.ctl[1];
    const int postclip = M > 10.f ? 1 : 0;  // main.py:408-418
    const int skip = (severe || nonfin_t || huge_t || postclip) ? 1 : 0;
    flags[0] = skip;
    flags[1] = repaired ? 1 : 0;
    flags[2] = severe;
    flags[3] = nonfin_t ? 1 : 0;
    flags[4] = huge_t ? 1 : 0;
    flags[5] = postclip;
    flags[6] = nresc_t;
    flags[7] = nzero_t;
    if (!skip) step[0] = step[0] + 1;
    step[1] = step[1] + 1;  // tail calls (the repair-noise key)
  }
}

// ---- K5: AdamW (torch.optim.AdamW, single-tensor path) honouring the skip ----
// p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps); g = ((g*f1)*f2)*c (or 0 if zeroed)
__global__ void __launch_bounds__(TAIL_THREADS) tail_adamw_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, const int* __restrict__ blk_seg, const int64_t* __restrict__ blk_lo,
    const int64_t* __restrict__ blk_hi, const float* __restrict__ seg_coef,
    const int* __restrict__ flags, const int* __restrict__ step, double lr, double beta1,
    double beta2, float eps, double weight_decay) {
  if (flags[0]) return;  // main.py:317/402/418 `continue`: no optimizer step
  const int b = blockIdx.x, sgi = blk_seg[b];
  const int64_t lo = blk_lo[b], hi = blk_hi[b];
  const float f1 = seg_coef[4 * sgi + 0], f2 = seg_coef[4 * sgi + 1], c = seg_coef[4 * sgi + 2];
  const bool zero = seg_coef[4 * sgi + 3] != 0.f;
  const double t = (double)step[0];
  const double bc1 = 1.0 - pow(beta1, t), bc2 = 1.0 - pow(beta2, t);
  const float decay = (float)(1.0 - lr * weight_decay);
  const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, w2 = (float)(1.0 - beta2);
  const float step_size = (float)(lr / bc1), bc2s = (float)sqrt(bc2);
  for (int64_t i = lo + threadIdx.x; i < hi; i += TAIL_THREADS) {
    float gi = 0.f;
    if (!zero) gi = ((g[i] * f1) * f2) * c;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i] * b2;
    vi = vi + (w2 * gi) * gi;
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace nsm

using namespace nsm;

// ============================== C ABI ======================================
extern "C" int64_t nsm_tail_chunk(void) { return TAIL_CHUNK; }

extern "C" int nsm_tail_plan(const int64_t* seg_off, int nseg, int* blk_seg, int64_t* blk_lo,
                             int64_t* blk_hi, int* seg_blk, int cap) {
  if (!seg_off || nseg <= 0) return -1;
  int nb = 0;
  for (int s = 0; s < nseg; ++s) {
    if (seg_blk) seg_blk[s] = nb;
    const int64_t a = seg_off[s], e = seg_off[s + 1];
    if (e < a) return -1;
    for (int64_t lo = a; lo < e; lo += TAIL_CHUNK) {
      if (blk_seg && nb < cap) {
        blk_seg[nb] = s;
        blk_lo[nb] = lo;
        blk_hi[nb] = lo + TAIL_CHUNK < e ? lo + TAIL_CHUNK : e;
      }
      ++nb;
    }
  }
  if (seg_blk) seg_blk[nseg] = nb;
  return nb;
}

extern "C" size_t nsm_tail_ws_bytes(int nseg, int nblk) {
  return tail_ws_layout(nseg, nblk, nullptr, nullptr);
}

extern "C" int nsm_grad_tail(float* g, int nseg, const int64_t* seg_off, const int* seg_blk,
                             const int* blk_seg, const int64_t* blk_lo, const int64_t* blk_hi,
                             int nblk, float inv_world, float scale, float max_norm,
                             const float* noise, uint64_t seed, void* ws, size_t ws_bytes,
                             float* seg_coef, float* stat, int* flags, int* step, void* stream) {
  NSM_CHECK_ARG(g && seg_off && seg_blk && blk_seg && blk_lo && blk_hi && ws && seg_coef && stat &&
                    flags && step && nseg > 0 && nblk > 0 && scale > 0.f,
                "grad_tail: bad args");
  NSM_CHECK_ARG(ws_bytes >= nsm_tail_ws_bytes(nseg, nblk), "grad_tail: workspace too small");
  TailWs w;
  tail_ws_layout(nseg, nblk, (char*)ws, &w);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(tail_stats_kernel, dim3(nblk), dim3(TAIL_THREADS), 0, s, g, blk_lo, blk_hi,
                     inv_world, w);
  NSM_LAUNCH_CHECK("tail_stats");
  hipLaunchKernelGGL(tail_decide_kernel, dim3(1), dim3(1024), 0, s, seg_off, seg_blk, nseg, w);
  NSM_LAUNCH_CHECK("tail_decide");
  hipLaunchKernelGGL(tail_repair_kernel, dim3(nblk), dim3(TAIL_THREADS), 0, s, g, blk_seg, blk_lo,
                     blk_hi, noise, seed, step, w);
  NSM_LAUNCH_CHECK("tail_repair");
  hipLaunchKernelGGL(tail_finalize_kernel, dim3(1), dim3(1024), 0, s, seg_blk, nseg, scale,
                     max_norm, w, seg_coef, stat, flags, step);
  NSM_LAUNCH_CHECK("tail_finalize");
  return 0;
}

extern "C" int nsm_adamw_tail(float* p, const float* g, float* m, float* v, const int* blk_seg,
                              const int64_t* blk_lo, const int64_t* blk_hi, int nblk,
                              const float* seg_coef, const int* flags, const int* step, double lr,
                              double beta1, double beta2, double eps, double weight_decay,
                              void* stream) {
  NSM_CHECK_ARG(p && g && m && v && blk_seg && blk_lo && blk_hi && seg_coef && flags && step &&
                    nblk > 0,
                "adamw_tail: bad args");
  hipLaunchKernelGGL(tail_adamw_kernel, dim3(nblk), dim3(TAIL_THREADS), 0, as_stream(stream), p, g,
                     m, v, blk_seg, blk_lo, blk_hi, seg_coef, flags, step, lr, beta1, beta2,
                     (float)eps, weight_decay);
  NSM_LAUNCH_CHECK("adamw_tail");
  return 0;
}
