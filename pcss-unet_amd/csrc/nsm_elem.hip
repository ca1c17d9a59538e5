// Memory-bound kernels of the U-Net hot path on gfx950: BatchNorm statistics /
// apply / backward, LeakyReLU, Dropout2d masks, AvgPool2d, bilinear resampling
// (align_corners=True), pixel (un)shuffle at the model boundary, the conv10 +
// pixel_shuffle + sigmoid head, the L1 / perturbation losses and the AdamW tail.
//
// All activations are NHWC fp32 with a padded channel count C (multiple of 4,
// 32 in practice), so every lane moves float4 (16 B) and a wave moves 1 KiB
// per instruction. Cross-block reductions are deterministic: each block writes
// a partial row, a tiny finalize kernel merges rows in a fixed order (double).
#include <algorithm>

#include "nsm_common.h"

namespace nsm {

// ---------------------------------------------------------------------------
// Streaming layout: every lane moves 8 consecutive channels (F8: one 16-B
// vector of bf16, two of fp32) and all index math is 32-bit with
// multiply-high division (no 64-bit divides in the loops).
// ---------------------------------------------------------------------------
// Column reductions over an [M][C] NHWC matrix: block = 256 threads laid out
// as rl row-lanes x cl 8-channel lanes; grid = (gx channel groups, nchunk).
// ---------------------------------------------------------------------------
static inline int gcd_i(int a, int b) {
  while (b) {
    int t = a % b;
    a = b;
    b = t;
  }
  return a;
}
struct ColRed {
  int cl, rl, gx, nchunk, rpc;
};
static ColRed colred_plan(int M, int C) {
  ColRed r;
  r.cl = gcd_i(C / 8, 64);
  r.rl = 256 / r.cl;
  r.gx = (C / 8) / r.cl;
  long long want = (M + 63) / 64;
  long long cap = 1024 / r.gx;  // ~1024 blocks fill the 256 CUs; finalize stays short
  if (cap < 1) cap = 1;
  r.nchunk = (int)(want < cap ? want : cap);
  if (r.nchunk < 1) r.nchunk = 1;
  r.rpc = ceil_div(M, r.nchunk);
  return r;
}

// reduce red[rl][cl] (F8) over rl; result valid in red[0][tc] for all tc.
__device__ __forceinline__ void col_tree_reduce(F8* red, int cl, int rl, int tid) {
  for (int s = rl / 2; s > 0; s >>= 1) {
    __syncthreads();
    int tr = tid / cl;
    if (tr < s) red[tid] += red[tid + s * cl];
  }
  __syncthreads();
}

__device__ __forceinline__ F8 ldf8(const float* p) { return ld8(p); }  // fp32 parameter vectors

template <typename T>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ y, int ld, int M,
                                                       int C, int cl, int rl, int rpc,
                                                       float* __restrict__ partial) {
  __shared__ F8 red[256];
  const int tid = threadIdx.x, tc = tid % cl, tr = tid / cl;
  const int c = (blockIdx.x * cl + tc) * 8;
  const int r0 = blockIdx.y * rpc, r1 = min(M, r0 + rpc);
  F8 s = f8zero();
#pragma unroll 4
  for (int r = r0 + tr; r < r1; r += rl) s += ld8(y + (size_t)r * ld + c);
  red[tid] = s;
  col_tree_reduce(red, cl, rl, tid);
  const float n = (float)max(r1 - r0, 1);
  const F8 sum = red[tc];
  const F8 mean = (1.f / n) * sum;
  __syncthreads();
  F8 s2 = f8zero();
#pragma unroll 4
  for (int r = r0 + tr; r < r1; r += rl) {
    F8 d = ld8(y + (size_t)r * ld + c) - mean;
    s2 += d * d;
  }
  red[tid] = s2;
  col_tree_reduce(red, cl, rl, tid);
  if (tr == 0) {
    float* pr = partial + (size_t)blockIdx.y * 2 * C;
    st8(pr + c, sum);
    st8(pr + C + c, red[tc]);
  }
}

// Finalize kernels: one wave per channel; lanes stride over the partial rows
// (4 independent accumulators keep several loads in flight), fixed-order
// double reduction with cross-lane butterflies.
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// fixed-order double sum over a 256-thread block (red: 4 doubles of LDS)
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  __syncthreads();  // red may still be read from a previous call
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// One 256-thread block per channel: every partial row of a pass is loaded by
// one lane in one round (the per-wave form took ~nchunk/256 dependent rounds).
__global__ void __launch_bounds__(256) bn_finalize_train_kernel(
    const float* __restrict__ partial, int nchunk, int rpc, int M, int C, int c_real,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* run_mean,
    float* run_var, int64_t* num_batches, float momentum, float eps, int n_updates, float* mean_o,
    float* invstd_o, float* scale_o, float* shift_o, uint32_t* bound, float bound_mul) {
  __shared__ double red[4];
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  if (blockIdx.x == 0 && tid == 0 && num_batches) *num_batches += n_updates;
  // rpc == 0: counted partials [nchunk][3][C] = {sum, M2, count} (the Winograd
  // output transform's slots); else {sum, M2} of rpc-row chunks
  const size_t st = (size_t)(rpc ? 2 : 3) * C;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int k = tid;
  for (; k + 768 < nchunk; k += 1024) {
    s0 += partial[k * st + c];
    s1 += partial[(k + 256) * st + c];
    s2 += partial[(k + 512) * st + c];
    s3 += partial[(k + 768) * st + c];
  }
  for (; k < nchunk; k += 256) s0 += partial[k * st + c];
  const double mean = block_sum_d((s0 + s1) + (s2 + s3), red) / M;
  double q0 = 0.0, q1 = 0.0;
  for (k = tid; k < nchunk; k += 512) {
    int n0 = rpc ? min(M, k * rpc + rpc) - k * rpc : (int)partial[k * st + 2 * C + c];
    if (n0 > 0) {
      double d = partial[k * st + c] / n0 - mean;
      q0 += partial[k * st + C + c] + n0 * d * d;
    }
    int k1 = k + 256;
    if (k1 < nchunk) {
      int n1 = rpc ? min(M, k1 * rpc + rpc) - k1 * rpc : (int)partial[k1 * st + 2 * C + c];
      if (n1 > 0) {
        double d = partial[k1 * st + c] / n1 - mean;
        q1 += partial[k1 * st + C + c] + n1 * d * d;
      }
    }
  }
  const double m2 = block_sum_d(q0 + q1, red);
  if (tid != 0) return;
  const float var_b = (float)(m2 / M);
  const float var_u = M > 1 ? (float)(m2 / (M - 1)) : var_b;
  const float mf = (float)mean;
  const float inv = 1.0f / sqrtf(var_b + eps);
  const float sc = gamma[c] * inv;
  mean_o[c] = mf;
  invstd_o[c] = inv;
  scale_o[c] = sc;
  shift_o[c] = beta[c] - mf * sc;
  if (bound) {
    // max over the batch of |lrelu(y*scale+shift)| * mask_max, the scale source
    // of the h2 activated operand (nsm_bn_act_h2) known before it is written:
    // y*scale + shift = scale (y - mean) + beta and, for n values with biased
    // variance var, max|y - mean| <= sqrt(var (n - 1)) (Samuelson), so
    // |BN(y)| <= |scale| sqrt(var (n - 1)) + |beta|; LeakyReLU does not grow
    // it. In double, 1e-6 up (the fp32 apply rounds within the s headroom).
    const double b = ((double)fabsf(sc) * sqrt((double)var_b * (double)(M - 1)) +
                      (double)fabsf(beta[c])) * (double)bound_mul * (1.0 + 1e-6);
    atomicMax(bound + (c & (AMAX_LINES - 1)) * AMAX_STRIDE, __float_as_uint((float)b) & 0x7fffffffu);
  }
  if (c < c_real && run_mean) {
    float rm = run_mean[c], rv = run_var[c];
    for (int u = 0; u < n_updates; ++u) {
      rm = momentum * mf + (1.f - momentum) * rm;
      rv = momentum * var_u + (1.f - momentum) * rv;
    }
    run_mean[c] = rm;
    run_var[c] = rv;
  }
}

// First level of the BN-partial merge for grids with many row chunks:
// out[g] = Chan merge of chunks [g*G, (g+1)*G) (fixed order, double), one
// thread per (group, channel), coalesced along channels.
// rpc == 0: counted rows in and out ({sum, M2, count}, stride 3C)
__global__ void bn_partials_merge_kernel(const float* __restrict__ partial, int nchunk, int rpc,
                                         int M, int C, int G, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (c >= C) return;
  const size_t st = (size_t)(rpc ? 2 : 3) * C;
  const int k0 = g * G, k1 = min(nchunk, k0 + G);
  double s = 0.0;
  long long n = 0;
  for (int k = k0; k < k1; ++k) {
    s += partial[(size_t)k * st + c];
    n += rpc ? max(0, min(M, (k + 1) * rpc) - k * rpc) : (long long)partial[(size_t)k * st + 2 * C + c];
  }
  const double mean = n > 0 ? s / (double)n : 0.0;
  double m2 = 0.0;
  for (int k = k0; k < k1; ++k) {
    const int nk = rpc ? min(M, (k + 1) * rpc) - k * rpc : (int)partial[(size_t)k * st + 2 * C + c];
    if (nk <= 0) continue;
    const double d = partial[(size_t)k * st + c] / nk - mean;
    m2 += partial[(size_t)k * st + C + c] + nk * d * d;
  }
  out[(size_t)g * st + c] = (float)s;
  out[(size_t)g * st + C + c] = (float)m2;
  if (!rpc) out[(size_t)g * st + 2 * C + c] = (float)n;
}

// Plain-sum merge of partial rows (the BN-backward {sum dz, sum dz*xhat}
// format): out[g][j] = sum over rows [g*G, (g+1)*G) of part[.][j], fixed
// order, one thread per column (coalesced along the row)
__global__ void sum_rows_kernel(const float* __restrict__ part, int nrows, int width, int G,
                                float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
  if (j >= width) return;
  const int k0 = g * G, k1 = min(nrows, k0 + G);
  double s = 0.0, s1 = 0.0;  // two rows' loads in flight, fixed order
  int k = k0;
  for (; k + 1 < k1; k += 2) {
    s += part[(size_t)k * width + j];
    s1 += part[(size_t)(k + 1) * width + j];
  }
  if (k < k1) s += part[(size_t)k * width + j];
  out[(size_t)g * width + j] = (float)(s + s1);
}

__global__ void bn_finalize_eval_kernel(const float* __restrict__ rm, const float* __restrict__ rv,
                                        const float* __restrict__ gamma,
                                        const float* __restrict__ beta, int C, int c_real, float eps,
                                        float* mean_o, float* invstd_o, float* scale_o,
                                        float* shift_o) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float m = c < c_real ? rm[c] : 0.f;
  float v = c < c_real ? rv[c] : 1.f;
  float inv = 1.0f / sqrtf(v + eps);
  float sc = gamma[c] * inv;
  mean_o[c] = m;
  invstd_o[c] = inv;
  scale_o[c] = sc;
  shift_o[c] = beta[c] - m * sc;
}

__device__ __forceinline__ f32x4 lrelu4(f32x4 v, float slope) {
  return f32x4{lrelu(v.x, slope), lrelu(v.y, slope), lrelu(v.z, slope), lrelu(v.w, slope)};
}
__device__ __forceinline__ F8 lrelu8(F8 v, float slope) {
  return F8{lrelu4(v.a, slope), lrelu4(v.b, slope)};
}

// Pixel-row streaming (bn_act, bn_bwd_apply): a block covers whole pixels
// (blockDim = k*C8, pix_launch), so each lane keeps ONE 8-channel group for
// the whole grid-stride loop and its per-channel vectors stay in registers.
//
// out = lrelu(y*scale+shift) (* mask[b][c]) (+ res)
template <typename T>
__global__ void __launch_bounds__(256) bn_act_kernel(const T* __restrict__ y, int ldy, int M,
                                                     int C8, FastDiv fdHW,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift, float slope,
                                                     const float* __restrict__ mask,
                                                     const T* __restrict__ res, int ldres,
                                                     T* __restrict__ out, int ldo,
                                                     uint32_t* __restrict__ amax) {
  const int ppb = blockDim.x / C8, tp = threadIdx.x / C8;
  const int c = (threadIdx.x - tp * C8) * 8;
  const F8 sc = ldf8(scale + c), sh = ldf8(shift + c);
  const int pstep = gridDim.x * ppb;
  uint32_t am = 0;  // max|out| (an f16x2 GEMM operand scale, fp32 only)
  for (int p = blockIdx.x * ppb + tp; p < M; p += pstep) {
    F8 o = lrelu8(ld8(y + (size_t)p * ldy + c) * sc + sh, slope);
    // Dropout2d after the LeakyReLU (Unetmodel.py:23-24)
    if (mask) o = o * ld8(mask + (size_t)fdiv((uint32_t)p, fdHW) * (C8 * 8) + c);
    if (res) o += ld8(res + (size_t)p * ldres + c);
    st8(out + (size_t)p * ldo + c, o);
    if (amax) {
      amax_fold(am, o.a);
      amax_fold(am, o.b);
    }
  }
  amax_flush(am, amax);
}

// bn_act's activated operand written as an h2 tensor out [M][2C] (fp32 in):
// the 1x1 conv's A1 (nsm_conv_h2d.inc), scale from the bound slot its BN
// finalize filled (nsm_bn_finalize_train `bound`)
__global__ void __launch_bounds__(256) bn_act_h2_kernel(const float* __restrict__ y, int ldy, int M,
                                                        int C8, FastDiv fdHW,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        float slope,
                                                        const float* __restrict__ mask,
                                                        bf16_t* __restrict__ out, H2Scale hs) {
  const float s = exp2i(h2_exp(hs));  // every lane: amax_read is a wave reduction
  const int ppb = blockDim.x / C8, tp = threadIdx.x / C8;
  const int c = (threadIdx.x - tp * C8) * 8;
  const F8 sc = ldf8(scale + c), sh = ldf8(shift + c);
  const int pstep = gridDim.x * ppb;
  for (int p = blockIdx.x * ppb + tp; p < M; p += pstep) {
    F8 o = lrelu8(ld8(y + (size_t)p * ldy + c) * sc + sh, slope);
    if (mask) o = o * ld8(mask + (size_t)fdiv((uint32_t)p, fdHW) * (C8 * 8) + c);
    h2_store8(out + (size_t)p * 16 * C8, c, o, s);
  }
}

// dz = g * mask[b][c] * lrelu'(y*scale+shift)
__device__ __forceinline__ f32x4 lrelu_grad4(f32x4 z, float slope) {
  return f32x4{lrelu_grad(z.x, slope), lrelu_grad(z.y, slope), lrelu_grad(z.z, slope),
               lrelu_grad(z.w, slope)};
}
__device__ __forceinline__ F8 bn_dz8(const F8 g, const F8 v, const F8 sc, const F8 sh,
                                     float slope, const float* mask, int b, int C, int c) {
  const F8 z = v * sc + sh;
  F8 d{g.a * lrelu_grad4(z.a, slope), g.b * lrelu_grad4(z.b, slope)};
  // Dropout2d sits AFTER the LeakyReLU (Unetmodel.py:23-24): d(out)/d(z) =
  // mask * lrelu'(z); multiplication order does not matter for the value.
  if (mask) d = d * ld8(mask + (size_t)b * C + c);
  return d;
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(
    const T* __restrict__ g, int ldg, const T* __restrict__ y, int ldy, int M, int C,
    FastDiv fdHW, const float* __restrict__ scale, const float* __restrict__ shift, float slope,
    const float* __restrict__ mask, const float* __restrict__ mean,
    const float* __restrict__ invstd, int cl, int rl, int rpc, float* __restrict__ partial,
    uint32_t* __restrict__ amax) {
  __shared__ F8 red[256];
  const int tid = threadIdx.x, tc = tid % cl, tr = tid / cl;
  const int c = (blockIdx.x * cl + tc) * 8;
  const int r0 = blockIdx.y * rpc, r1 = min(M, r0 + rpc);
  const F8 sc = ldf8(scale + c), sh = ldf8(shift + c);
  const F8 mu = ldf8(mean + c), is = ldf8(invstd + c);
  F8 s1 = f8zero(), s2 = f8zero();
  uint32_t am = 0;  // max|scale * dz| (scale = gamma * invstd = k1 of the finalize)
#pragma unroll 2
  for (int r = r0 + tr; r < r1; r += rl) {
    const F8 v = ld8(y + (size_t)r * ldy + c);
    const F8 gg = ld8(g + (size_t)r * ldg + c);
    const int b = mask ? (int)fdiv((uint32_t)r, fdHW) : 0;
    const F8 dz = bn_dz8(gg, v, sc, sh, slope, mask, b, C, c);
    s1 += dz;
    s2 += dz * ((v - mu) * is);
    if (amax) {
      amax_fold(am, sc.a * dz.a);
      amax_fold(am, sc.b * dz.b);
    }
  }
  amax_flush(am, amax);
  red[tid] = s1;
  col_tree_reduce(red, cl, rl, tid);
  const F8 t1 = red[tc];
  __syncthreads();
  red[tid] = s2;
  col_tree_reduce(red, cl, rl, tid);
  if (tr == 0) {
    float* pr = partial + (size_t)blockIdx.y * 2 * C;
    st8(pr + c, t1);
    st8(pr + C + c, red[tc]);
  }
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(
    const float* __restrict__ partial, int nchunk, int M, int C, int c_real,
    const float* __restrict__ gamma, const float* __restrict__ invstd, float* dgamma,
    float* dbeta, float* dbias_prev, float* coef, const uint32_t* __restrict__ amax_k1dz,
    uint32_t* __restrict__ bound) {
  __shared__ double red[4];
  const int tid = threadIdx.x;
  const int c = blockIdx.x;  // one block per channel (see bn_finalize_train_kernel)
  // max over the tensor of |k1 dz| (recorded by the reduction's producer): every
  // lane of the block's waves (amax_read is a wave reduction)
  const float a_k1dz = bound ? __uint_as_float(amax_read(amax_k1dz)) : 0.f;
  const size_t st = (size_t)2 * C;
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
  int k = tid;
  for (; k + 256 < nchunk; k += 512) {
    a0 += partial[k * st + c];
    b0 += partial[k * st + C + c];
    a1 += partial[(k + 256) * st + c];
    b1 += partial[(k + 256) * st + C + c];
  }
  for (; k < nchunk; k += 256) {
    a0 += partial[k * st + c];
    b0 += partial[k * st + C + c];
  }
  const double S1 = block_sum_d(a0 + a1, red), S2 = block_sum_d(b0 + b1, red);
  if (tid != 0) return;
  const float gm = gamma[c], is = invstd[c];
  const double mdz = S1 / M, mdzx = S2 / M;
  const float k1 = gm * is;
  const float k2 = (float)(-(double)gm * is * is * mdzx);
  const float k3 = (float)(-(double)k1 * mdz);
  coef[c] = k1;
  coef[C + c] = k2;
  coef[2 * C + c] = k3;
  if (bound) {
    // dy = k1 dz + k2 (y - mean) + k3 with max|y - mean| <= sqrt(var (M - 1))
    // <= sqrt(M - 1) / invstd (Samuelson, biased var): a bound of max|dy| known
    // before nsm_bn_bwd_apply_h2 writes dy, the scale source of that h2 tensor
    const double b = ((double)a_k1dz + fabs((double)k2) * sqrt((double)(M - 1)) / (double)is +
                      fabs((double)k3)) * (1.0 + 1e-6);
    atomicMax(bound + (c & (AMAX_LINES - 1)) * AMAX_STRIDE, __float_as_uint((float)b) & 0x7fffffffu);
  }
  if (c < c_real) {
    if (dgamma) dgamma[c] = (float)S2;
    if (dbeta) dbeta[c] = (float)S1;
    // sum_p dy = k1*S1 + k2*sum(y-mean) + k3*M == 0 analytically (pre-BN bias)
    if (dbias_prev) dbias_prev[c] = (float)((double)k1 * S1 + (double)k3 * M);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const T* __restrict__ g, int ldg, const T* __restrict__ y, int ldy, int M, int C, int C8,
    FastDiv fdHW, const float* __restrict__ scale, const float* __restrict__ shift, float slope,
    const float* __restrict__ mask, const float* __restrict__ mean,
    const float* __restrict__ coef, T* __restrict__ dy, int lddy, uint32_t* __restrict__ amax) {
  const int ppb = blockDim.x / C8, tp = threadIdx.x / C8;
  const int c = (threadIdx.x - tp * C8) * 8;
  const F8 sc = ldf8(scale + c), sh = ldf8(shift + c), mu = ldf8(mean + c);
  const F8 k1 = ldf8(coef + c), k2 = ldf8(coef + C + c), k3 = ldf8(coef + 2 * C + c);
  const int pstep = gridDim.x * ppb;
  uint32_t am = 0;  // max|dy| (an f16x2 GEMM operand scale, fp32 only)
  for (int p = blockIdx.x * ppb + tp; p < M; p += pstep) {
    const F8 v = ld8(y + (size_t)p * ldy + c);
    const F8 gg = ld8(g + (size_t)p * ldg + c);
    const int b = mask ? (int)fdiv((uint32_t)p, fdHW) : 0;
    const F8 dz = bn_dz8(gg, v, sc, sh, slope, mask, b, C, c);
    const F8 d = k1 * dz + k2 * (v - mu) + k3;
    st8(dy + (size_t)p * lddy + c, d);
    if (amax) {
      amax_fold(am, d.a);
      amax_fold(am, d.b);
    }
  }
  amax_flush(am, amax);
}

// nsm_bn_bwd_apply (fp32) writing dy as an h2 tensor [M][2C] with the scale
// source `bound` (nsm_bn_bwd_finalize's): the 1x1 conv's output gradient dY2
// read by its h2 weight and input gradients (nsm_conv_h2d.inc)
__global__ void __launch_bounds__(256) bn_bwd_apply_h2_kernel(
    const float* __restrict__ g, int ldg, const float* __restrict__ y, int ldy, int M, int C,
    int C8, FastDiv fdHW, const float* __restrict__ scale, const float* __restrict__ shift,
    float slope, const float* __restrict__ mask, const float* __restrict__ mean,
    const float* __restrict__ coef, bf16_t* __restrict__ dy, H2Scale hs) {
  const float s = exp2i(h2_exp(hs));  // every lane: amax_read is a wave reduction
  const int ppb = blockDim.x / C8, tp = threadIdx.x / C8;
  const int c = (threadIdx.x - tp * C8) * 8;
  const F8 sc = ldf8(scale + c), sh = ldf8(shift + c), mu = ldf8(mean + c);
  const F8 k1 = ldf8(coef + c), k2 = ldf8(coef + C + c), k3 = ldf8(coef + 2 * C + c);
  const int pstep = gridDim.x * ppb;
  for (int p = blockIdx.x * ppb + tp; p < M; p += pstep) {
    const F8 v = ld8(y + (size_t)p * ldy + c);
    const F8 gg = ld8(g + (size_t)p * ldg + c);
    const int b = mask ? (int)fdiv((uint32_t)p, fdHW) : 0;
    const F8 dz = bn_dz8(gg, v, sc, sh, slope, mask, b, C, c);
    h2_store8(dy + (size_t)p * 2 * C, c, k1 * dz + k2 * (v - mu) + k3, s);
  }
}

// BN-backward reduction fused into the kernel that PRODUCES a block output's
// gradient g (the pooling / resize backward): with y = that block's BN input
// Y2, {sum dz, sum dz*xhat} per channel of dz = g * lrelu'(y*scale+shift)
// (no dropout after the second BN, Unetmodel.py:27-28), summed over the
// kernel's block and written as partial row blockIdx.x of [gridDim.x][2][C]
// (the nsm_bn_bwd_reduce format) — the separate reduce pass and its read of g
// are gone. Each thread keeps ONE 8-channel group (C/8 divides 256).
struct BnRedP {
  const void* y;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* invstd;
  float slope;
  float* partial;
  uint32_t* amax;  // max|scale * dz| (may be NULL): the k1 term of the dy bound (finalize)
};
template <typename T>
__device__ __forceinline__ F8 as_stored8(F8 v);
template <>
__device__ __forceinline__ F8 as_stored8<float>(F8 v) { return v; }
template <>
__device__ __forceinline__ F8 as_stored8<f16_t>(F8 v) {
  const u32x4 w = u32x4{pack_hh(v.a.x, v.a.y), pack_hh(v.a.z, v.a.w), pack_hh(v.b.x, v.b.y),
                        pack_hh(v.b.z, v.b.w)};
  return F8{f32x4{h_lo(w.x), h_hi(w.x), h_lo(w.y), h_hi(w.y)},
            f32x4{h_lo(w.z), h_hi(w.z), h_lo(w.w), h_hi(w.w)}};
}
template <>
__device__ __forceinline__ F8 as_stored8<bf16_t>(F8 v) {
  const u32x4 w = u32x4{pack_bf2(v.a.x, v.a.y), pack_bf2(v.a.z, v.a.w), pack_bf2(v.b.x, v.b.y),
                        pack_bf2(v.b.z, v.b.w)};
  return F8{f32x4{bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)},
            f32x4{bf_lo(w.z), bf_hi(w.z), bf_lo(w.w), bf_hi(w.w)}};
}
struct BnRedAcc {
  F8 sc, sh, mu, is, s1, s2;
  uint32_t am;
  __device__ void init(const BnRedP& r, int c) {
    sc = ldf8(r.scale + c);
    sh = ldf8(r.shift + c);
    mu = ldf8(r.mean + c);
    is = ldf8(r.invstd + c);
    s1 = f8zero();
    s2 = f8zero();
    am = 0;
  }
  // g: the value as written (T-rounded); p: its pixel row in y
  template <typename T>
  __device__ void add(const BnRedP& r, F8 g, size_t p, int C, int c) {
    const F8 v = ld8((const T*)r.y + p * C + c);
    const F8 dz = bn_dz8(g, v, sc, sh, r.slope, nullptr, 0, C, c);
    s1 += dz;
    s2 += dz * ((v - mu) * is);
    if (r.amax) {
      amax_fold(am, sc.a * dz.a);
      amax_fold(am, sc.b * dz.b);
    }
  }
  // whole block (256 threads, group = tid % C8) -> partial row blockIdx.x
  __device__ void write(const BnRedP& r, int C8) {
    __shared__ F8 red[256];
    const int tid = threadIdx.x, rl = 256 / C8, tc = tid % C8, C = C8 * 8;
    red[tid] = s1;
    col_tree_reduce(red, C8, rl, tid);
    const F8 t1 = red[tc];
    __syncthreads();
    red[tid] = s2;
    col_tree_reduce(red, C8, rl, tid);
    if (tid < C8) {
      float* pr = r.partial + (size_t)blockIdx.x * 2 * C;
      st8(pr + tc * 8, t1);
      st8(pr + C + tc * 8, red[tc]);
    }
    amax_flush(am, r.amax);
  }
  // a block covering channels [c0, c0 + 8 G) of a C-channel tensor (group =
  // tid % G): its slice of partial row `row`
  __device__ void write_slice(const BnRedP& r, int G, int c0, int C, int row) {
    __shared__ F8 red[256];
    const int tid = threadIdx.x, rl = 256 / G, tc = tid % G;
    red[tid] = s1;
    col_tree_reduce(red, G, rl, tid);
    const F8 t1 = red[tc];
    __syncthreads();
    red[tid] = s2;
    col_tree_reduce(red, G, rl, tid);
    if (tid < G) {
      float* pr = r.partial + (size_t)row * 2 * C + c0;
      st8(pr + tc * 8, t1);
      st8(pr + C + tc * 8, red[tc]);
    }
    amax_flush(am, r.amax);
  }
};

// ---------------------------------------------------------------------------
// AvgPool2d(2), floor mode
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) avgpool2_fwd_kernel(const T* __restrict__ x, int B, int H,
                                                           int W, int C8, FastDiv fdC8,
                                                           FastDiv fdWo, FastDiv fdHo,
                                                           T* __restrict__ y) {
  const int Ho = H / 2, Wo = W / 2, C = C8 * 8;
  const uint32_t total = (uint32_t)B * Ho * Wo * C8;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t p = fdiv(i, fdC8);
    const int c = (int)(i - p * (uint32_t)C8) * 8;
    const uint32_t t = fdiv(p, fdWo);
    const int ox = (int)(p - t * Wo);
    const uint32_t b = fdiv(t, fdHo);
    const int oy = (int)(t - b * Ho);
    const T* base = x + (((size_t)b * H + 2 * oy) * W + 2 * ox) * C + c;
    const size_t rs = (size_t)W * C;
    F8 s = ld8(base);
    s += ld8(base + C);
    s += ld8(base + rs);
    s += ld8(base + rs + C);
    st8(y + (size_t)p * C + c, 0.25f * s);
  }
}

// The encoder block output z = lrelu(bn2(Y2)) (Unetmodel.py:27-28) and its
// AvgPool2d(2) (:105,108,111) from one read of Y2: each thread takes a 2x2
// pixel quad (ceil grid, so odd rows / columns still get their z) of one
// 8-channel group, writes the quad's z (the skip tensor) and, inside the floor
// grid, their mean from the stored values (as avgpool2_fwd would read them).
template <typename T>
__global__ void __launch_bounds__(256) bn_act_pool_kernel(const T* __restrict__ y, int B, int H,
                                                          int W, int C8, FastDiv fdC8,
                                                          FastDiv fdWc, FastDiv fdHc,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          float slope, T* __restrict__ z,
                                                          T* __restrict__ pooled,
                                                          uint32_t* __restrict__ amax) {
  const int Hc = (H + 1) / 2, Wc = (W + 1) / 2, Ho = H / 2, Wo = W / 2, C = C8 * 8;
  uint32_t am = 0;  // max|pooled| (the next Winograd conv's h2 scale source)
  const uint32_t total = (uint32_t)B * Hc * Wc * C8;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t p = fdiv(i, fdC8);
    const int c = (int)(i - p * (uint32_t)C8) * 8;
    const uint32_t t = fdiv(p, fdWc);
    const int cx = (int)(p - t * Wc);
    const uint32_t b = fdiv(t, fdHc);
    const int cy = (int)(t - b * Hc);
    const F8 sc = ldf8(scale + c), sh = ldf8(shift + c);
    F8 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int yy = 2 * cy + (k >> 1), xx = 2 * cx + (k & 1);
      q[k] = f8zero();
      if (yy < H && xx < W) {
        const size_t off = (((size_t)b * H + yy) * W + xx) * C + c;
        q[k] = as_stored8<T>(lrelu8(ld8(y + off) * sc + sh, slope));
        st8(z + off, q[k]);
      }
    }
    if (cy < Ho && cx < Wo) {
      F8 sum = q[0];
      sum += q[1];
      sum += q[2];
      sum += q[3];
      const F8 pv = 0.25f * sum;
      st8(pooled + (((size_t)b * Ho + cy) * Wo + cx) * C + c, pv);
      if (amax) {
        amax_fold(am, pv.a);
        amax_fold(am, pv.b);
      }
    }
  }
  amax_flush(am, amax);
}

template <typename T, bool RED>
__global__ void __launch_bounds__(256) avgpool2_bwd_add_kernel(const T* __restrict__ dy, int B,
                                                               int H, int W, int C8, FastDiv fdC8,
                                                               FastDiv fdW, FastDiv fdH,
                                                               const T* __restrict__ skip,
                                                               T* __restrict__ dx, BnRedP rp) {
  const int Ho = H / 2, Wo = W / 2, C = C8 * 8;
  const uint32_t total = (uint32_t)B * H * W * C8;
  BnRedAcc ra;
  if (RED) ra.init(rp, (threadIdx.x % C8) * 8);
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t p = fdiv(i, fdC8);
    const int c = (int)(i - p * (uint32_t)C8) * 8;
    const uint32_t t = fdiv(p, fdW);
    const int xx = (int)(p - t * W);
    const uint32_t b = fdiv(t, fdH);
    const int yy = (int)(t - b * H);
    F8 v = skip ? ld8(skip + (size_t)p * C + c) : f8zero();
    const int oy = yy >> 1, ox = xx >> 1;
    if (oy < Ho && ox < Wo) v += 0.25f * ld8(dy + (((size_t)b * Ho + oy) * Wo + ox) * C + c);
    st8(dx + (size_t)p * C + c, v);
    if (RED) ra.add<T>(rp, as_stored8<T>(v), p, C, c);
  }
  if (RED) ra.write(rp, C8);
}

// ---------------------------------------------------------------------------
// Bilinear resize, align_corners=True (ATen upsample_bilinear2d semantics:
// scale=(in-1)/(out-1) in fp32, src=scale*dst, i0=floor, i1=i0+(i0<in-1),
// l1=src-i0, l0=1-l1).
// ---------------------------------------------------------------------------
// lin_idx / ac_scale: nsm_common.h

// (pixel, 8-channel group) of a flat index over [B][H][W][C8] (32-bit fast division)
struct Pix8 {
  int b, y, x, c;
};
__device__ __forceinline__ Pix8 pix8(uint32_t i, int C8, int H, int W, const FastDiv& fdC8,
                                     const FastDiv& fdW, const FastDiv& fdH, uint32_t& p) {
  Pix8 r;
  p = fdiv(i, fdC8);
  r.c = (int)(i - p * (uint32_t)C8) * 8;
  const uint32_t t = fdiv(p, fdW);
  r.x = (int)(p - t * (uint32_t)W);
  const uint32_t b = fdiv(t, fdH);
  r.y = (int)(t - b * (uint32_t)H);
  r.b = (int)b;
  return r;
}

// XCD-local block order for the resampling gathers: consecutive blocks are
// dispatched round-robin over the 8 XCDs (separate L2s); renumber so each XCD
// sweeps a contiguous slice of every grid-stride window and the rows its
// neighbours share stay in its own L2 (grid % 8 == 0, see xcd_grid)
__device__ __forceinline__ uint32_t xcd_block() {
  const uint32_t per = gridDim.x >> 3;
  return (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
}

// 8 channels (one 16-B bf16 vector / two fp32 vectors) per lane: the model's
// activations (C % 8 == 0)
// ACT ("act on load"): the source is not materialised — every tap is the
// decoder block output z = lrelu(Y2*scale+shift) (+ skip), rounded as bn_act
// stores it (Unetmodel.py:27-28,125-137 then :122-141's upsample), so z is
// never written or re-read. ActSrc carries Y2's BN vectors and the skip.
struct ActSrc {
  const float* scale;
  const float* shift;
  const void* res;
  float slope;
};
template <typename T, bool ACT>
__device__ __forceinline__ F8 src8(const T* x, size_t off, const ActSrc& a, int c) {
  if constexpr (!ACT) {
    return ld8(x + off);
  } else {
    F8 o = lrelu8(ld8(x + off) * ldf8(a.scale + c) + ldf8(a.shift + c), a.slope);
    if (a.res) o += ld8((const T*)a.res + off);
    return as_stored8<T>(o);
  }
}

template <typename T, bool ACT = false>
__global__ void __launch_bounds__(256) resize_fwd8_kernel(const T* __restrict__ x, int Hi, int Wi,
                                                          int C8, uint32_t total, FastDiv fdC8,
                                                          FastDiv fdWo, FastDiv fdHo,
                                                          T* __restrict__ y, int Ho, int Wo,
                                                          float sh, float sw,
                                                          ActSrc act = ActSrc{}) {
  const int C = C8 * 8;
  for (uint32_t i = xcd_block() * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t p;
    const Pix8 q = pix8(i, C8, Ho, Wo, fdC8, fdWo, fdHo, p);
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    lin_idx(sh, q.y, Hi, y0, y1, ly0, ly1);
    lin_idx(sw, q.x, Wi, x0, x1, lx0, lx1);
    const size_t rb = (size_t)q.b * Hi;
    const size_t r0 = (rb + y0) * Wi * C + q.c, r1 = (rb + y1) * Wi * C + q.c;
    const F8 v = ly0 * (lx0 * src8<T, ACT>(x, r0 + x0 * C, act, q.c) +
                        lx1 * src8<T, ACT>(x, r0 + x1 * C, act, q.c)) +
                 ly1 * (lx0 * src8<T, ACT>(x, r1 + x0 * C, act, q.c) +
                        lx1 * src8<T, ACT>(x, r1 + x1 * C, act, q.c));
    st8(y + (size_t)p * C + q.c, v);
  }
}

// any C: the odd-size input guard (Unetmodel.py:94-97) runs on [B*C][H][W][1]
template <typename T>
__global__ void resize_fwd1_kernel(const T* __restrict__ x, int B, int Hi, int Wi, int C,
                                   T* __restrict__ y, int Ho, int Wo, float sh, float sw) {
  long long total = (long long)B * Ho * Wo * C;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < total; i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long long t = i / C;
    int ox = (int)(t % Wo);
    t /= Wo;
    int oy = (int)(t % Ho);
    int b = (int)(t / Ho);
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    lin_idx(sh, oy, Hi, y0, y1, ly0, ly1);
    lin_idx(sw, ox, Wi, x0, x1, lx0, lx1);
    const size_t rb = (size_t)b * Hi;
    float v = ly0 * (lx0 * ld1(x + ((rb + y0) * Wi + x0) * C + c) +
                     lx1 * ld1(x + ((rb + y0) * Wi + x1) * C + c)) +
              ly1 * (lx0 * ld1(x + ((rb + y1) * Wi + x0) * C + c) +
                     lx1 * ld1(x + ((rb + y1) * Wi + x1) * C + c));
    st1(y + i, v);
  }
}

// weight of output index `o` on input index `i` (0 if none)
__device__ __forceinline__ float lin_w(float scale, int o, int in, int i) {
  int i0, i1;
  float l0, l1;
  lin_idx(scale, o, in, i0, i1, l0, l1);
  return (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
}

__device__ __forceinline__ void cand_range(float scale, int i, int out, int& lo, int& hi) {
  if (scale <= 0.f) {
    lo = 0;
    hi = out - 1;
    return;
  }
  lo = max(0, (int)floorf((float)(i - 1) / scale) - 1);
  hi = min(out - 1, (int)ceilf((float)(i + 1) / scale) + 1);
}

// The backward gathers: per axis, the candidate window is trimmed to the
// outputs with a non-zero weight (4-5 for a x2 upsample); the x weights and
// clamped column indices of a lane sit in fully unrolled register arrays, and
// each output row's loads are issued together, unconditionally, so a row costs
// one memory latency (a load under a per-lane branch would wait alone). Zero
// weights are skipped by select, exactly as a skipped term. Wider windows
// (strong downsizing) take the plain loop.
constexpr int RS_W = 6;

template <typename WF>
__device__ __forceinline__ void trim_range(int& lo, int& hi, WF w) {
  while (lo < hi && w(lo) == 0.f) ++lo;
  while (hi > lo && w(hi) == 0.f) --hi;
}

template <typename T>
__device__ __forceinline__ void gather_row(F8& acc, const T* __restrict__ row, int C, float wy,
                                           const float (&wx)[RS_W], const int (&xo)[RS_W]) {
  F8 v[RS_W];
#pragma unroll
  for (int k = 0; k < RS_W; ++k) v[k] = ld8(row + (size_t)xo[k] * C);
#pragma unroll
  for (int k = 0; k < RS_W; ++k) {
    const float w = wy * wx[k];
    const F8 t = acc + w * v[k];
    acc.a = wx[k] != 0.f ? t.a : acc.a;
    acc.b = wx[k] != 0.f ? t.b : acc.b;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) resize_bwd8_kernel(const T* __restrict__ dy, int Hi, int Wi,
                                                          int C8, uint32_t total, FastDiv fdC8,
                                                          FastDiv fdWi, FastDiv fdHi,
                                                          T* __restrict__ dx, int Ho, int Wo,
                                                          float sh, float sw) {
  const int C = C8 * 8;
  for (uint32_t i = xcd_block() * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t p;
    const Pix8 q = pix8(i, C8, Hi, Wi, fdC8, fdWi, fdHi, p);
    int ylo, yhi, xlo, xhi;
    cand_range(sh, q.y, Ho, ylo, yhi);
    cand_range(sw, q.x, Wo, xlo, xhi);
    trim_range(ylo, yhi, [&](int o) { return lin_w(sh, o, Hi, q.y); });
    trim_range(xlo, xhi, [&](int o) { return lin_w(sw, o, Wi, q.x); });
    const T* base = dy + (size_t)q.b * Ho * Wo * C + q.c;
    F8 acc = f8zero();
    if (xhi - xlo < RS_W) {
      float wx[RS_W];
      int xo[RS_W];
#pragma unroll
      for (int k = 0; k < RS_W; ++k) {
        xo[k] = min(xlo + k, xhi);
        wx[k] = xlo + k <= xhi ? lin_w(sw, xlo + k, Wi, q.x) : 0.f;
      }
      for (int oy = ylo; oy <= yhi; ++oy) {
        const float wy = lin_w(sh, oy, Hi, q.y);
        if (wy != 0.f) gather_row(acc, base + (size_t)oy * Wo * C, C, wy, wx, xo);
      }
    } else {
      for (int oy = ylo; oy <= yhi; ++oy) {
        const float wy = lin_w(sh, oy, Hi, q.y);
        if (wy == 0.f) continue;
        const T* row = base + (size_t)oy * Wo * C;
        for (int ox = xlo; ox <= xhi; ++ox) {
          const float w = lin_w(sw, ox, Wi, q.x);
          if (w != 0.f) acc += (wy * w) * ld8(row + (size_t)ox * C);
        }
      }
    }
    st8(dx + (size_t)p * C + q.c, acc);
  }
}

template <typename T>
__global__ void resize_bwd1_kernel(const T* __restrict__ dy, int B, int Hi, int Wi, int C,
                                   T* __restrict__ dx, int Ho, int Wo, float sh, float sw) {
  long long total = (long long)B * Hi * Wi * C;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < total; i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long long t = i / C;
    int ix = (int)(t % Wi);
    t /= Wi;
    int iy = (int)(t % Hi);
    int b = (int)(t / Hi);
    int ylo, yhi, xlo, xhi;
    cand_range(sh, iy, Ho, ylo, yhi);
    cand_range(sw, ix, Wo, xlo, xhi);
    float acc = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      const float wy = lin_w(sh, oy, Hi, iy);
      if (wy == 0.f) continue;
      const T* row = dy + ((size_t)b * Ho + oy) * Wo * C;
      for (int ox = xlo; ox <= xhi; ++ox) {
        const float w = lin_w(sw, ox, Wi, ix);
        if (w != 0.f) acc += (wy * w) * ld1(row + (size_t)ox * C + c);
      }
    }
    st1(dx + i, acc);
  }
}

// ---------------------------------------------------------------------------
// Composite: nn.Upsample(x2) to (2h,2w) followed by _upsample_and_match to
// (th,tw) (Unetmodel.py:140-141, the up9 "blur"), without materialising the
// 4x intermediate. The row-blocked forward (used for rows up to U2_MAXW)
// applies the separable combined weights as a 3x3 stencil; the per-element
// fallback evaluates the intermediate samples as the two-step path rounds
// them (fp32 per sample). Backward uses the combined weights
// W[o->i] = sum_m w2(o->m) w1(m->i).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ F8 up_sample8(const T* __restrict__ x, size_t rb, int h, int w, int C,
                                         int c, float s1h, float s1w, int my, int mx) {
  int y0, y1, x0, x1;
  float a0, a1, b0, b1;
  lin_idx(s1h, my, h, y0, y1, a0, a1);
  lin_idx(s1w, mx, w, x0, x1, b0, b1);
  const T* r0 = x + (rb + y0) * w * C + c;
  const T* r1 = x + (rb + y1) * w * C + c;
  return a0 * (b0 * ld8(r0 + x0 * C) + b1 * ld8(r0 + x1 * C)) +
         a1 * (b0 * ld8(r1 + x0 * C) + b1 * ld8(r1 + x1 * C));
}

template <typename T>
__global__ void __launch_bounds__(256) up2_resize_fwd8_kernel(const T* __restrict__ x, int h, int w,
                                                              int C8, uint32_t total,
                                                              FastDiv fdC8, FastDiv fdtw,
                                                              FastDiv fdth, T* __restrict__ y,
                                                              int th, int tw, float s1h, float s1w,
                                                              float s2h, float s2w) {
  const int C = C8 * 8, h2 = 2 * h, w2 = 2 * w;
  for (uint32_t i = xcd_block() * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t p;
    const Pix8 q = pix8(i, C8, th, tw, fdC8, fdtw, fdth, p);
    int m0, m1, n0, n1;
    float l0, l1, k0, k1;
    lin_idx(s2h, q.y, h2, m0, m1, l0, l1);
    lin_idx(s2w, q.x, w2, n0, n1, k0, k1);
    const size_t rb = (size_t)q.b * h;
    const F8 u00 = up_sample8(x, rb, h, w, C, q.c, s1h, s1w, m0, n0);
    const F8 u01 = up_sample8(x, rb, h, w, C, q.c, s1h, s1w, m0, n1);
    const F8 u10 = up_sample8(x, rb, h, w, C, q.c, s1h, s1w, m1, n0);
    const F8 u11 = up_sample8(x, rb, h, w, C, q.c, s1h, s1w, m1, n1);
    st8(y + (size_t)p * C + q.c, l0 * (k0 * u00 + k1 * u01) + l1 * (k0 * u10 + k1 * u11));
  }
}

// Row-blocked forward of the composite: one block per output row (b, oy). Per
// axis the two bilinear steps collapse to at most 3 consecutive input taps
// (m1 = m0 + 1 and each step spreads by < 1 input), so an output is a 3x3
// stencil: 9 loads instead of the 16 of evaluating the 4 intermediate samples.
// The taps and combined weights of every column live in LDS, the row's in
// registers (fp32 combination: within an ulp of the two-step rounding).
__device__ __forceinline__ int comb3(float s2, int o, int n2, float s1, int n1, float* wk) {
  int m0, m1, i00, i01, i10, i11;
  float l0, l1, a00, a01, a10, a11;
  lin_idx(s2, o, n2, m0, m1, l0, l1);
  lin_idx(s1, m0, n1, i00, i01, a00, a01);
  lin_idx(s1, m1, n1, i10, i11, a10, a11);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = i00 + k;
    wk[k] = l0 * ((i00 == i ? a00 : 0.f) + (i01 == i ? a01 : 0.f)) +
            l1 * ((i10 == i ? a10 : 0.f) + (i11 == i ? a11 : 0.f));
  }
  return i00;
}

template <typename T, bool ACT = false>
__global__ void __launch_bounds__(256) up2_resize_fwd_rows_kernel(
    const T* __restrict__ x, int h, int w, int C8, FastDiv fdC8, T* __restrict__ y, int th, int tw,
    float s1h, float s1w, float s2h, float s2w, ActSrc act = ActSrc{}) {
  extern __shared__ float u2f_tables[];  // [tw][3] weights, [tw] first tap
  float* xw = u2f_tables;
  int* xb = (int*)(u2f_tables + (size_t)tw * 3);
  const int C = C8 * 8;
  const int b = blockIdx.x / th, oy = blockIdx.x - b * th;
  for (int ox = threadIdx.x; ox < tw; ox += blockDim.x) xb[ox] = comb3(s2w, ox, 2 * w, s1w, w, xw + ox * 3);
  float wy[3];
  const int yb = comb3(s2h, oy, 2 * h, s1h, h, wy);
  __syncthreads();
  size_t rows[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) rows[a] = ((size_t)b * h + min(yb + a, h - 1)) * w * C;
  T* orow = y + ((size_t)b * th + oy) * tw * C;
  // gridDim.y segments per row (small batches: enough blocks for the chip)
  const uint32_t items = (uint32_t)tw * (uint32_t)C8;
  const uint32_t seg = (items + gridDim.y - 1) / gridDim.y;
  const uint32_t i0 = blockIdx.y * seg, i1 = min(items, i0 + seg);
  for (uint32_t it = i0 + threadIdx.x; it < i1; it += blockDim.x) {
    const int ox = (int)fdiv(it, fdC8);
    const int c = (int)(it - (uint32_t)ox * (uint32_t)C8) * 8;
    const int x0 = xb[ox];
    const float wx0 = xw[ox * 3], wx1 = xw[ox * 3 + 1], wx2 = xw[ox * 3 + 2];
    const int c0 = x0 * C + c, c1 = min(x0 + 1, w - 1) * C + c, c2 = min(x0 + 2, w - 1) * C + c;
    F8 v[9];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      v[3 * a] = src8<T, ACT>(x, rows[a] + c0, act, c);
      v[3 * a + 1] = src8<T, ACT>(x, rows[a] + c1, act, c);
      v[3 * a + 2] = src8<T, ACT>(x, rows[a] + c2, act, c);
    }
    F8 acc = f8zero();
#pragma unroll
    for (int a = 0; a < 3; ++a)
      acc += wy[a] * (wx0 * v[3 * a] + wx1 * v[3 * a + 1] + wx2 * v[3 * a + 2]);
    st8(orow + (size_t)ox * C + c, acc);
  }
}

// Separable form of the row-blocked composite forward: grid = (output row,
// channel slice). Phase 1 combines the row's 3 source rows with the y weights
// into an fp32 LDS row [w][cb] (each source element loaded once per block);
// phase 2 takes the 3 x taps of every output column from LDS: 3 global vector
// loads per output instead of 9.
template <typename T, bool ACT = false>
__global__ void __launch_bounds__(256) up2_resize_fwd_sep_kernel(
    const T* __restrict__ x, int h, int w, int C, int lcb8, T* __restrict__ y, int th, int tw,
    float s1h, float s1w, float s2h, float s2w, ActSrc act = ActSrc{}) {
  extern __shared__ float u2s_lds[];  // [w][cb] column sums, [tw][3] x weights, [tw] first taps
  const int cb8 = 1 << lcb8, cb = cb8 * 8;
  float* vcol = u2s_lds;
  float* xw = vcol + (size_t)w * cb;
  int* xb = (int*)(xw + (size_t)tw * 3);
  const int tid = threadIdx.x;
  const int b = blockIdx.x / th, oy = blockIdx.x - b * th;
  const int c0 = blockIdx.y * cb;
  for (int ox = tid; ox < tw; ox += blockDim.x) xb[ox] = comb3(s2w, ox, 2 * w, s1w, w, xw + ox * 3);
  float wy[3];
  const int yb = comb3(s2h, oy, 2 * h, s1h, h, wy);
  size_t rows[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) rows[a] = ((size_t)b * h + min(yb + a, h - 1)) * w * C + c0;
  const uint32_t items1 = (uint32_t)w << lcb8;
  for (uint32_t it = tid; it < items1; it += blockDim.x) {
    const int xi = (int)(it >> lcb8), c = (int)(it & (cb8 - 1)) * 8;
    const size_t o = (size_t)xi * C + c;
    const F8 v0 = src8<T, ACT>(x, rows[0] + o, act, c0 + c);
    const F8 v1 = src8<T, ACT>(x, rows[1] + o, act, c0 + c);
    const F8 v2 = src8<T, ACT>(x, rows[2] + o, act, c0 + c);
    F8 acc = wy[0] * v0;
    acc += wy[1] * v1;
    acc += wy[2] * v2;
    *(f32x4*)&vcol[xi * cb + c] = acc.a;
    *(f32x4*)&vcol[xi * cb + c + 4] = acc.b;
  }
  __syncthreads();
  T* orow = y + ((size_t)b * th + oy) * tw * C + c0;
  const uint32_t items2 = (uint32_t)tw << lcb8;
  for (uint32_t it = tid; it < items2; it += blockDim.x) {
    const int ox = (int)(it >> lcb8), c = (int)(it & (cb8 - 1)) * 8;
    const int x0 = xb[ox];
    const float wx0 = xw[ox * 3], wx1 = xw[ox * 3 + 1], wx2 = xw[ox * 3 + 2];
    F8 acc = wx0 * ld8(&vcol[x0 * cb + c]);
    acc += wx1 * ld8(&vcol[min(x0 + 1, w - 1) * cb + c]);
    acc += wx2 * ld8(&vcol[min(x0 + 2, w - 1) * cb + c]);
    st8(orow + (size_t)ox * C + c, acc);
  }
}

// combined 1-D weight of final output index o on input index i
__device__ __forceinline__ float comb_w(float s2, int o, int n2, float s1, int n1, int i) {
  int m0, m1;
  float l0, l1;
  lin_idx(s2, o, n2, m0, m1, l0, l1);
  float wgt = 0.f;
  if (l0 != 0.f) wgt += l0 * lin_w(s1, m0, n1, i);
  if (l1 != 0.f) wgt += l1 * lin_w(s1, m1, n1, i);
  return wgt;
}

template <typename T>
__global__ void __launch_bounds__(256) up2_resize_bwd8_kernel(const T* __restrict__ dy, int h,
                                                              int w, int C8, uint32_t total,
                                                              FastDiv fdC8, FastDiv fdw,
                                                              FastDiv fdh, T* __restrict__ dx,
                                                              int th, int tw, float s1h, float s1w,
                                                              float s2h, float s2w) {
  const int C = C8 * 8, h2 = 2 * h, w2 = 2 * w;
  for (uint32_t i = xcd_block() * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    uint32_t p;
    const Pix8 q = pix8(i, C8, h, w, fdC8, fdw, fdh, p);
    // intermediate rows touching iy, then final rows touching those
    int mlo, mhi, olo, ohi, olo2, ohi2;
    cand_range(s1h, q.y, h2, mlo, mhi);
    cand_range(s2h, mlo, th, olo, ohi2);
    cand_range(s2h, mhi, th, olo2, ohi);
    olo = min(olo, olo2);
    ohi = max(ohi, ohi2);
    int nlo, nhi, plo, phi, plo2, phi2;
    cand_range(s1w, q.x, w2, nlo, nhi);
    cand_range(s2w, nlo, tw, plo, phi2);
    cand_range(s2w, nhi, tw, plo2, phi);
    plo = min(plo, plo2);
    phi = max(phi, phi2);
    trim_range(olo, ohi, [&](int o) { return comb_w(s2h, o, h2, s1h, h, q.y); });
    trim_range(plo, phi, [&](int o) { return comb_w(s2w, o, w2, s1w, w, q.x); });
    const T* base = dy + (size_t)q.b * th * tw * C + q.c;
    F8 acc = f8zero();
    if (phi - plo < RS_W) {
      float wx[RS_W];
      int xo[RS_W];
#pragma unroll
      for (int k = 0; k < RS_W; ++k) {
        xo[k] = min(plo + k, phi);
        wx[k] = plo + k <= phi ? comb_w(s2w, plo + k, w2, s1w, w, q.x) : 0.f;
      }
      for (int oy = olo; oy <= ohi; ++oy) {
        const float wy = comb_w(s2h, oy, h2, s1h, h, q.y);
        if (wy != 0.f) gather_row(acc, base + (size_t)oy * tw * C, C, wy, wx, xo);
      }
    } else {
      for (int oy = olo; oy <= ohi; ++oy) {
        const float wy = comb_w(s2h, oy, h2, s1h, h, q.y);
        if (wy == 0.f) continue;
        const T* row = base + (size_t)oy * tw * C;
        for (int ox = plo; ox <= phi; ++ox) {
          const float wxk = comb_w(s2w, ox, w2, s1w, w, q.x);
          if (wxk != 0.f) acc += (wy * wxk) * ld8(row + (size_t)ox * C);
        }
      }
    }
    st8(dx + (size_t)p * C + q.c, acc);
  }
}

// Row-blocked form of the composite backward: one block per input row (b, iy).
// The x-axis windows and combined weights of every column are built once per
// block into LDS (the per-element form recomputes ~25 composite weights per
// lane: ALU-bound), the row's y window once; the lanes then only gather.
constexpr int U2_MAXW = 2048;  // widest row the LDS tables hold

template <typename T, bool RED>
__global__ void __launch_bounds__(256) up2_resize_bwd_rows_kernel(
    const T* __restrict__ dy, int h, int w, int C8, FastDiv fdC8, T* __restrict__ dx, int th,
    int tw, float s1h, float s1w, float s2h, float s2w, BnRedP rp) {
  extern __shared__ float u2_tables[];  // [w][RS_W] weights, [w] window starts, [w] widths
  float* xw = u2_tables;
  int* xlo = (int*)(u2_tables + (size_t)w * RS_W);
  int* xn = xlo + w;
  __shared__ float yw[RS_W];
  __shared__ int ywin[2];
  const int C = C8 * 8, h2 = 2 * h, w2 = 2 * w;
  const int b = blockIdx.x / h, iy = blockIdx.x - b * h;
  for (int ix = threadIdx.x; ix < w; ix += blockDim.x) {
    int nlo, nhi, plo, phi, plo2, phi2;
    cand_range(s1w, ix, w2, nlo, nhi);
    cand_range(s2w, nlo, tw, plo, phi2);
    cand_range(s2w, nhi, tw, plo2, phi);
    plo = min(plo, plo2);
    phi = max(phi, phi2);
    trim_range(plo, phi, [&](int o) { return comb_w(s2w, o, w2, s1w, w, ix); });
    xlo[ix] = plo;
    xn[ix] = phi - plo + 1;
#pragma unroll
    for (int k = 0; k < RS_W; ++k)
      xw[ix * RS_W + k] = plo + k <= phi ? comb_w(s2w, plo + k, w2, s1w, w, ix) : 0.f;
  }
  if (threadIdx.x == 0) {
    int mlo, mhi, olo, ohi, olo2, ohi2;
    cand_range(s1h, iy, h2, mlo, mhi);
    cand_range(s2h, mlo, th, olo, ohi2);
    cand_range(s2h, mhi, th, olo2, ohi);
    olo = min(olo, olo2);
    ohi = max(ohi, ohi2);
    trim_range(olo, ohi, [&](int o) { return comb_w(s2h, o, h2, s1h, h, iy); });
    ywin[0] = olo;
    ywin[1] = ohi;
#pragma unroll
    for (int k = 0; k < RS_W; ++k) yw[k] = olo + k <= ohi ? comb_w(s2h, olo + k, h2, s1h, h, iy) : 0.f;
  }
  __syncthreads();
  const int olo = ywin[0], ohi = ywin[1];
  const T* base = dy + (size_t)b * th * tw * C;
  T* orow = dx + ((size_t)b * h + iy) * w * C;
  const uint32_t items = (uint32_t)w * (uint32_t)C8;
  BnRedAcc ra;
  if (RED) ra.init(rp, (threadIdx.x % C8) * 8);
  for (uint32_t it = threadIdx.x; it < items; it += blockDim.x) {
    const int ix = (int)fdiv(it, fdC8);
    const int c = (int)(it - (uint32_t)ix * (uint32_t)C8) * 8;
    const int plo = xlo[ix], n = xn[ix];
    F8 acc = f8zero();
    if (n <= RS_W && ohi - olo < RS_W) {
      float wx[RS_W];
      int xo[RS_W];
#pragma unroll
      for (int k = 0; k < RS_W; ++k) {
        wx[k] = xw[ix * RS_W + k];
        xo[k] = plo + min(k, n - 1);
      }
      for (int oy = olo; oy <= ohi; ++oy) {
        const float wy = yw[oy - olo];
        if (wy != 0.f) gather_row(acc, base + (size_t)oy * tw * C + c, C, wy, wx, xo);
      }
    } else {  // wide windows: weights on the fly, as the per-element kernel
      for (int oy = olo; oy <= ohi; ++oy) {
        const float wy = comb_w(s2h, oy, h2, s1h, h, iy);
        if (wy == 0.f) continue;
        const T* row = base + (size_t)oy * tw * C + c;
        for (int ox = plo; ox < plo + n; ++ox) {
          const float wxk = comb_w(s2w, ox, w2, s1w, w, ix);
          if (wxk != 0.f) acc += (wy * wxk) * ld8(row + (size_t)ox * C);
        }
      }
    }
    st8(orow + (size_t)ix * C + c, acc);
    if (RED) ra.add<T>(rp, as_stored8<T>(acc), ((size_t)b * h + iy) * w + ix, C, c);
  }
  if (RED) ra.write(rp, C8);
}

// Row-blocked single-step resize backward (same scheme as the composite's).
template <typename T, bool RED>
__global__ void __launch_bounds__(256) resize_bwd_rows_kernel(
    const T* __restrict__ dy, int h, int w, int C8, FastDiv fdC8, T* __restrict__ dx, int th,
    int tw, float sh, float sw, BnRedP rp) {
  extern __shared__ float rs_tables[];  // [w][RS_W] weights, [w] window starts, [w] widths
  float* xw = rs_tables;
  int* xlo = (int*)(rs_tables + (size_t)w * RS_W);
  int* xn = xlo + w;
  __shared__ float yw[RS_W];
  __shared__ int ywin[2];
  const int C = C8 * 8;
  const int b = blockIdx.x / h, iy = blockIdx.x - b * h;
  for (int ix = threadIdx.x; ix < w; ix += blockDim.x) {
    int plo, phi;
    cand_range(sw, ix, tw, plo, phi);
    trim_range(plo, phi, [&](int o) { return lin_w(sw, o, w, ix); });
    xlo[ix] = plo;
    xn[ix] = phi - plo + 1;
#pragma unroll
    for (int k = 0; k < RS_W; ++k)
      xw[ix * RS_W + k] = plo + k <= phi ? lin_w(sw, plo + k, w, ix) : 0.f;
  }
  if (threadIdx.x == 0) {
    int olo, ohi;
    cand_range(sh, iy, th, olo, ohi);
    trim_range(olo, ohi, [&](int o) { return lin_w(sh, o, h, iy); });
    ywin[0] = olo;
    ywin[1] = ohi;
#pragma unroll
    for (int k = 0; k < RS_W; ++k) yw[k] = olo + k <= ohi ? lin_w(sh, olo + k, h, iy) : 0.f;
  }
  __syncthreads();
  const int olo = ywin[0], ohi = ywin[1];
  const T* base = dy + (size_t)b * th * tw * C;
  T* orow = dx + ((size_t)b * h + iy) * w * C;
  const uint32_t items = (uint32_t)w * (uint32_t)C8;
  BnRedAcc ra;
  if (RED) ra.init(rp, (threadIdx.x % C8) * 8);
  for (uint32_t it = threadIdx.x; it < items; it += blockDim.x) {
    const int ix = (int)fdiv(it, fdC8);
    const int c = (int)(it - (uint32_t)ix * (uint32_t)C8) * 8;
    const int plo = xlo[ix], n = xn[ix];
    F8 acc = f8zero();
    if (n <= RS_W && ohi - olo < RS_W) {
      float wx[RS_W];
      int xo[RS_W];
#pragma unroll
      for (int k = 0; k < RS_W; ++k) {
        wx[k] = xw[ix * RS_W + k];
        xo[k] = plo + min(k, n - 1);
      }
      for (int oy = olo; oy <= ohi; ++oy) {
        const float wy = yw[oy - olo];
        if (wy != 0.f) gather_row(acc, base + (size_t)oy * tw * C + c, C, wy, wx, xo);
      }
    } else {  // wide windows: weights on the fly, as the per-element kernel
      for (int oy = olo; oy <= ohi; ++oy) {
        const float wy = lin_w(sh, oy, h, iy);
        if (wy == 0.f) continue;
        const T* row = base + (size_t)oy * tw * C + c;
        for (int ox = plo; ox < plo + n; ++ox) {
          const float wxk = lin_w(sw, ox, w, ix);
          if (wxk != 0.f) acc += (wy * wxk) * ld8(row + (size_t)ox * C);
        }
      }
    }
    st8(orow + (size_t)ix * C + c, acc);
    if (RED) ra.add<T>(rp, as_stored8<T>(acc), ((size_t)b * h + iy) * w + ix, C, c);
  }
  if (RED) ra.write(rp, C8);
}

// Separable row-blocked backward of a bilinear upsample: the single resize
// (COMP false: nn.Upsample x2, Unetmodel.py:122-134) or the x2 + match
// composite (COMP true: up9, :140-141). Grid = (input row, channel slice).
// Phase 1 sums the block's dY rows (its y window) with their weights into an
// fp32 LDS row [tw][cb] — every dY element is loaded once per block with
// 16-B vector loads; phase 2 gathers each input column's x window from LDS.
// The 2-D gather form issued RS_W x-taps per dY row per output (~24 vector
// loads per output) and was load-issue bound at 2.2-2.9 TB/s.
__device__ __forceinline__ void comp_window(float s1, float s2, int i, int n1, int out, int& lo,
                                            int& hi) {
  int mlo, mhi, lo2, hi2;
  cand_range(s1, i, 2 * n1, mlo, mhi);
  cand_range(s2, mlo, out, lo, hi2);
  cand_range(s2, mhi, out, lo2, hi);
  lo = min(lo, lo2);
  hi = max(hi, hi2);
}

template <bool COMP>
__device__ __forceinline__ float sep_w(float s1, float s2, int o, int n1, int i) {
  if constexpr (COMP) return comb_w(s2, o, 2 * n1, s1, n1, i);
  return lin_w(s1, o, n1, i);
}

template <bool COMP>
__device__ __forceinline__ void sep_window(float s1, float s2, int i, int n1, int out, int& lo,
                                           int& hi) {
  if constexpr (COMP) comp_window(s1, s2, i, n1, out, lo, hi);
  else cand_range(s1, i, out, lo, hi);
  trim_range(lo, hi, [&](int o) { return sep_w<COMP>(s1, s2, o, n1, i); });
}

constexpr int SEP_YW = 32;  // union-window y weights kept per row (wider: computed per use)

// R consecutive input rows per block share one pass over the dY rows of
// their union window: each dY row is loaded once per block (a x2 upsample
// spreads a dY row over 2 input rows, the composite over ~3, so one row per
// block re-read dY 2-3x) and accumulated into R LDS rows.
template <typename T, bool RED, bool COMP, int R>
__global__ void __launch_bounds__(256) resize_bwd_sep_kernel(
    const T* __restrict__ dy, int h, int w, int C, int lcb8, T* __restrict__ dx, int th, int tw,
    float s1h, float s1w, float s2h, float s2w, BnRedP rp) {
  // [R][tw][cb] row sums, [w][RS_W] x weights, [w] window starts, [w] widths
  extern __shared__ float sep_lds[];
  __shared__ float yw[R][SEP_YW];
  __shared__ int ywin[2];
  const int cb8 = 1 << lcb8, cb = cb8 * 8;
  float* vrow = sep_lds;
  float* xw = sep_lds + (size_t)R * tw * cb;
  int* xlo = (int*)(xw + (size_t)w * RS_W);
  int* xn = xlo + w;
  const int tid = threadIdx.x;
  const int hb = (h + R - 1) / R;
  const int b = blockIdx.x / hb, iy0 = (blockIdx.x - b * hb) * R;
  const int nr = min(R, h - iy0);
  const int c0 = blockIdx.y * cb;
  for (int ix = tid; ix < w; ix += blockDim.x) {
    int lo, hi;
    sep_window<COMP>(s1w, s2w, ix, w, tw, lo, hi);
    xlo[ix] = lo;
    xn[ix] = hi - lo + 1;
#pragma unroll
    for (int k = 0; k < RS_W; ++k)
      xw[ix * RS_W + k] = lo + k <= hi ? sep_w<COMP>(s1w, s2w, lo + k, w, ix) : 0.f;
  }
  if (tid == 0) {
    int lo, hi, lo2, hi2;
    sep_window<COMP>(s1h, s2h, iy0, h, th, lo, hi);
    sep_window<COMP>(s1h, s2h, iy0 + nr - 1, h, th, lo2, hi2);
    ywin[0] = min(lo, lo2);
    ywin[1] = max(hi, hi2);
  }
  __syncthreads();
  const int olo = ywin[0], ny = ywin[1] - ywin[0] + 1;
  // weight of union-window row k on input row iy0 + r (0 outside its window)
  if (tid < R * SEP_YW) {
    const int r = tid / SEP_YW, k = tid % SEP_YW;
    yw[r][k] = (r < nr && k < ny) ? sep_w<COMP>(s1h, s2h, olo + k, h, iy0 + r) : 0.f;
  }
  __syncthreads();
  // phase 1: vrow[r][ox][c] = sum_oy wy(oy, iy0 + r) dY[b][oy][ox][c0 + c]
  const T* base = dy + (size_t)b * th * tw * C + c0;
  const size_t rstride = (size_t)tw * C;
  const uint32_t items1 = (uint32_t)tw << lcb8;
  for (uint32_t it = tid; it < items1; it += blockDim.x) {
    const int ox = (int)(it >> lcb8), c = (int)(it & (cb8 - 1)) * 8;
    const T* p = base + (size_t)olo * rstride + (size_t)ox * C + c;
    F8 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = f8zero();
    auto add = [&](const F8& v, int k) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float wk = k < SEP_YW ? yw[r][k]
                                    : (r < nr ? sep_w<COMP>(s1h, s2h, olo + k, h, iy0 + r) : 0.f);
        const F8 t = acc[r] + wk * v;  // a zero weight must not pass an Inf / NaN on
        acc[r].a = wk != 0.f ? t.a : acc[r].a;
        acc[r].b = wk != 0.f ? t.b : acc[r].b;
      }
    };
    int k = 0;
    for (; k + 1 < ny; k += 2) {  // two rows' loads in flight
      const F8 v0 = ld8(p + (size_t)k * rstride), v1 = ld8(p + (size_t)(k + 1) * rstride);
      add(v0, k);
      add(v1, k + 1);
    }
    if (k < ny) add(ld8(p + (size_t)k * rstride), k);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float* q = &vrow[((size_t)r * tw + ox) * cb + c];
      *(f32x4*)q = acc[r].a;
      *(f32x4*)(q + 4) = acc[r].b;
    }
  }
  __syncthreads();
  // phase 2: dx[b][iy0 + r][ix][c0 + c] = sum_k wx(ix, k) vrow[r][xlo + k][c]
  const uint32_t items2 = (uint32_t)w << lcb8;
  for (int r = 0; r < nr; ++r) {
    const int iy = iy0 + r;
    T* orow = dx + ((size_t)b * h + iy) * w * C + c0;
    const float* vr = vrow + (size_t)r * tw * cb;
    BnRedAcc ra;
    if (RED) ra.init(rp, c0 + (tid & (cb8 - 1)) * 8);
    for (uint32_t it = tid; it < items2; it += blockDim.x) {
      const int ix = (int)(it >> lcb8), c = (int)(it & (cb8 - 1)) * 8;
      const int lo = xlo[ix], n = xn[ix];
      F8 acc = f8zero();
      if (n <= RS_W) {
#pragma unroll
        for (int k = 0; k < RS_W; ++k)
          if (k < n) acc += xw[ix * RS_W + k] * ld8(&vr[(lo + k) * cb + c]);
      } else {
        for (int k = 0; k < n; ++k)
          acc += sep_w<COMP>(s1w, s2w, lo + k, w, ix) * ld8(&vr[(lo + k) * cb + c]);
      }
      st8(orow + (size_t)ix * C + c, acc);
      if (RED) ra.add<T>(rp, as_stored8<T>(acc), ((size_t)b * h + iy) * w + ix, C, c0 + c);
    }
    // partial row b * h + iy (the B * h rows nsm_bnred_chunks reports)
    if (RED) ra.write_slice(rp, cb8, c0, C, b * h + iy);
  }
}

// channel slice of the separable kernels: the widest power-of-two multiple
// of 8 channels dividing C (at most 256 groups) whose fp32 LDS rows (rows x
// width x cb) fit `budget` bytes; -1 if 8 channels do not fit
static int sep_lcb8(int C, int width, int rows = 1, size_t budget = 32768) {
  int l = 0;
  while ((8 << (l + 1)) <= C && C % (8 << (l + 1)) == 0 &&
         (size_t)rows * width * (8 << (l + 1)) * 4 <= budget && (1 << (l + 1)) <= 256)
    ++l;
  if ((size_t)rows * width * (8 << l) * 4 > budget) return -1;
  return l;
}
// the backward's rows per block and channel slice: 4 rows where a 32-channel
// (fp32 128-B) slice still fits 48 KiB, else 2, else 1
struct SepPlan {
  int R, lcb8;
};
// NSM_SEP_RMAX: cap on the rows per block. 2 by measurement (tools/
// elem_bench_f32.py, B=8 fp32): R = 2 vs 1 cuts the x2 backward 126 -> 110 us
// (C=512), and R = 4 is no faster without the fused BN reduction and slower
// with it (124 -> 145 us: four partial-row reductions per block)
static int sep_rmax() {
  static int v = [] {
    const char* e = getenv("NSM_SEP_RMAX");
    return e ? atoi(e) : 2;
  }();
  return v;
}
// NSM_SEP_LDS_KB: the LDS budget of the backward's fp32 row sums per block
// (64 KiB: two blocks per CU; 16 / 32 measured slower, B=8 fp32 step)
static size_t sep_lds_budget() {
  static size_t v = [] {
    const char* e = getenv("NSM_SEP_LDS_KB");
    return (size_t)(e ? atoi(e) : 64) * 1024;
  }();
  return v;
}
static SepPlan sep_bwd_plan(int C, int tw) {
  const size_t budget = sep_lds_budget();
  for (int R : {4, 2}) {
    if (R > sep_rmax()) continue;
    const int l = sep_lcb8(C, tw, R, budget);
    if (l >= 2 || (l >= 0 && (8 << l) == C)) return SepPlan{R, l};
  }
  return SepPlan{1, sep_lcb8(C, tw, 1, budget)};
}
// dynamic LDS above the default 64 KiB (gfx950: 160 KiB per workgroup)
template <typename K>
static void allow_big_lds(K kernel) {
  static const bool once = [&] {
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              120 * 1024);
    return true;
  }();
  (void)once;
}
template <typename T, bool RED, bool COMP, int R>
static void launch_sep_bwd(dim3 g, size_t lds, hipStream_t s, const void* dy, int h, int w, int C,
                           int lcb8, void* dx, int th, int tw, float s1h, float s1w, float s2h,
                           float s2w, const BnRedP& rp) {
  auto k = resize_bwd_sep_kernel<T, RED, COMP, R>;
  allow_big_lds(k);
  hipLaunchKernelGGL(k, g, dim3(256), lds, s, (const T*)dy, h, w, C, lcb8, (T*)dx, th, tw, s1h,
                     s1w, s2h, s2w, rp);
}
template <bool COMP>
static void dispatch_sep_bwd(const SepPlan& pl, int B, size_t lds, hipStream_t s, const void* dy,
                             int h, int w, int C, void* dx, int th, int tw, float s1h, float s1w,
                             float s2h, float s2w, const BnRedP* rp, int dtype) {
  const dim3 g((unsigned)(B * ((h + pl.R - 1) / pl.R)), (unsigned)(C >> (pl.lcb8 + 3)));
  const BnRedP r = rp ? *rp : BnRedP{};
#define NSM_SEP(T, RED, R)                                                                      \
  launch_sep_bwd<T, RED, COMP, R>(g, lds, s, dy, h, w, C, pl.lcb8, dx, th, tw, s1h, s1w, s2h, s2w, r)
#define NSM_SEP_R(T, RED) \
  (pl.R == 4 ? NSM_SEP(T, RED, 4) : pl.R == 2 ? NSM_SEP(T, RED, 2) : NSM_SEP(T, RED, 1))
  if (dtype == NSM_BF16) {
    if (rp) NSM_SEP_R(bf16_t, true); else NSM_SEP_R(bf16_t, false);
  }
  else if (dtype == NSM_F16) {
    if (rp) NSM_SEP_R(f16_t, true); else NSM_SEP_R(f16_t, false);
  } else {
    if (rp) NSM_SEP_R(float, true); else NSM_SEP_R(float, false);
  }
#undef NSM_SEP_R
#undef NSM_SEP
}
// fp32 only: in bf16 (16-B lanes, half the bytes per pixel) the 2-D gather
// forms measured faster (B=64: x2 backward 401 vs 675 us, composite forward
// 366 vs 541 us; 1080p eval 505 vs 457 frames/s)
// (NSM_RESIZE_SEP=2: the separable forms for the 16-bit storage too; measured
// slower again in round 6: B=64 bf16 x2 backward 516 -> 773 us at conv8)
static int sep_resize_mode() {
  static int v = [] {
    const char* e = getenv("NSM_RESIZE_SEP");
    return e ? atoi(e) : 1;
  }();
  return v;
}
static bool sep_resize() { return sep_resize_mode() != 0; }
static bool sep_for(int dtype) { return dtype == NSM_F32 ? sep_resize() : sep_resize_mode() == 2; }

// ---------------------------------------------------------------------------
// Model boundary: pixel_unshuffle(2) + NCHW->NHWC (+ zero channel pad), and its
// inverse for the input gradient.
// ---------------------------------------------------------------------------
// thread per output pixel: each group of 8 output channels = 2 input planes x
// 2 rows x 2 columns (channel 4c + 2i + j, F.pixel_unshuffle), read as float2
// pairs coalesced along x and written as one 16-B (bf16) / 32-B (fp32) vector
// H2: out is an h2 tensor [npix][2 cp] scaled from the slot `amax` holds
// (max|x|, filled beforehand), T = bf16_t (16-bit storage)
template <typename T, bool H2 = false>
__global__ void __launch_bounds__(256) input_prep_kernel(const float* __restrict__ x, int B, int C,
                                                         int H, int W, T* __restrict__ out, int cp,
                                                         uint32_t npix, FastDiv fdRw, FastDiv fdRh,
                                                         uint32_t* __restrict__ amax) {
  const int Rh = H / 2, Rw = W / 2;
  const size_t plane = (size_t)H * W;
  float hs = 0.f;
  if constexpr (H2) hs = exp2i(h2_exp(H2Scale{amax, 1.f}));
  uint32_t am = 0;  // max|out| (conv2's f16x2 operand scale)
  for (uint32_t p = blockIdx.x * 256u + threadIdx.x; p < npix; p += gridDim.x * 256u) {
    const uint32_t t = fdiv(p, fdRw);
    const int rx = (int)(p - t * (uint32_t)Rw);
    const uint32_t b = fdiv(t, fdRh);
    const int ry = (int)(t - b * (uint32_t)Rh);
    const float* src = x + (size_t)b * C * plane + (size_t)(2 * ry) * W + 2 * rx;
    for (int g = 0; g < cp / 8; ++g) {
      f32x2 r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // plane 2g + (q >> 1), row 2ry + (q & 1)
        const int c = 2 * g + (q >> 1);
        r[q] = c < C ? *(const f32x2*)(src + (size_t)c * plane + (q & 1) * W) : f32x2{0.f, 0.f};
      }
      const F8 v{f32x4{r[0].x, r[0].y, r[1].x, r[1].y}, f32x4{r[2].x, r[2].y, r[3].x, r[3].y}};
      if constexpr (H2) {
        h2_store8((bf16_t*)out + (size_t)p * 2 * cp, 8 * g, v, hs);
      } else {
        st8(out + (size_t)p * cp + 8 * g, v);
        if (amax) {
          amax_fold(am, v.a);
          amax_fold(am, v.b);
        }
      }
    }
  }
  if constexpr (!H2) amax_flush(am, amax);
}

template <typename T>
__global__ void input_grad_kernel(const T* __restrict__ dX, int B, int C, int H, int W, int cp,
                                  float* __restrict__ dx) {
  // thread per (b, c, ry, rx): one float4 of dX (channels 4c..4c+3 of pixel
  // (ry,rx)) -> the 2x2 block of plane c; rx fastest so stores coalesce.
  const int Rh = H / 2, Rw = W / 2;
  long long total = (long long)B * C * Rh * Rw;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < total; i += (long long)gridDim.x * blockDim.x) {
    int rx = (int)(i % Rw);
    long long t = i / Rw;
    int ry = (int)(t % Rh);
    t /= Rh;
    int c = (int)(t % C);
    int b = (int)(t / C);
    f32x4 v = ld4(dX + (((size_t)b * Rh + ry) * Rw + rx) * cp + 4 * c);
    float* o = dx + (((size_t)b * C + c) * H + 2 * ry) * W + 2 * rx;
    *(f32x2*)o = f32x2{v.x, v.y};
    *(f32x2*)(o + W) = f32x2{v.z, v.w};
  }
}

// ---------------------------------------------------------------------------
// Head: conv10 (1x1, 16->4, bias) -> pixel_shuffle(2) -> sigmoid
// ---------------------------------------------------------------------------
template <typename T>
__global__ void head_fwd_kernel(const T* __restrict__ z, int ldz, int B, int Rh, int Rw,
                                const float* __restrict__ w10, const float* __restrict__ b10,
                                float* __restrict__ out) {
  __shared__ float w[68];
  if (threadIdx.x < 64) w[threadIdx.x] = w10[threadIdx.x];
  if (threadIdx.x < 4) w[64 + threadIdx.x] = b10[threadIdx.x];
  __syncthreads();
  long long npix = (long long)B * Rh * Rw;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < npix;
       p += (long long)gridDim.x * blockDim.x) {
    float zz[16];
    const T* zr = z + (size_t)p * ldz;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v = ld4(zr + 4 * q);
      zz[4 * q] = v.x;
      zz[4 * q + 1] = v.y;
      zz[4 * q + 2] = v.z;
      zz[4 * q + 3] = v.w;
    }
    int rx = (int)(p % Rw);
    long long t = p / Rw;
    int ry = (int)(t % Rh);
    int b = (int)(t / Rh);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) acc += w[j * 16 + c] * zz[c];
      acc += w[64 + j];
      float s = 1.f / (1.f + expf(-acc));
      int di = j >> 1, dj = j & 1;
      out[((size_t)b * 2 * Rh + 2 * ry + di) * (2 * Rw) + 2 * rx + dj] = s;
    }
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256) head_bwd_kernel(
    const float* __restrict__ gout, const float* __restrict__ out, const T* __restrict__ z,
    int ldz, int B, int Rh, int Rw, const float* __restrict__ w10, T* __restrict__ dz,
    float* __restrict__ partial) {
  __shared__ float w[64];
  __shared__ float red[4][68];
  if (threadIdx.x < 64) w[threadIdx.x] = w10[threadIdx.x];
  __syncthreads();
  float accw[68];
#pragma unroll
  for (int k = 0; k < 68; ++k) accw[k] = 0.f;
  long long npix = (long long)B * Rh * Rw;
  for (long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x; p < npix;
       p += (long long)gridDim.x * blockDim.x) {
    int rx = (int)(p % Rw);
    long long t = p / Rw;
    int ry = (int)(t % Rh);
    int b = (int)(t / Rh);
    float d[4];
#pragma unroll
    for (int di = 0; di < 2; ++di) {  // the (dj = 0, 1) pair is adjacent: one 8-B load each
      size_t o = ((size_t)b * 2 * Rh + 2 * ry + di) * (2 * Rw) + 2 * rx;
      const f32x2 ov = *(const f32x2*)(out + o), gv = *(const f32x2*)(gout + o);
      d[2 * di] = gv.x * (1.f - ov.x) * ov.x;  // ATen sigmoid_backward
      d[2 * di + 1] = gv.y * (1.f - ov.y) * ov.y;
    }
    const T* zr = z + (size_t)p * ldz;
    T* dzr = dz + (size_t)p * ldz;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v = ld4(zr + 4 * q);
      float zv[4] = {v.x, v.y, v.z, v.w};
      f32x4 g;
      float gv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int c = 4 * q + e;
        gv[e] = d[0] * w[c] + d[1] * w[16 + c] + d[2] * w[32 + c] + d[3] * w[48 + c];
#pragma unroll
        for (int j = 0; j < 4; ++j) accw[j * 16 + c] += d[j] * zv[e];
      }
      g.x = gv[0];
      g.y = gv[1];
      g.z = gv[2];
      g.w = gv[3];
      st4(dzr + 4 * q, g);
    }
    for (int c = 16; c < ldz; c += 4) st4(dzr + c, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[64 + j] += d[j];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // dw10 (64 sums): a reduce-scatter butterfly. Each xor step halves the values
  // a lane holds (it keeps the half its lane bit selects and adds the partner's
  // copy of it), so after 6 steps lane L holds the wave sum of accw[L]: 63
  // cross-lane moves instead of 64 full wave reductions (384)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const bool up = (lane & o) != 0;
#pragma unroll
    for (int i = 0; i < o; ++i) {
      const float lo = accw[i], hi = accw[i + o];
      accw[i] = (up ? hi : lo) + __shfl_xor(up ? lo : hi, o, 64);
    }
  }
  red[wv][lane] = accw[0];
#pragma unroll
  for (int k = 64; k < 68; ++k) {
    float s = wave_sum(accw[k]);
    if (lane == 0) red[wv][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < 68) {
    float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    partial[(size_t)blockIdx.x * 68 + threadIdx.x] = s;
  }
}

// out[j] = sum_b partial[b][j]: one block per output column j (< 68)
__global__ void __launch_bounds__(256) head_reduce_kernel(const float* __restrict__ partial,
                                                          int nblk, float* dw10, float* db10) {
  __shared__ double sh[256];
  const int j = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 256) s += partial[(size_t)b * 68 + j];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (j < 64)
      dw10[j] = (float)sh[0];
    else
      db10[j - 64] = (float)sh[0];
  }
}

// ---------------------------------------------------------------------------
// Losses
// ---------------------------------------------------------------------------
__device__ __forceinline__ float block_sum256(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0) {
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) r += sh[k];
  }
  return r;
}

__global__ void __launch_bounds__(256) l1_partial_kernel(const float* __restrict__ o,
                                                         const float* __restrict__ t, int64_t n,
                                                         float* __restrict__ partial) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += fabsf(o[i] - t[i]);
  float r = block_sum256(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = r;
}

// sum of exp(alpha*|a-b|) - 1 (measure_temporal_instability, pert_loss.py:170-199)
__global__ void __launch_bounds__(256) expdiff_partial_kernel(const float* __restrict__ a,
                                                              const float* __restrict__ b,
                                                              int64_t n, float alpha,
                                                              float* __restrict__ partial) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += expf(alpha * fabsf(a[i] - b[i])) - 1.f;
  float r = block_sum256(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = r;
}

__global__ void finalize_mean_kernel(const float* __restrict__ partial, int nblk, double scale,
                                     float* out) {
  // one wave; fixed-order double accumulation
  __shared__ double sh[64];
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 64) s += partial[b];
  sh[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int k = 0; k < 64; ++k) tot += sh[k];
    out[0] = (float)(tot * scale);
  }
}

__global__ void l1_bwd_kernel(const float* __restrict__ o, const float* __restrict__ t, int64_t n,
                              float alpha, const float* __restrict__ gscale, float* grad,
                              int accumulate) {
  const float gs = gscale ? gscale[0] : 1.f;
  const float mag = (alpha * gs) / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float d = o[i] - t[i];
    float s = d > 0.f ? mag : (d < 0.f ? -mag : 0.f);
    grad[i] = accumulate ? grad[i] + s : s;
  }
}

__global__ void __launch_bounds__(1024) channel_std_kernel(const float* __restrict__ x, int B, int C,
                                                           int HW, float* __restrict__ std_o) {
  // one block per channel, double accumulation, two passes (torch.std, unbiased)
  __shared__ double sh[16];
  const int c = blockIdx.x;
  const long long n = (long long)B * HW;
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    long long b = i / HW, r = i - b * HW;
    s += x[((size_t)b * C + c) * HW + r];
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  double tot = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += sh[k];
  const double mean = tot / n;
  __syncthreads();
  double s2 = 0.0;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    long long b = i / HW, r = i - b * HW;
    double d = x[((size_t)b * C + c) * HW + r] - mean;
    s2 += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t2 = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t2 += sh[k];
    std_o[c] = (float)sqrt(t2 / (double)(n > 1 ? n - 1 : 1));
  }
}

// setdata.py:316: x = (x - mean[c]) / (std[c] + eps), in place on [B][C][HW]
__global__ void normalize_frames_kernel(float* __restrict__ x, int C, long long HW, long long total,
                                        const float* __restrict__ mean,
                                        const float* __restrict__ stdv, float eps) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)((i / HW) % C);
    const float d = stdv[c] + eps;
    x[i] = (x[i] - mean[c]) / d;
  }
}

__global__ void perturb_kernel(const float* __restrict__ x, const float* __restrict__ noise,
                               const float* __restrict__ stdv, int C, int HW, long long total,
                               float factor, float* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int c = (int)((i / HW) % C);
    out[i] = x[i] + (noise[i] * stdv[c]) * factor;
  }
}

// ---------------------------------------------------------------------------
// Train-step tail: global grad norm, clip coefficient, AdamW (torch semantics)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sumsq_partial_kernel(const float* __restrict__ g, int64_t n,
                                                            float* __restrict__ partial) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = g[i];
    s += v * v;
  }
  float r = block_sum256(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = r;
}

__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float inv_world, float max_norm,
                                 float* coef) {
  float norm = sqrtf(sumsq[0]) * inv_world;
  float c = max_norm / (norm + 1e-6f);
  coef[0] = inv_world * fminf(c, 1.f);
}

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, int64_t n, float decay,
                             float beta1, float beta2, float eps, float step_size,
                             float bc2_sqrt, const float* __restrict__ gcoef) {
  const float gc = gcoef ? gcoef[0] : 1.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gc;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + (1.f - beta1) * (gi - mi);
    float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

// grid for the xcd_block() kernels: a multiple of 8 blocks, <= 2048
static inline int xcd_grid(long long work) {
  long long g = (work + 255) / 256;
  g = g > 2048 ? 2048 : g;
  return (int)((g + 7) / 8 * 8);
}

static inline int grid_for(long long work, int per_block = 256, int cap = 8192) {
  long long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace nsm

using namespace nsm;

// ============================== C ABI ======================================
extern "C" int nsm_reduce_chunks(int M, int C) {
  if (M <= 0 || C <= 0 || C % 8) return 0;
  return colred_plan(M, C).nchunk;
}

#define NSM_T(T, p) ((T*)(p))
#define NSM_CT(T, p) ((const T*)(p))

extern "C" int nsm_bn_stats(const void* y, int ld, int M, int C, float* partial, int nchunk,
                            int dtype, void* stream) {
  NSM_CHECK_ARG(y && partial && M > 0 && C % 8 == 0 && ld % 8 == 0, "bn_stats: bad args");
  ColRed r = colred_plan(M, C);
  NSM_CHECK_ARG(nchunk == r.nchunk, "bn_stats: nchunk %d != %d", nchunk, r.nchunk);
  dim3 g(r.gx, r.nchunk);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(bn_stats_kernel<bf16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(bf16_t, y), ld, M, C, r.cl, r.rl, r.rpc, partial);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(bn_stats_kernel<f16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(f16_t, y), ld, M, C, r.cl, r.rl, r.rpc, partial);
  else
    hipLaunchKernelGGL(bn_stats_kernel<float>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(float, y), ld, M, C, r.cl, r.rl, r.rpc, partial);
  NSM_LAUNCH_CHECK("bn_stats");
  return 0;
}

extern "C" int nsm_reduce_rows(int M, int C) {
  if (M <= 0 || C <= 0 || C % 8) return 0;
  return colred_plan(M, C).rpc;
}

extern "C" int nsm_bn_finalize_train(const float* partial, int nchunk, int rows_per_chunk, int M,
                                     int C, int c_real, const float* gamma, const float* beta,
                                     float* run_mean, float* run_var, int64_t* num_batches,
                                     float momentum, float eps, int n_updates, float* mean,
                                     float* invstd, float* scale, float* shift, uint32_t* bound,
                                     float bound_mul, void* stream) {
  NSM_CHECK_ARG(partial && gamma && beta && mean && invstd && scale && shift, "bn_finalize: null");
  NSM_CHECK_ARG(M > 1, "bn_finalize: Expected more than 1 value per channel when training");
  NSM_CHECK_ARG(nchunk >= 1 && (rows_per_chunk == 0 ||
                                (rows_per_chunk >= 1 && (long long)nchunk * rows_per_chunk >= M)),
                "bn_finalize: chunks do not cover M");
  hipLaunchKernelGGL(bn_finalize_train_kernel, dim3(C), dim3(256), 0,
                     as_stream(stream), partial, nchunk, rows_per_chunk, M, C, c_real, gamma, beta,
                     run_mean,
                     run_var, num_batches, momentum, eps, n_updates, mean, invstd, scale, shift,
                     bound, bound_mul);
  NSM_LAUNCH_CHECK("bn_finalize_train");
  return 0;
}

extern "C" int nsm_bn_partials_merge(const float* partial, int nchunk, int rows_per_chunk, int M,
                                     int C, int group, float* out, void* stream) {
  NSM_CHECK_ARG(partial && out && nchunk >= 1 && group >= 1 && rows_per_chunk >= 0,
                "bn_partials_merge: bad args");
  dim3 grid(ceil_div(C, 256), ceil_div(nchunk, group));
  hipLaunchKernelGGL(bn_partials_merge_kernel, grid, dim3(256), 0, as_stream(stream), partial,
                     nchunk, rows_per_chunk, M, C, group, out);
  NSM_LAUNCH_CHECK("bn_partials_merge");
  return 0;
}

extern "C" int nsm_sum_rows(const float* part, int nrows, int width, int group, float* out,
                            void* stream) {
  NSM_CHECK_ARG(part && out && nrows >= 1 && width >= 1 && group >= 1, "sum_rows: bad args");
  dim3 grid(ceil_div(width, 256), ceil_div(nrows, group));
  hipLaunchKernelGGL(sum_rows_kernel, grid, dim3(256), 0, as_stream(stream), part, nrows, width,
                     group, out);
  NSM_LAUNCH_CHECK("sum_rows");
  return 0;
}

extern "C" int nsm_bn_finalize_eval(const float* run_mean, const float* run_var,
                                    const float* gamma, const float* beta, int C, int c_real,
                                    float eps, float* mean, float* invstd, float* scale,
                                    float* shift, void* stream) {
  NSM_CHECK_ARG(run_mean && run_var && gamma && beta && scale && shift, "bn_finalize_eval: null");
  hipLaunchKernelGGL(bn_finalize_eval_kernel, dim3(ceil_div(C, 256)), dim3(256), 0,
                     as_stream(stream), run_mean, run_var, gamma, beta, C, c_real, eps, mean, invstd,
                     scale, shift);
  NSM_LAUNCH_CHECK("bn_finalize_eval");
  return 0;
}

// streaming launch over [M pixels][C8 channel groups]: blockDim = the largest
// multiple of C8 <= 256 (each lane keeps one channel group), <= 2048 blocks
static void pix_launch(long long M, int C8, dim3& grid, dim3& block) {
  const int tpb = (256 / C8) * C8;
  const long long ppb = tpb / C8;
  long long g = (M + ppb - 1) / ppb;
  g = g < 1 ? 1 : (g > 2048 ? 2048 : g);
  grid = dim3((unsigned)g);
  block = dim3((unsigned)tpb);
}

extern "C" int nsm_bn_act(const void* y, int ldy, int M, int C, const float* scale,
                          const float* shift, float slope, const float* mask, int HW,
                          const void* res, int ldres, void* out, int ldo, int dtype,
                          uint32_t* amax, void* stream) {
  NSM_CHECK_ARG(y && scale && shift && out && C % 8 == 0 && C <= 2048 && ldy % 8 == 0 &&
                    ldo % 8 == 0 && (!res || ldres % 8 == 0) && (!mask || HW > 0),
                "bn_act: bad args");
  NSM_CHECK_ARG(M >= 0 && M < (1 << 30), "bn_act: too large");
  if (M == 0) return 0;
  dim3 g, b;
  pix_launch(M, C / 8, g, b);
  const FastDiv fh = make_fastdiv(mask ? HW : 1);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(bn_act_kernel<bf16_t>, g, b, 0, as_stream(stream), NSM_CT(bf16_t, y), ldy,
                       M, C / 8, fh, scale, shift, slope, mask, NSM_CT(bf16_t, res), ldres,
                       NSM_T(bf16_t, out), ldo, amax);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(bn_act_kernel<f16_t>, g, b, 0, as_stream(stream), NSM_CT(f16_t, y), ldy,
                       M, C / 8, fh, scale, shift, slope, mask, NSM_CT(f16_t, res), ldres,
                       NSM_T(f16_t, out), ldo, amax);
  else
    hipLaunchKernelGGL(bn_act_kernel<float>, g, b, 0, as_stream(stream), NSM_CT(float, y), ldy, M,
                       C / 8, fh, scale, shift, slope, mask, NSM_CT(float, res), ldres,
                       NSM_T(float, out), ldo, amax);
  NSM_LAUNCH_CHECK("bn_act");
  return 0;
}

extern "C" int nsm_bn_act_h2(const float* y, int ldy, int M, int C, const float* scale,
                             const float* shift, float slope, const float* mask, int HW, void* out,
                             const uint32_t* bound, void* stream) {
  NSM_CHECK_ARG(y && scale && shift && out && bound && C % 8 == 0 && C <= 2048 && ldy % 8 == 0 &&
                    (!mask || HW > 0) && ((uintptr_t)out % 16) == 0,
                "bn_act_h2: bad args");
  NSM_CHECK_ARG(M >= 0 && M < (1 << 30), "bn_act_h2: too large");
  if (M == 0) return 0;
  dim3 g, b;
  pix_launch(M, C / 8, g, b);
  hipLaunchKernelGGL(bn_act_h2_kernel, g, b, 0, as_stream(stream), y, ldy, M, C / 8,
                     make_fastdiv(mask ? HW : 1), scale, shift, slope, mask, (bf16_t*)out,
                     H2Scale{bound, 1.f});
  NSM_LAUNCH_CHECK("bn_act_h2");
  return 0;
}

extern "C" int nsm_bn_bwd_reduce(const void* g, int ldg, const void* y, int ldy, int M, int C,
                                 int HW, const float* scale, const float* shift, float slope,
                                 const float* mask, const float* mean, const float* invstd,
                                 float* partial, int nchunk, int dtype, uint32_t* amax_k1dz,
                                 void* stream) {
  NSM_CHECK_ARG(g && y && scale && shift && mean && invstd && partial && C % 8 == 0 &&
                    ldg % 8 == 0 && ldy % 8 == 0, "bn_bwd_reduce: bad args");
  ColRed r = colred_plan(M, C);
  NSM_CHECK_ARG(nchunk == r.nchunk, "bn_bwd_reduce: nchunk mismatch");
  dim3 gr(r.gx, r.nchunk);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16_t>, gr, dim3(256), 0, as_stream(stream),
                       NSM_CT(bf16_t, g), ldg, NSM_CT(bf16_t, y), ldy, M, C, make_fastdiv(HW),
                       scale, shift, slope, mask, mean, invstd, r.cl, r.rl, r.rpc, partial,
                       amax_k1dz);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<f16_t>, gr, dim3(256), 0, as_stream(stream),
                       NSM_CT(f16_t, g), ldg, NSM_CT(f16_t, y), ldy, M, C, make_fastdiv(HW),
                       scale, shift, slope, mask, mean, invstd, r.cl, r.rl, r.rpc, partial,
                       amax_k1dz);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, gr, dim3(256), 0, as_stream(stream),
                       NSM_CT(float, g), ldg, NSM_CT(float, y), ldy, M, C, make_fastdiv(HW), scale,
                       shift, slope, mask, mean, invstd, r.cl, r.rl, r.rpc, partial, amax_k1dz);
  NSM_LAUNCH_CHECK("bn_bwd_reduce");
  return 0;
}

extern "C" int nsm_bn_bwd_finalize(const float* partial, int nchunk, int M, int C, int c_real,
                                   const float* gamma, const float* invstd, float* dgamma,
                                   float* dbeta, float* dbias_prev, float* coef,
                                   const uint32_t* amax_k1dz, uint32_t* bound, void* stream) {
  NSM_CHECK_ARG(partial && gamma && invstd && coef, "bn_bwd_finalize: bad args");
  NSM_CHECK_ARG(!bound || amax_k1dz, "bn_bwd_finalize: a bound needs the max|k1 dz| slot");
  NSM_CHECK_ARG(M > 1 || !bound, "bn_bwd_finalize: M");
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0,
                     as_stream(stream), partial, nchunk, M, C, c_real, gamma, invstd, dgamma, dbeta,
                     dbias_prev, coef, amax_k1dz, bound);
  NSM_LAUNCH_CHECK("bn_bwd_finalize");
  return 0;
}

extern "C" int nsm_bn_bwd_apply(const void* g, int ldg, const void* y, int ldy, int M, int C,
                                int HW, const float* scale, const float* shift, float slope,
                                const float* mask, const float* mean, const float* coef, void* dy,
                                int lddy, int dtype, uint32_t* amax, void* stream) {
  NSM_CHECK_ARG(g && y && scale && shift && mean && coef && dy && C % 8 == 0 && C <= 2048 &&
                    ldg % 8 == 0 && ldy % 8 == 0 && lddy % 8 == 0 && (!mask || HW > 0),
                "bn_bwd_apply: bad args");
  NSM_CHECK_ARG(M >= 0 && M < (1 << 30), "bn_bwd_apply: too large");
  if (M == 0) return 0;
  dim3 gr, b;
  pix_launch(M, C / 8, gr, b);
  const FastDiv fh = make_fastdiv(mask ? HW : 1);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16_t>, gr, b, 0, as_stream(stream),
                       NSM_CT(bf16_t, g), ldg, NSM_CT(bf16_t, y), ldy, M, C, C / 8, fh, scale,
                       shift, slope, mask, mean, coef, NSM_T(bf16_t, dy), lddy, amax);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<f16_t>, gr, b, 0, as_stream(stream),
                       NSM_CT(f16_t, g), ldg, NSM_CT(f16_t, y), ldy, M, C, C / 8, fh, scale,
                       shift, slope, mask, mean, coef, NSM_T(f16_t, dy), lddy, amax);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, gr, b, 0, as_stream(stream),
                       NSM_CT(float, g), ldg, NSM_CT(float, y), ldy, M, C, C / 8, fh, scale,
                       shift, slope, mask, mean, coef, NSM_T(float, dy), lddy, amax);
  NSM_LAUNCH_CHECK("bn_bwd_apply");
  return 0;
}

extern "C" int nsm_bn_bwd_apply_h2(const float* g, int ldg, const float* y, int ldy, int M, int C,
                                   int HW, const float* scale, const float* shift, float slope,
                                   const float* mask, const float* mean, const float* coef,
                                   void* dy, const uint32_t* bound, void* stream) {
  NSM_CHECK_ARG(g && y && scale && shift && mean && coef && dy && bound && C % 8 == 0 &&
                    C <= 2048 && ldg % 8 == 0 && ldy % 8 == 0 && (!mask || HW > 0) &&
                    ((uintptr_t)dy % 16) == 0,
                "bn_bwd_apply_h2: bad args");
  NSM_CHECK_ARG(M >= 0 && M < (1 << 30), "bn_bwd_apply_h2: too large");
  if (M == 0) return 0;
  dim3 gr, b;
  pix_launch(M, C / 8, gr, b);
  hipLaunchKernelGGL(bn_bwd_apply_h2_kernel, gr, b, 0, as_stream(stream), g, ldg, y, ldy, M, C,
                     C / 8, make_fastdiv(mask ? HW : 1), scale, shift, slope, mask, mean, coef,
                     (bf16_t*)dy, H2Scale{bound, 1.f});
  NSM_LAUNCH_CHECK("bn_bwd_apply_h2");
  return 0;
}

extern "C" int nsm_bn_act_pool(const void* y, int B, int H, int W, int C, const float* scale,
                               const float* shift, float slope, void* z, void* pooled, int dtype,
                               uint32_t* amax, void* stream) {
  NSM_CHECK_ARG(y && z && pooled && scale && shift && C % 8 == 0 && H >= 2 && W >= 2,
                "bn_act_pool: bad args");
  const long long work = (long long)B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  NSM_CHECK_ARG(work < (1ll << 31), "bn_act_pool: too large");
  dim3 g(grid_for(work));
  const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv((W + 1) / 2),
                fh = make_fastdiv((H + 1) / 2);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(bn_act_pool_kernel<bf16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(bf16_t, y), B, H, W, C / 8, f8, fw, fh, scale, shift, slope,
                       NSM_T(bf16_t, z), NSM_T(bf16_t, pooled), amax);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(bn_act_pool_kernel<f16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(f16_t, y), B, H, W, C / 8, f8, fw, fh, scale, shift, slope,
                       NSM_T(f16_t, z), NSM_T(f16_t, pooled), amax);
  else
    hipLaunchKernelGGL(bn_act_pool_kernel<float>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(float, y), B, H, W, C / 8, f8, fw, fh, scale, shift, slope,
                       NSM_T(float, z), NSM_T(float, pooled), amax);
  NSM_LAUNCH_CHECK("bn_act_pool");
  return 0;
}

extern "C" int nsm_avgpool2_fwd(const void* x, int B, int H, int W, int C, void* y, int dtype,
                                void* stream) {
  NSM_CHECK_ARG(x && y && C % 8 == 0 && H >= 2 && W >= 2, "avgpool2_fwd: bad args");
  long long work = (long long)B * (H / 2) * (W / 2) * (C / 8);
  NSM_CHECK_ARG(work < (1ll << 31), "avgpool2_fwd: too large");
  dim3 g(grid_for(work));
  const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(W / 2), fh = make_fastdiv(H / 2);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(avgpool2_fwd_kernel<bf16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(bf16_t, x), B, H, W, C / 8, f8, fw, fh, NSM_T(bf16_t, y));
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(avgpool2_fwd_kernel<f16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(f16_t, x), B, H, W, C / 8, f8, fw, fh, NSM_T(f16_t, y));
  else
    hipLaunchKernelGGL(avgpool2_fwd_kernel<float>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(float, x), B, H, W, C / 8, f8, fw, fh, NSM_T(float, y));
  NSM_LAUNCH_CHECK("avgpool2_fwd");
  return 0;
}

// Blocks of the fused-reduction form: at most one chip-wide pass of 8 waves per
// SIMD (2048 blocks of 256), so every block folds several pixels into its
// partial row. At 8192 blocks the conv4-level call (64x64, 512 channels) ran one
// pixel per thread and wrote 4 KB of partials per block: 33.5 MB, half the size
// of dx, written and read back by the merge
static inline int pool_bnred_grid(long long work) { return grid_for(work, 256, 2048); }

static int avgpool2_bwd_add(const void* dy, int B, int H, int W, int C, const void* skip, void* dx,
                            int dtype, const BnRedP* rp, void* stream) {
  NSM_CHECK_ARG(dy && dx && C % 8 == 0, "avgpool2_bwd: bad args");
  long long work = (long long)B * H * W * (C / 8);
  NSM_CHECK_ARG(work < (1ll << 31), "avgpool2_bwd: too large");
  NSM_CHECK_ARG(!rp || 256 % (C / 8) == 0, "avgpool2_bwd: fused BN reduction needs C/8 | 256");
  dim3 g(rp ? pool_bnred_grid(work) : grid_for(work));  // rp: the rows nsm_bnred_chunks reports
  const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(W), fh = make_fastdiv(H);
  const BnRedP r = rp ? *rp : BnRedP{};
  hipStream_t s = as_stream(stream);
#define A_(T) NSM_CT(T, dy), B, H, W, C / 8, f8, fw, fh, NSM_CT(T, skip), NSM_T(T, dx), r
  if (dtype == NSM_BF16) {
    if (rp) hipLaunchKernelGGL((avgpool2_bwd_add_kernel<bf16_t, true>), g, dim3(256), 0, s, A_(bf16_t));
    else hipLaunchKernelGGL((avgpool2_bwd_add_kernel<bf16_t, false>), g, dim3(256), 0, s, A_(bf16_t));
  }
  else if (dtype == NSM_F16) {
    if (rp) hipLaunchKernelGGL((avgpool2_bwd_add_kernel<f16_t, true>), g, dim3(256), 0, s, A_(f16_t));
    else hipLaunchKernelGGL((avgpool2_bwd_add_kernel<f16_t, false>), g, dim3(256), 0, s, A_(f16_t));
  } else {
    if (rp) hipLaunchKernelGGL((avgpool2_bwd_add_kernel<float, true>), g, dim3(256), 0, s, A_(float));
    else hipLaunchKernelGGL((avgpool2_bwd_add_kernel<float, false>), g, dim3(256), 0, s, A_(float));
  }
#undef A_
  NSM_LAUNCH_CHECK("avgpool2_bwd");
  return 0;
}

extern "C" int nsm_avgpool2_bwd_add(const void* dy, int B, int H, int W, int C, const void* skip,
                                    void* dx, int dtype, void* stream) {
  return avgpool2_bwd_add(dy, B, H, W, C, skip, dx, dtype, nullptr, stream);
}

// NSM_RESIZE_ROWS=0: per-element resize backward instead of the row-blocked one
static bool rows_resize() {
  static bool v = [] {
    const char* e = getenv("NSM_RESIZE_ROWS");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// 8-channel path when C % 8 == 0 (all model activations), scalar otherwise
#define NSM_DT(KER, ...)                                                        \
  do {                                                                          \
    if (dtype == NSM_BF16)                                                      \
      hipLaunchKernelGGL(KER<bf16_t>, g, dim3(256), 0, s, __VA_ARGS__(bf16_t)); \
    else if (dtype == NSM_F16)                                                  \
      hipLaunchKernelGGL(KER<f16_t>, g, dim3(256), 0, s, __VA_ARGS__(f16_t));   \
    else                                                                        \
      hipLaunchKernelGGL(KER<float>, g, dim3(256), 0, s, __VA_ARGS__(float));   \
  } while (0)

extern "C" int nsm_resize_fwd(const void* x, int B, int Hi, int Wi, int C, void* y, int Ho, int Wo,
                              int dtype, void* stream) {
  NSM_CHECK_ARG(x && y && B > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && C > 0,
                "resize_fwd: bad args");
  const float sh = ac_scale(Hi, Ho), sw = ac_scale(Wi, Wo);
  hipStream_t s = as_stream(stream);
  const long long tot8 = (long long)B * Ho * Wo * (C / 8);
  if (C % 8 == 0 && tot8 < (1ll << 31)) {
    dim3 g(xcd_grid(tot8));
    const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(Wo), fh = make_fastdiv(Ho);
#define A_(T) NSM_CT(T, x), Hi, Wi, C / 8, (uint32_t)tot8, f8, fw, fh, NSM_T(T, y), Ho, Wo, sh, sw
    NSM_DT(resize_fwd8_kernel, A_);
#undef A_
  } else {
    dim3 g(grid_for((long long)B * Ho * Wo * C));
#define A_(T) NSM_CT(T, x), B, Hi, Wi, C, NSM_T(T, y), Ho, Wo, sh, sw
    NSM_DT(resize_fwd1_kernel, A_);
#undef A_
  }
  NSM_LAUNCH_CHECK("resize_fwd");
  return 0;
}

static int resize_bwd(const void* dy, int B, int Hi, int Wi, int C, void* dx, int Ho, int Wo,
                      int dtype, const BnRedP* rp, void* stream) {
  NSM_CHECK_ARG(dy && dx && B > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 && C > 0,
                "resize_bwd: bad args");
  const float sh = ac_scale(Hi, Ho), sw = ac_scale(Wi, Wo);
  hipStream_t s = as_stream(stream);
  const long long tot8 = (long long)B * Hi * Wi * (C / 8);
  const BnRedP r = rp ? *rp : BnRedP{};
  if (C % 8 == 0 && tot8 < (1ll << 31)) {
    dim3 g(xcd_grid(tot8));
    const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(Wi), fh = make_fastdiv(Hi);
    const SepPlan pl = sep_bwd_plan(C, Wo);
    const size_t slds = pl.lcb8 < 0 ? 0
                                    : (size_t)pl.R * Wo * (8 << pl.lcb8) * 4 +
                                          (size_t)Wi * (RS_W + 2) * 4;
    if (sep_for(dtype) && pl.lcb8 >= 0 && slds <= 96 * 1024 && (long long)B * Hi < (1ll << 31)) {
      dispatch_sep_bwd<false>(pl, B, slds, s, dy, Hi, Wi, C, dx, Ho, Wo, sh, sw, 0.f, 0.f, rp,
                              dtype);
    } else if (Wi <= U2_MAXW && (long long)B * Hi < (1ll << 31) && rows_resize()) {
      NSM_CHECK_ARG(!rp || 256 % (C / 8) == 0, "resize_bwd: fused BN reduction needs C/8 | 256");
      const size_t lds = (size_t)Wi * (RS_W + 2) * 4;
      const dim3 gr((unsigned)(B * Hi));
#define A_(T) NSM_CT(T, dy), Hi, Wi, C / 8, f8, NSM_T(T, dx), Ho, Wo, sh, sw, r
      if (dtype == NSM_BF16) {
        if (rp) hipLaunchKernelGGL((resize_bwd_rows_kernel<bf16_t, true>), gr, dim3(256), lds, s, A_(bf16_t));
        else hipLaunchKernelGGL((resize_bwd_rows_kernel<bf16_t, false>), gr, dim3(256), lds, s, A_(bf16_t));
      }
      else if (dtype == NSM_F16) {
        if (rp) hipLaunchKernelGGL((resize_bwd_rows_kernel<f16_t, true>), gr, dim3(256), lds, s, A_(f16_t));
        else hipLaunchKernelGGL((resize_bwd_rows_kernel<f16_t, false>), gr, dim3(256), lds, s, A_(f16_t));
      } else {
        if (rp) hipLaunchKernelGGL((resize_bwd_rows_kernel<float, true>), gr, dim3(256), lds, s, A_(float));
        else hipLaunchKernelGGL((resize_bwd_rows_kernel<float, false>), gr, dim3(256), lds, s, A_(float));
      }
#undef A_
    } else {
      NSM_CHECK_ARG(!rp, "resize_bwd: fused BN reduction needs the row-blocked kernel");
#define A_(T) NSM_CT(T, dy), Hi, Wi, C / 8, (uint32_t)tot8, f8, fw, fh, NSM_T(T, dx), Ho, Wo, sh, sw
      NSM_DT(resize_bwd8_kernel, A_);
#undef A_
    }
  } else {
    NSM_CHECK_ARG(!rp, "resize_bwd: fused BN reduction needs C % 8 == 0");
    dim3 g(grid_for((long long)B * Hi * Wi * C));
#define A_(T) NSM_CT(T, dy), B, Hi, Wi, C, NSM_T(T, dx), Ho, Wo, sh, sw
    NSM_DT(resize_bwd1_kernel, A_);
#undef A_
  }
  NSM_LAUNCH_CHECK("resize_bwd");
  return 0;
}

extern "C" int nsm_resize_bwd(const void* dy, int B, int Hi, int Wi, int C, void* dx, int Ho, int Wo,
                              int dtype, void* stream) {
  return resize_bwd(dy, B, Hi, Wi, C, dx, Ho, Wo, dtype, nullptr, stream);
}

// ---- upsample of a decoder block output that is never materialised ---------
extern "C" int nsm_resize_fwd_act(const void* y2, int B, int Hi, int Wi, int C, void* out, int Ho,
                                  int Wo, const float* scale, const float* shift, float slope,
                                  const void* res, int dtype, void* stream) {
  NSM_CHECK_ARG(y2 && out && scale && shift && B > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0 &&
                    C % 8 == 0, "resize_fwd_act: bad args");
  const long long tot8 = (long long)B * Ho * Wo * (C / 8);
  NSM_CHECK_ARG(tot8 < (1ll << 31), "resize_fwd_act: too large");
  const float sh = ac_scale(Hi, Ho), sw = ac_scale(Wi, Wo);
  hipStream_t s = as_stream(stream);
  dim3 g(xcd_grid(tot8));
  const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(Wo), fh = make_fastdiv(Ho);
  const ActSrc act{scale, shift, res, slope};
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL((resize_fwd8_kernel<bf16_t, true>), g, dim3(256), 0, s,
                       NSM_CT(bf16_t, y2), Hi, Wi, C / 8, (uint32_t)tot8, f8, fw, fh,
                       NSM_T(bf16_t, out), Ho, Wo, sh, sw, act);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL((resize_fwd8_kernel<f16_t, true>), g, dim3(256), 0, s,
                       NSM_CT(f16_t, y2), Hi, Wi, C / 8, (uint32_t)tot8, f8, fw, fh,
                       NSM_T(f16_t, out), Ho, Wo, sh, sw, act);
  else
    hipLaunchKernelGGL((resize_fwd8_kernel<float, true>), g, dim3(256), 0, s, NSM_CT(float, y2),
                       Hi, Wi, C / 8, (uint32_t)tot8, f8, fw, fh, NSM_T(float, out), Ho, Wo, sh,
                       sw, act);
  NSM_LAUNCH_CHECK("resize_fwd_act");
  return 0;
}

extern "C" int nsm_up2_resize_fwd_act(const void* y2, int B, int h, int w, int C, void* out,
                                      int th, int tw, const float* scale, const float* shift,
                                      float slope, const void* res, int dtype, void* stream) {
  NSM_CHECK_ARG(y2 && out && scale && shift && B > 0 && h > 0 && w > 0 && th > 0 && tw > 0 &&
                    C % 8 == 0, "up2_resize_fwd_act: bad args");
  const long long tot8 = (long long)B * th * tw * (C / 8);
  NSM_CHECK_ARG(tot8 < (1ll << 31), "up2_resize_fwd_act: too large");
  NSM_CHECK_ARG(tw <= U2_MAXW && (long long)B * th < (1ll << 31) && th * 2 >= 2 * h - 1 &&
                    tw * 2 >= 2 * w - 1, "up2_resize_fwd_act: needs the row-blocked kernel");
  hipStream_t s = as_stream(stream);
  const float a = ac_scale(h, 2 * h), b = ac_scale(w, 2 * w), c = ac_scale(2 * h, th),
              d = ac_scale(2 * w, tw);
  const FastDiv f8 = make_fastdiv(C / 8);
  const size_t lds = (size_t)tw * 4 * 4;
  const long long rows = (long long)B * th, per_row = (long long)tw * (C / 8);
  long long segs = (2048 + rows - 1) / rows;
  segs = std::max(1ll, std::min({segs, 16ll, (per_row + 1023) / 1024}));
  const dim3 gr((unsigned)rows, (unsigned)segs);
  const ActSrc act{scale, shift, res, slope};
  const int lcb8 = sep_lcb8(C, w);
  const size_t slds = lcb8 < 0 ? 0 : (size_t)w * (8 << lcb8) * 4 + (size_t)tw * 16;
  if (sep_for(dtype) && lcb8 >= 0 && slds <= 65536) {
    const dim3 gs((unsigned)rows, (unsigned)(C / (8 << lcb8)));
    if (dtype == NSM_BF16)
      hipLaunchKernelGGL((up2_resize_fwd_sep_kernel<bf16_t, true>), gs, dim3(256), slds, s,
                         NSM_CT(bf16_t, y2), h, w, C, lcb8, NSM_T(bf16_t, out), th, tw, a, b, c,
                         d, act);
    else if (dtype == NSM_F16)
      hipLaunchKernelGGL((up2_resize_fwd_sep_kernel<f16_t, true>), gs, dim3(256), slds, s,
                         NSM_CT(f16_t, y2), h, w, C, lcb8, NSM_T(f16_t, out), th, tw, a, b, c,
                         d, act);
    else
      hipLaunchKernelGGL((up2_resize_fwd_sep_kernel<float, true>), gs, dim3(256), slds, s,
                         NSM_CT(float, y2), h, w, C, lcb8, NSM_T(float, out), th, tw, a, b, c, d,
                         act);
  } else if (dtype == NSM_BF16)
    hipLaunchKernelGGL((up2_resize_fwd_rows_kernel<bf16_t, true>), gr, dim3(256), lds, s,
                       NSM_CT(bf16_t, y2), h, w, C / 8, f8, NSM_T(bf16_t, out), th, tw, a, b, c,
                       d, act);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL((up2_resize_fwd_rows_kernel<f16_t, true>), gr, dim3(256), lds, s,
                       NSM_CT(f16_t, y2), h, w, C / 8, f8, NSM_T(f16_t, out), th, tw, a, b, c,
                       d, act);
  else
    hipLaunchKernelGGL((up2_resize_fwd_rows_kernel<float, true>), gr, dim3(256), lds, s,
                       NSM_CT(float, y2), h, w, C / 8, f8, NSM_T(float, out), th, tw, a, b, c, d,
                       act);
  NSM_LAUNCH_CHECK("up2_resize_fwd_act");
  return 0;
}

extern "C" int nsm_up2_resize_fwd(const void* x, int B, int h, int w, int C, void* y, int th,
                                  int tw, int dtype, void* stream) {
  NSM_CHECK_ARG(x && y && B > 0 && h > 0 && w > 0 && th > 0 && tw > 0 && C % 8 == 0,
                "up2_resize_fwd: bad args");
  const long long tot8 = (long long)B * th * tw * (C / 8);
  NSM_CHECK_ARG(tot8 < (1ll << 31), "up2_resize_fwd: too large");
  hipStream_t s = as_stream(stream);
  dim3 g(xcd_grid(tot8));
  const float a = ac_scale(h, 2 * h), b = ac_scale(w, 2 * w), c = ac_scale(2 * h, th),
              d = ac_scale(2 * w, tw);
  const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(tw), fh = make_fastdiv(th);
  if (tw <= U2_MAXW && (long long)B * th < (1ll << 31) && th * 2 >= 2 * h - 1 && tw * 2 >= 2 * w - 1) {
    // second step downsizes (or keeps) the x2 grid: the 3-tap collapse holds
    const size_t lds = (size_t)tw * 4 * 4;
    // row segments: >= ~2048 blocks when B * th is small (1080p inference: 135 rows)
    const long long rows = (long long)B * th, per_row = (long long)tw * (C / 8);
    long long segs = (2048 + rows - 1) / rows;
    segs = std::max(1ll, std::min({segs, 16ll, (per_row + 1023) / 1024}));
    const dim3 gr((unsigned)rows, (unsigned)segs);
    const int lcb8 = sep_lcb8(C, w);
    const size_t slds = lcb8 < 0 ? 0 : (size_t)w * (8 << lcb8) * 4 + (size_t)tw * 16;
    if (sep_for(dtype) && lcb8 >= 0 && slds <= 65536) {
      const dim3 gs((unsigned)rows, (unsigned)(C / (8 << lcb8)));
#define A_(T) NSM_CT(T, x), h, w, C, lcb8, NSM_T(T, y), th, tw, a, b, c, d
      if (dtype == NSM_BF16)
        hipLaunchKernelGGL(up2_resize_fwd_sep_kernel<bf16_t>, gs, dim3(256), slds, s, A_(bf16_t));
      else if (dtype == NSM_F16)
        hipLaunchKernelGGL(up2_resize_fwd_sep_kernel<f16_t>, gs, dim3(256), slds, s, A_(f16_t));
      else
        hipLaunchKernelGGL(up2_resize_fwd_sep_kernel<float>, gs, dim3(256), slds, s, A_(float));
#undef A_
    } else {
#define A_(T) NSM_CT(T, x), h, w, C / 8, f8, NSM_T(T, y), th, tw, a, b, c, d
    if (dtype == NSM_BF16)
      hipLaunchKernelGGL(up2_resize_fwd_rows_kernel<bf16_t>, gr, dim3(256), lds, s, A_(bf16_t));
    else if (dtype == NSM_F16)
      hipLaunchKernelGGL(up2_resize_fwd_rows_kernel<f16_t>, gr, dim3(256), lds, s, A_(f16_t));
    else
      hipLaunchKernelGGL(up2_resize_fwd_rows_kernel<float>, gr, dim3(256), lds, s, A_(float));
#undef A_
    }
  } else {
#define A_(T) NSM_CT(T, x), h, w, C / 8, (uint32_t)tot8, f8, fw, fh, NSM_T(T, y), th, tw, a, b, c, d
    NSM_DT(up2_resize_fwd8_kernel, A_);
#undef A_
  }
  NSM_LAUNCH_CHECK("up2_resize_fwd");
  return 0;
}

static int up2_resize_bwd(const void* dy, int B, int h, int w, int C, void* dx, int th, int tw,
                          int dtype, const BnRedP* rp, void* stream) {
  NSM_CHECK_ARG(dy && dx && B > 0 && h > 0 && w > 0 && th > 0 && tw > 0 && C % 8 == 0,
                "up2_resize_bwd: bad args");
  const long long tot8 = (long long)B * h * w * (C / 8);
  NSM_CHECK_ARG(tot8 < (1ll << 31), "up2_resize_bwd: too large");
  hipStream_t s = as_stream(stream);
  dim3 g(xcd_grid(tot8));
  const float a = ac_scale(h, 2 * h), b = ac_scale(w, 2 * w), c = ac_scale(2 * h, th),
              d = ac_scale(2 * w, tw);
  const FastDiv f8 = make_fastdiv(C / 8), fw = make_fastdiv(w), fh = make_fastdiv(h);
  const BnRedP r = rp ? *rp : BnRedP{};
  const SepPlan pl = sep_bwd_plan(C, tw);
  const size_t slds = pl.lcb8 < 0 ? 0
                                  : (size_t)pl.R * tw * (8 << pl.lcb8) * 4 +
                                        (size_t)w * (RS_W + 2) * 4;
  if (sep_for(dtype) && pl.lcb8 >= 0 && slds <= 96 * 1024 && (long long)B * h < (1ll << 31)) {
    dispatch_sep_bwd<true>(pl, B, slds, s, dy, h, w, C, dx, th, tw, a, b, c, d, rp, dtype);
  } else if (w <= U2_MAXW && (long long)B * h < (1ll << 31)) {
    NSM_CHECK_ARG(!rp || 256 % (C / 8) == 0, "up2_resize_bwd: fused BN reduction needs C/8 | 256");
    const size_t lds = (size_t)w * (RS_W + 2) * 4;
    const dim3 gr((unsigned)(B * h));
#define A_(T) NSM_CT(T, dy), h, w, C / 8, f8, NSM_T(T, dx), th, tw, a, b, c, d, r
    if (dtype == NSM_BF16) {
      if (rp) hipLaunchKernelGGL((up2_resize_bwd_rows_kernel<bf16_t, true>), gr, dim3(256), lds, s, A_(bf16_t));
      else hipLaunchKernelGGL((up2_resize_bwd_rows_kernel<bf16_t, false>), gr, dim3(256), lds, s, A_(bf16_t));
    }
    else if (dtype == NSM_F16) {
      if (rp) hipLaunchKernelGGL((up2_resize_bwd_rows_kernel<f16_t, true>), gr, dim3(256), lds, s, A_(f16_t));
      else hipLaunchKernelGGL((up2_resize_bwd_rows_kernel<f16_t, false>), gr, dim3(256), lds, s, A_(f16_t));
    } else {
      if (rp) hipLaunchKernelGGL((up2_resize_bwd_rows_kernel<float, true>), gr, dim3(256), lds, s, A_(float));
      else hipLaunchKernelGGL((up2_resize_bwd_rows_kernel<float, false>), gr, dim3(256), lds, s, A_(float));
    }
#undef A_
  } else {
    NSM_CHECK_ARG(!rp, "up2_resize_bwd: fused BN reduction needs the row-blocked kernel");
#define A_(T) NSM_CT(T, dy), h, w, C / 8, (uint32_t)tot8, f8, fw, fh, NSM_T(T, dx), th, tw, a, b, c, d
    NSM_DT(up2_resize_bwd8_kernel, A_);
#undef A_
  }
  NSM_LAUNCH_CHECK("up2_resize_bwd");
  return 0;
}

extern "C" int nsm_up2_resize_bwd(const void* dy, int B, int h, int w, int C, void* dx, int th,
                                  int tw, int dtype, void* stream) {
  return up2_resize_bwd(dy, B, h, w, C, dx, th, tw, dtype, nullptr, stream);
}

// ---- gradient producers with the fused BN-backward reduction (BnRedP) ----
// kind 0: nsm_avgpool2_bwd_add (H, W: dx's size), 1: nsm_resize_bwd (Hi, Wi),
// 2: nsm_up2_resize_bwd (h, w). Partial rows the call writes; 0 = the fused
// form does not apply (use the plain call + nsm_bn_bwd_reduce).
extern "C" int nsm_bnred_chunks(int kind, int B, int H, int W, int C) {
  if (B <= 0 || H <= 0 || W <= 0 || C % 8 || 256 % (C / 8)) return 0;
  if (kind == 0) {
    const long long work = (long long)B * H * W * (C / 8);
    return work < (1ll << 31) ? pool_bnred_grid(work) : 0;
  }
  if (kind == 1 && !rows_resize()) return 0;
  if ((kind == 1 || kind == 2) && W <= U2_MAXW && (long long)B * H < (1ll << 31) &&
      (long long)B * H * W * (C / 8) < (1ll << 31))
    return B * H;
  return 0;
}

#define NSM_BNRED_ARGS                                                                  \
  const void *y2, const float *scale, const float *shift, const float *mean,            \
      const float *invstd, float slope, float *partial, uint32_t *amax_k1dz
#define NSM_BNRED_CHECK(what)                                                           \
  NSM_CHECK_ARG(y2 && scale && shift && mean && invstd && partial, what ": null BN args"); \
  const BnRedP rp{y2, scale, shift, mean, invstd, slope, partial, amax_k1dz}

extern "C" int nsm_avgpool2_bwd_add_bnred(const void* dy, int B, int H, int W, int C,
                                          const void* skip, void* dx, int dtype, NSM_BNRED_ARGS,
                                          void* stream) {
  NSM_BNRED_CHECK("avgpool2_bwd_add_bnred");
  return avgpool2_bwd_add(dy, B, H, W, C, skip, dx, dtype, &rp, stream);
}
extern "C" int nsm_resize_bwd_bnred(const void* dy, int B, int Hi, int Wi, int C, void* dx, int Ho,
                                    int Wo, int dtype, NSM_BNRED_ARGS, void* stream) {
  NSM_BNRED_CHECK("resize_bwd_bnred");
  return resize_bwd(dy, B, Hi, Wi, C, dx, Ho, Wo, dtype, &rp, stream);
}
extern "C" int nsm_up2_resize_bwd_bnred(const void* dy, int B, int h, int w, int C, void* dx,
                                        int th, int tw, int dtype, NSM_BNRED_ARGS, void* stream) {
  NSM_BNRED_CHECK("up2_resize_bwd_bnred");
  return up2_resize_bwd(dy, B, h, w, C, dx, th, tw, dtype, &rp, stream);
}
#undef NSM_BNRED_ARGS
#undef NSM_BNRED_CHECK
#undef NSM_DT

extern "C" int nsm_input_prep(const float* x, int B, int C, int H, int W, void* out, int cp,
                              int dtype, uint32_t* amax, void* stream) {
  NSM_CHECK_ARG(x && out && H % 2 == 0 && W % 2 == 0 && cp >= 4 * C && cp % 8 == 0,
                "input_prep: bad args");
  NSM_CHECK_ARG(((uintptr_t)x % 8) == 0, "input_prep: x must be 8-byte aligned");
  const long long npix = (long long)B * (H / 2) * (W / 2);
  NSM_CHECK_ARG(npix < (1ll << 31), "input_prep: too large");
  dim3 g(grid_for(npix, 256, 2048));
  const FastDiv fw = make_fastdiv(W / 2), fh = make_fastdiv(H / 2);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(input_prep_kernel<bf16_t>, g, dim3(256), 0, as_stream(stream), x, B, C, H, W,
                       NSM_T(bf16_t, out), cp, (uint32_t)npix, fw, fh, nullptr);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(input_prep_kernel<f16_t>, g, dim3(256), 0, as_stream(stream), x, B, C, H, W,
                       NSM_T(f16_t, out), cp, (uint32_t)npix, fw, fh, nullptr);
  else
    hipLaunchKernelGGL(input_prep_kernel<float>, g, dim3(256), 0, as_stream(stream), x, B, C, H, W,
                       NSM_T(float, out), cp, (uint32_t)npix, fw, fh, amax);
  NSM_LAUNCH_CHECK("input_prep");
  return 0;
}

extern "C" int nsm_input_prep_h2(const float* x, int B, int C, int H, int W, void* out, int cp,
                                 uint32_t* amax, void* stream) {
  NSM_CHECK_ARG(x && out && amax && H % 2 == 0 && W % 2 == 0 && cp >= 4 * C && cp % 8 == 0,
                "input_prep_h2: bad args");
  NSM_CHECK_ARG(((uintptr_t)x % 8) == 0 && ((uintptr_t)out % 16) == 0, "input_prep_h2: alignment");
  const long long npix = (long long)B * (H / 2) * (W / 2);
  NSM_CHECK_ARG(npix < (1ll << 31), "input_prep_h2: too large");
  const int rc = nsm_absmax(x, (int64_t)B * C * H * W, amax, stream);  // the scale source
  if (rc) return rc;
  dim3 g(grid_for(npix, 256, 2048));
  hipLaunchKernelGGL((input_prep_kernel<bf16_t, true>), g, dim3(256), 0, as_stream(stream), x, B, C,
                     H, W, (bf16_t*)out, cp, (uint32_t)npix, make_fastdiv(W / 2),
                     make_fastdiv(H / 2), amax);
  NSM_LAUNCH_CHECK("input_prep_h2");
  return 0;
}

extern "C" int nsm_input_grad(const void* dX, int B, int C, int H, int W, int cp, float* dx,
                              int dtype, void* stream) {
  NSM_CHECK_ARG(dX && dx && H % 2 == 0 && W % 2 == 0 && cp >= 4 * C && cp % 4 == 0,
                "input_grad: bad args");
  long long work = (long long)B * C * (H / 2) * (W / 2);
  dim3 g(grid_for(work));
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(input_grad_kernel<bf16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(bf16_t, dX), B, C, H, W, cp, dx);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(input_grad_kernel<f16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(f16_t, dX), B, C, H, W, cp, dx);
  else
    hipLaunchKernelGGL(input_grad_kernel<float>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(float, dX), B, C, H, W, cp, dx);
  NSM_LAUNCH_CHECK("input_grad");
  return 0;
}

extern "C" int nsm_head_fwd(const void* z, int ldz, int B, int Rh, int Rw, const float* w10,
                            const float* b10, float* out, int dtype, void* stream) {
  NSM_CHECK_ARG(z && w10 && b10 && out && ldz >= 16 && ldz % 4 == 0, "head_fwd: bad args");
  long long npix = (long long)B * Rh * Rw;
  dim3 g(grid_for(npix));
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(bf16_t, z), ldz, B, Rh, Rw, w10, b10, out);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(head_fwd_kernel<f16_t>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(f16_t, z), ldz, B, Rh, Rw, w10, b10, out);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, g, dim3(256), 0, as_stream(stream),
                       NSM_CT(float, z), ldz, B, Rh, Rw, w10, b10, out);
  NSM_LAUNCH_CHECK("head_fwd");
  return 0;
}

extern "C" int nsm_head_bwd_blocks(int B, int Rh, int Rw) {
  return grid_for((long long)B * Rh * Rw, 256, 1024);
}

extern "C" int nsm_head_bwd(const float* gout, const float* out, const void* z, int ldz, int B,
                            int Rh, int Rw, const float* w10, void* dz, float* partial, float* dw10,
                            float* db10, int dtype, void* stream) {
  NSM_CHECK_ARG(gout && out && z && w10 && dz && partial && dw10 && db10 && ldz % 4 == 0,
                "head_bwd: bad args");
  int nblk = nsm_head_bwd_blocks(B, Rh, Rw);
  hipStream_t s = as_stream(stream);
  if (dtype == NSM_BF16)
    hipLaunchKernelGGL(head_bwd_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, gout, out,
                       NSM_CT(bf16_t, z), ldz, B, Rh, Rw, w10, NSM_T(bf16_t, dz), partial);
  else if (dtype == NSM_F16)
    hipLaunchKernelGGL(head_bwd_kernel<f16_t>, dim3(nblk), dim3(256), 0, s, gout, out,
                       NSM_CT(f16_t, z), ldz, B, Rh, Rw, w10, NSM_T(f16_t, dz), partial);
  else
    hipLaunchKernelGGL(head_bwd_kernel<float>, dim3(nblk), dim3(256), 0, s, gout, out,
                       NSM_CT(float, z), ldz, B, Rh, Rw, w10, NSM_T(float, dz), partial);
  NSM_LAUNCH_CHECK("head_bwd");
  hipLaunchKernelGGL(head_reduce_kernel, dim3(68), dim3(256), 0, s, partial, nblk, dw10, db10);
  NSM_LAUNCH_CHECK("head_reduce");
  return 0;
}

extern "C" int nsm_loss_blocks(int64_t n) { return grid_for(n, 1024, 1024); }

extern "C" int nsm_l1_loss_fwd(const float* o, const float* t, int64_t n, float alpha,
                               float* partial, float* out, void* stream) {
  NSM_CHECK_ARG(o && t && partial && out && n > 0, "l1_loss_fwd: bad args");
  int nb = nsm_loss_blocks(n);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(l1_partial_kernel, dim3(nb), dim3(256), 0, s, o, t, n, partial);
  hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, partial, nb,
                     (double)alpha / (double)n, out);
  NSM_LAUNCH_CHECK("l1_loss_fwd");
  return 0;
}

extern "C" int nsm_expdiff_mean(const float* a, const float* b, int64_t n, float alpha,
                                float* partial, float* out, void* stream) {
  NSM_CHECK_ARG(a && b && partial && out && n > 0, "expdiff_mean: bad args");
  int nb = nsm_loss_blocks(n);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(expdiff_partial_kernel, dim3(nb), dim3(256), 0, s, a, b, n, alpha, partial);
  hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, partial, nb, 1.0 / (double)n,
                     out);
  NSM_LAUNCH_CHECK("expdiff_mean");
  return 0;
}

extern "C" int nsm_l1_loss_bwd(const float* o, const float* t, int64_t n, float alpha,
                               const float* gscale, float* grad, int accumulate, void* stream) {
  NSM_CHECK_ARG(o && t && grad && n > 0, "l1_loss_bwd: bad args");
  hipLaunchKernelGGL(l1_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), o, t, n,
                     alpha, gscale, grad, accumulate);
  NSM_LAUNCH_CHECK("l1_loss_bwd");
  return 0;
}

extern "C" int nsm_channel_std(const float* x, int B, int C, int H, int W, float* partial,
                               float* std_o, void* stream) {
  (void)partial;
  NSM_CHECK_ARG(x && std_o && B * H * W > 0, "channel_std: bad args");
  hipLaunchKernelGGL(channel_std_kernel, dim3(C), dim3(1024), 0, as_stream(stream), x, B, C, H * W,
                     std_o);
  NSM_LAUNCH_CHECK("channel_std");
  return 0;
}

extern "C" int nsm_perturb(const float* x, const float* noise, const float* stdv, int B, int C,
                           int H, int W, float factor, float* out, void* stream) {
  NSM_CHECK_ARG(x && noise && stdv && out, "perturb: bad args");
  long long total = (long long)B * C * H * W;
  hipLaunchKernelGGL(perturb_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), x,
                     noise, stdv, C, H * W, total, factor, out);
  NSM_LAUNCH_CHECK("perturb");
  return 0;
}

extern "C" int nsm_normalize_frames(float* x, int B, int C, int64_t HW, const float* mean,
                                    const float* stdv, float eps, void* stream) {
  NSM_CHECK_ARG(x && mean && stdv && B > 0 && C > 0 && HW > 0, "normalize_frames: bad args");
  long long total = (long long)B * C * HW;
  hipLaunchKernelGGL(normalize_frames_kernel, dim3(grid_for(total)), dim3(256), 0,
                     as_stream(stream), x, C, (long long)HW, total, mean, stdv, eps);
  NSM_LAUNCH_CHECK("normalize_frames");
  return 0;
}

extern "C" int nsm_sumsq(const float* g, int64_t n, float* partial, float* out, void* stream) {
  NSM_CHECK_ARG(g && partial && out && n > 0, "sumsq: bad args");
  int nb = nsm_loss_blocks(n);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(nb), dim3(256), 0, s, g, n, partial);
  hipLaunchKernelGGL(finalize_mean_kernel, dim3(1), dim3(64), 0, s, partial, nb, 1.0, out);
  NSM_LAUNCH_CHECK("sumsq");
  return 0;
}

extern "C" int nsm_clip_coef(const float* sumsq, float inv_world, float max_norm, float* coef,
                             void* stream) {
  NSM_CHECK_ARG(sumsq && coef, "clip_coef: bad args");
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, as_stream(stream), sumsq, inv_world,
                     max_norm, coef);
  NSM_LAUNCH_CHECK("clip_coef");
  return 0;
}

extern "C" int nsm_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                              float beta1, float beta2, float eps, float weight_decay, int step,
                              const float* gcoef, void* stream) {
  NSM_CHECK_ARG(p && g && m && v && n > 0 && step >= 1, "adamw: bad args");
  double bc1 = 1.0 - pow((double)beta1, step);
  double bc2 = 1.0 - pow((double)beta2, step);
  float step_size = (float)(lr / bc1);
  float bc2_sqrt = (float)sqrt(bc2);
  float decay = 1.f - lr * weight_decay;
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), p, g, m, v,
                     n, decay, beta1, beta2, eps, step_size, bc2_sqrt, gcoef);
  NSM_LAUNCH_CHECK("adamw");
  return 0;
}

// ===========================================================================
// VGG19 perceptual-loss feature stack (customLoss.py:7-90), forward only.
// ===========================================================================
// out[img][pixel][0..31]: channels 0-2 = (nan_to_num(clamp(v, 0, 1)) - mean) / denom
// (the 1-channel image repeated x3, customLoss.py:44-62), channels 3..31 = 0.
// Images 0..B-1 come from `a`, B..2B-1 from `b` (output and target batched).
__global__ void vgg_prep_kernel(const float* __restrict__ a, const float* __restrict__ b, int B,
                                long long HW, float mean, float denom, float* __restrict__ out) {
  long long total = 2ll * B * HW;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long half = (long long)B * HW;
    float v = i < half ? a[i] : b[i - half];
    // torch.clamp keeps NaN; nan_to_num(nan=0.5) then maps it (inf cannot survive the clamp)
    v = v != v ? 0.5f : fminf(fmaxf(v, 0.f), 1.f);
    const float n = (v - mean) / denom;
    f32x4* row = (f32x4*)(out + (size_t)i * 32);
    row[0] = f32x4{n, n, n, 0.f};
#pragma unroll
    for (int k = 1; k < 8; ++k) row[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// 2x2/2 max pool on NHWC (nn.MaxPool2d(2, 2), floor); NaN propagates as in ATen
__device__ __forceinline__ float nanmax(float m, float v) { return (v > m || v != v) ? v : m; }

__global__ void maxpool2_fwd_kernel(const float* __restrict__ x, int B, int H, int W, int C4,
                                    float* __restrict__ y) {
  const int Ho = H / 2, Wo = W / 2;
  long long total = (long long)B * Ho * Wo * C4;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < total; i += (long long)gridDim.x * blockDim.x) {
    int c = (int)(i % C4);
    long long t = i / C4;
    int ox = (int)(t % Wo);
    t /= Wo;
    int oy = (int)(t % Ho);
    int b = (int)(t / Ho);
    const float* base = x + (((size_t)b * H + 2 * oy) * W + 2 * ox) * (C4 * 4) + c * 4;
    size_t rs = (size_t)W * C4 * 4, cs = (size_t)C4 * 4;
    f32x4 m = *(const f32x4*)base;
    const f32x4 v1 = *(const f32x4*)(base + cs), v2 = *(const f32x4*)(base + rs),
                v3 = *(const f32x4*)(base + rs + cs);
    m.x = nanmax(nanmax(nanmax(m.x, v1.x), v2.x), v3.x);
    m.y = nanmax(nanmax(nanmax(m.y, v1.y), v2.y), v3.y);
    m.z = nanmax(nanmax(nanmax(m.z, v1.z), v2.z), v3.z);
    m.w = nanmax(nanmax(nanmax(m.w, v1.w), v2.w), v3.w);
    *(f32x4*)(y + (size_t)i * 4) = m;
  }
}

extern "C" int nsm_vgg_prep(const float* output, const float* target, int B, int H, int W,
                            float mean, float denom, float* out, void* stream) {
  NSM_CHECK_ARG(output && target && out && B > 0 && H > 0 && W > 0, "vgg_prep: bad args");
  long long work = 2ll * B * H * W;
  hipLaunchKernelGGL(vgg_prep_kernel, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), output,
                     target, B, (long long)H * W, mean, denom, out);
  NSM_LAUNCH_CHECK("vgg_prep");
  return 0;
}

extern "C" int nsm_maxpool2_fwd(const float* x, int B, int H, int W, int C, float* y,
                                void* stream) {
  NSM_CHECK_ARG(x && y && C % 4 == 0 && H >= 2 && W >= 2, "maxpool2_fwd: bad args");
  long long work = (long long)B * (H / 2) * (W / 2) * (C / 4);
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), x,
                     B, H, W, C / 4, y);
  NSM_LAUNCH_CHECK("maxpool2_fwd");
  return 0;
}
