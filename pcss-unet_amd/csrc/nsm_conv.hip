// MFMA implicit-GEMM convolutions for gfx950 (CDNA4), fp32 in / fp32 accumulate.
//
// One kernel template, three problems (NHWC activations, p = flattened pixel):
//   fwd   : y[p][co]  = sum_{tap,ci} x[p+off(tap)][ci] * Wf[co][tap][ci]       M=pixels N=co   K=9*ci
//   dgrad : dx[p][ci] = sum_{tap,co} dy[p+off(tap)][co] * Wd[ci][tap'][co]     (same kernel, flipped taps)
//   wgrad : dW[co][tap,ci] = sum_p dy[p][co] * x[p+off(tap)][ci]                M=co N=tap*ci K=pixels (split-K)
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact f32 fmaf chain, 64 FLOP/clk/SIMD,
// the fp32 peak of the chip). Each lane feeds ONE f32 of A and of B per MFMA:
// lane l supplies A[m=l&31][kk=l>>5] and B[kk=l>>5][n=l&31]. The K order inside
// a BK=32 slab is permuted so a lane's 16 k-values are contiguous in LDS:
// (half h, group j, step q) -> physical k = 16h + 4j + q. Both operands use the
// same permutation, so the contraction is unchanged (only fp rounding order).
//
// Operand LDS images (per pipeline stage):
//   MK: [rows][BK+4]  k contiguous, read with ds_read_b128 (4 k-steps per read);
//       the +4 pad makes the 16-lane groups of ds_read_b128 conflict-free.
//   KM: [BK][rows+4]  rows contiguous, read with ds_read_b32 (one k-step);
//       32 consecutive lanes -> 32 consecutive dwords: conflict-free.
// Global -> LDS staging goes through registers (float4 per lane, coalesced
// along channels), double-buffered: the next slab's global loads are issued
// before the current slab's MFMAs, and written to the other LDS stage after.
#include <type_traits>

#include "nsm_common.h"

namespace nsm {

constexpr int BK = 32;
constexpr int LDK = BK + 4;

// Branch-free operand loads: buffer_load_dwordx4 through a per-block resource
// descriptor whose base sits just below the block's lowest address; an
// invalid lane gets an offset past num_records and the hardware returns 0
// (zero padding / tails without exec-mask branches).
constexpr uint32_t OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, long long floats) {
  long long bytes = floats * 4;
  if (bytes > 0x7FFFFFFFll) bytes = 0x7FFFFFFFll;
  if (bytes < 0) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

// ---------------------------------------------------------------------------
// Operand loaders. R = rows of the operand tile (BM or BN), NT = threads.
// ---------------------------------------------------------------------------
struct ConvActP {  // im2col of NHWC activations; rows = pixels, K = (tap, channel)
  const float* x;
  int ld, cin, H, W, M, ksize;
  FastDiv fdW, fdH;
  const float* scale;  // prologue: lrelu(v*scale+shift)*mask on in-bounds pixels; halo stays 0
  const float* shift;
  const float* mask;
  int mask_ld, mask_on;
  float slope;
};

template <int R, int NT, bool PRO>
struct ConvActLoader {  // MK image
  static constexpr bool KM = false;
  static constexpr int NPT = R * (BK / 4) / NT;
  static constexpr int RSTEP = NT / (BK / 4);
  static constexpr int LDS_FLOATS = R * LDK;
  static_assert(NPT >= 1 && NPT * RSTEP == R, "loader shape");
  __amdgpu_buffer_rsrc_t rsrc;
  int rel[NPT];  // pixel index relative to the descriptor base
  int py[NPT], px[NPT], pb[NPT];
  int kc, row0, tap, c0;

  __device__ void init(const ConvActP& p, int m0, int kbeg, int tid, int) {
    kc = (tid & 7) * 4;
    row0 = tid >> 3;
    const int base_pix = max(0, m0 - p.W - 1);
    rsrc = make_rsrc(p.x + (size_t)base_pix * p.ld, (long long)(p.M - base_pix) * p.ld);
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      int q = m0 + row0 + i * RSTEP;
      bool v = q < p.M;
      q = v ? q : 0;
      int t = (int)fdiv((uint32_t)q, p.fdW);
      int xx = q - t * p.W;
      int b = (int)fdiv((uint32_t)t, p.fdH);
      int yy = t - b * p.H;
      rel[i] = q - base_pix;
      px[i] = xx;
      py[i] = v ? yy : -0x40000000;  // invalid rows never pass the bounds test
      pb[i] = b;
    }
    tap = kbeg / p.cin;
    c0 = kbeg - tap * p.cin;
  }
  __device__ void load(const ConvActP& p, f32x4* r) const {
    int dy = 0, dx = 0;
    if (p.ksize == 3) {
      dy = tap / 3 - 1;
      dx = tap - (tap / 3) * 3 - 1;
    }
    const int c = c0 + kc;
    const int shift = dy * p.W + dx;
    f32x4 sc, sh;
    if constexpr (PRO) {
      sc = *(const f32x4*)(p.scale + c);
      sh = *(const f32x4*)(p.shift + c);
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      int yy = py[i] + dy, xx = px[i] + dx;
      bool ok = ((unsigned)yy < (unsigned)p.H) & ((unsigned)xx < (unsigned)p.W);
      // OR-ing the OOB bit (not a select of two addresses) keeps this
      // straight-line: no exec-masked region splitting the K-loop block
      uint32_t off = ((uint32_t)((rel[i] + shift) * p.ld + c) * 4u) | (ok ? 0u : OOB);
      f32x4 v = bload4(rsrc, off);
      if constexpr (PRO) {
        f32x4 a;
        a.x = lrelu(v.x * sc.x + sh.x, p.slope);
        a.y = lrelu(v.y * sc.y + sh.y, p.slope);
        a.z = lrelu(v.z * sc.z + sh.z, p.slope);
        a.w = lrelu(v.w * sc.w + sh.w, p.slope);
        // mask always readable (host points it at `scale` with ld 0 when absent)
        const f32x4 mk = *(const f32x4*)(p.mask + (size_t)pb[i] * p.mask_ld + c);
        a *= p.mask_on ? mk : f32x4{1.f, 1.f, 1.f, 1.f};
        // rows past M only feed masked output rows, but keep them 0 anyway
        v = ok ? a : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      r[i] = v;
    }
  }
  __device__ void advance(const ConvActP& p) {
    c0 += BK;
    if (c0 >= p.cin) {
      c0 = 0;
      ++tap;
    }
  }
  __device__ void store(float* S, const f32x4* r) const {
#pragma unroll
    for (int i = 0; i < NPT; ++i) *(f32x4*)&S[(row0 + i * RSTEP) * LDK + kc] = r[i];
  }
};

struct RowsKP {  // dense rows with contiguous K (packed weights); rows >= nrows are zero
  const float* w;
  int ldw, nrows;
  long long bstride;  // floats between batch entries (Winograd: one GEMM per xi = blockIdx.z)
};

template <int R, int NT>
struct RowsKLoader {  // MK / NK image
  static constexpr bool KM = false;
  static constexpr int NPT = R * (BK / 4) / NT;
  static constexpr int RSTEP = NT / (BK / 4);
  static constexpr int LDS_FLOATS = R * LDK;
  static_assert(NPT >= 1 && NPT * RSTEP == R, "loader shape");
  __amdgpu_buffer_rsrc_t rsrc;
  int kc, row0, k0, n0;

  __device__ void init(const RowsKP& p, int n0_, int kbeg, int tid, int batch) {
    kc = (tid & 7) * 4;
    row0 = tid >> 3;
    k0 = kbeg;
    n0 = n0_;
    const float* base = p.w + (size_t)batch * p.bstride;
    rsrc = make_rsrc(base + (size_t)n0 * p.ldw, (long long)(p.nrows - n0) * p.ldw);
  }
  __device__ void load(const RowsKP& p, f32x4* r) const {
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      int row = row0 + i * RSTEP;
      uint32_t off = ((uint32_t)(row * p.ldw + k0 + kc) * 4u) | (n0 + row < p.nrows ? 0u : OOB);
      r[i] = bload4(rsrc, off);
    }
  }
  __device__ void advance(const RowsKP&) { k0 += BK; }
  __device__ void store(float* S, const f32x4* r) const {
#pragma unroll
    for (int i = 0; i < NPT; ++i) *(f32x4*)&S[(row0 + i * RSTEP) * LDK + kc] = r[i];
  }
};

struct PixRowsP {  // rows = pixels (the GEMM K of wgrad), columns contiguous channels
  const float* x;
  int ld, ncols;   // channel stride, valid columns (cp)
  int cin;         // channels per tap (N split into taps) — 0: no tap split
  int H, W, M, ksize;
  FastDiv fdW, fdH;
  const float* scale;  // prologue (1x1 wgrad B operand: recomputed BN+LReLU+dropout)
  const float* shift;
  const float* mask;
  int mask_ld, mask_on;
  float slope;
  long long bstride;  // batched GEMM: floats between batch entries
};

template <int R, int NT, bool SHIFT, bool PRO>
struct PixRowsLoader {  // KM / KN image
  static constexpr bool KM = true;
  static constexpr int C4 = R / 4;
  static constexpr int KSTEP = NT / C4;
  static constexpr int NPT = BK / KSTEP;
  static constexpr int LDS_FLOATS = BK * (R + 4);
  static_assert(NPT >= 1 && NPT * KSTEP == BK && KSTEP * C4 == NT, "loader shape");
  __amdgpu_buffer_rsrc_t rsrc;
  int col, c4o, krow0, k0, kend, dy, dx, base_pix;
  bool colok;
  f32x4 sc, sh;

  __device__ void init(const PixRowsP& p, int off, int kbeg, int kend_, int tid, int batch) {
    int c4 = tid % C4;
    c4o = c4 * 4;
    krow0 = tid / C4;
    // this thread's column (fixed over K) and, for the shifted operand, its
    // own tap: an N tile may span several taps when BN > Cin
    int tap = 0, c = off + c4 * 4;
    if (p.cin > 0) {
      tap = c / p.cin;
      c -= tap * p.cin;
    }
    col = c;
    colok = col < p.ncols && (p.cin == 0 || tap < p.ksize * p.ksize);
    dy = dx = 0;
    if (SHIFT && p.ksize == 3) {
      dy = tap / 3 - 1;
      dx = tap % 3 - 1;
    }
    k0 = kbeg;
    kend = kend_;
    base_pix = max(0, kbeg - p.W - 1);
    rsrc = make_rsrc(p.x + (size_t)batch * p.bstride + (size_t)base_pix * p.ld,
                     (long long)(p.M - base_pix) * p.ld);
    if constexpr (PRO) {
      sc = colok ? *(const f32x4*)(p.scale + col) : f32x4{0.f, 0.f, 0.f, 0.f};
      sh = colok ? *(const f32x4*)(p.shift + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ void load(const PixRowsP& p, f32x4* r) const {
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int q = k0 + krow0 + i * KSTEP;  // < 2^30 always: no guard needed for fdiv
      bool ok = colok & (q < kend);
      int b = 0;
      int src = q;
      if constexpr (SHIFT || PRO) {
        const int t = (int)fdiv((uint32_t)q, p.fdW);
        const int xx = q - t * p.W;
        b = (int)fdiv((uint32_t)t, p.fdH);
        const int yy = t - b * p.H;
        if constexpr (SHIFT) {
          ok = ok & ((unsigned)(yy + dy) < (unsigned)p.H) & ((unsigned)(xx + dx) < (unsigned)p.W);
          src = q + dy * p.W + dx;
        }
        if constexpr (PRO) b = ok ? b : 0;
      }
      uint32_t off = ((uint32_t)((src - base_pix) * p.ld + col) * 4u) | (ok ? 0u : OOB);
      f32x4 v = bload4(rsrc, off);
      if constexpr (PRO) {
        f32x4 a;
        a.x = lrelu(v.x * sc.x + sh.x, p.slope);
        a.y = lrelu(v.y * sc.y + sh.y, p.slope);
        a.z = lrelu(v.z * sc.z + sh.z, p.slope);
        a.w = lrelu(v.w * sc.w + sh.w, p.slope);
        const f32x4 mk = *(const f32x4*)(p.mask + (size_t)b * p.mask_ld + col);
        a *= p.mask_on ? mk : f32x4{1.f, 1.f, 1.f, 1.f};
        v = ok ? a : f32x4{0.f, 0.f, 0.f, 0.f};  // pixels past the split must add 0
      }
      r[i] = v;
    }
  }
  __device__ void advance(const PixRowsP&) { k0 += BK; }
  __device__ void store(float* S, const f32x4* r) const {
#pragma unroll
    for (int i = 0; i < NPT; ++i) *(f32x4*)&S[(krow0 + i * KSTEP) * (R + 4) + c4o] = r[i];
  }
};

// ---------------------------------------------------------------------------
// Fragment reads (see the K permutation in the file header).
// ---------------------------------------------------------------------------
template <bool KM, int R>
__device__ __forceinline__ void read_frag(const float* S, int rb, int lane, int j, float* f) {
  const int r = lane & 31, h = lane >> 5;
  if constexpr (!KM) {
    f32x4 v = *(const f32x4*)&S[(rb + r) * LDK + h * 16 + 4 * j];
    f[0] = v.x;
    f[1] = v.y;
    f[2] = v.z;
    f[3] = v.w;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = S[(h * 16 + 4 * j + q) * (R + 4) + rb + r];
  }
}

// ---------------------------------------------------------------------------
// Epilogues. acc[tm][tn] register i holds C[row][col] with
//   col = lane & 31, row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5).
// ---------------------------------------------------------------------------
struct EpiCtx {
  int m0, n0;  // block origin
  int mb, nb;  // this wave's tile origin
  int wm, wn, lane;
  float* lds;  // the GEMM's LDS array (free after the main loop)
  int mblk;    // M-block index (BN-partial row)
  int zslab;   // split-K / batch slab of EpiSlab (blockIdx.z unless remapped)
};

struct EpiStoreP {
  float* y;
  int ldy;
  const float* bias;
  float* stats;  // optional BN partials [gridDim.x][2][N]: {sum, M2 about block mean}
  long long bstride;  // batched GEMM (Winograd): output offset per blockIdx.z
  // optional eval-mode BN + LeakyReLU (+ skip) on the stored value:
  // y = lrelu((acc + bias) * act_scale + act_shift, slope) (+ res)
  const float* act_scale;
  const float* act_shift;
  float slope;
  const float* res;
  int ldres;
  int vec;  // 16-B row stores staged through LDS (NSM_F32_EPI_VEC=0: 4-byte stores)
};
struct EpiStore {
  using P = EpiStoreP;
  template <int TM, int TN, int WM, int WN>
  __device__ static void apply(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M, int N,
                               int) {
    const int col = cx.lane & 31, h = cx.lane >> 5;
    float* yb = e.y + (size_t)cx.zslab * e.bstride;  // store paths run with zsplit == 1
    float bv[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      int n = cx.nb + tn * 32 + col;
      bv[tn] = (e.bias && n < N) ? e.bias[n] : 0.f;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[tm][tn][i] += bv[tn];
    }
    if (e.vec && (e.ldy & 3) == 0 && (((uintptr_t)yb) & 15) == 0 &&
        (!e.res || ((e.ldres & 3) == 0 && (((uintptr_t)e.res) & 15) == 0))) {
      // each wave stages its tile as rows in LDS (stride WC + 4 floats: the two
      // row halves of a store land on different banks) and writes 16-B chunks
      constexpr int WR = TM * 32, WC = TN * 32, WCP = WC + 4, CPR = WC / 4;
      float* reg = cx.lds + (cx.wm * WN + cx.wn) * (WR * WCP);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            reg[(tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * WCP + tn * 32 + col] = acc[tm][tn][i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int it = 0; it < WR * CPR / 64; ++it) {
        const int q = it * 64 + cx.lane, r = q / CPR, cc = q - r * CPR;
        const int m = cx.mb + r, n = cx.nb + cc * 4;
        if (m >= M || n >= N) continue;
        f32x4 v = *(const f32x4*)&reg[r * WCP + cc * 4];
        if (e.act_scale) {
          const f32x4 a = *(const f32x4*)(e.act_scale + n), b = *(const f32x4*)(e.act_shift + n);
          v = v * a + b;
          v = f32x4{lrelu(v.x, e.slope), lrelu(v.y, e.slope), lrelu(v.z, e.slope),
                    lrelu(v.w, e.slope)};
          if (e.res) v += *(const f32x4*)(e.res + (size_t)m * e.ldres + n);
        }
        *(f32x4*)(yb + (size_t)m * e.ldy + n) = v;
      }
      if (!e.stats) return;
      __syncthreads();  // stats_only reuses the LDS
      stats_only<TM, TN, WM, WN>(e, acc, cx, M, N);
      return;
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      int n = cx.nb + tn * 32 + col;
      if (n >= N) continue;
      const float asc = e.act_scale ? e.act_scale[n] : 0.f;
      const float ash = e.act_scale ? e.act_shift[n] : 0.f;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          int m = cx.mb + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (m >= M) continue;
          float v = acc[tm][tn][i];
          if (e.act_scale) {
            v = lrelu(v * asc + ash, e.slope);
            if (e.res) v += e.res[(size_t)m * e.ldres + n];
          }
          yb[(size_t)m * e.ldy + n] = v;
        }
      }
    }
    if (!e.stats) return;
    stats_only<TM, TN, WM, WN>(e, acc, cx, M, N);
  }
  // fused BatchNorm batch statistics of this block's rows (two-pass); also
  // used by the bf16 store epilogue on its rounded values
  // RPP: rows per partial; a block of WM*TM*32 rows writes (WM*TM*32)/RPP
  // partial rows, each over its own group of M-waves
  template <int TM, int TN, int WM, int WN, int RPP = WM * TM * 32>
  __device__ static void stats_only(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M,
                                    int N) {
    const int col = cx.lane & 31, h = cx.lane >> 5;
    constexpr int BN = WN * TN * 32;
    constexpr int G = (WM * TM * 32) / RPP, WG = WM / G;
    static_assert(G >= 1 && G * RPP == WM * TM * 32 && WG * G == WM, "partial groups");
    float* red = cx.lds;  // [WM][BN]
    const int g = cx.wm / WG, w0 = g * WG;
    const int cnt = min(M - (cx.m0 + g * RPP), RPP);
    float s[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      float t = 0.f;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          int m = cx.mb + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          t += (m < M) ? acc[tm][tn][i] : 0.f;
        }
      t += __shfl_xor(t, 32, 64);
      s[tn] = t;
    }
    if (h == 0)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) red[cx.wm * BN + cx.wn * TN * 32 + tn * 32 + col] = s[tn];
    __syncthreads();
    float mean[TN], tot[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WG; ++w) t += red[(w0 + w) * BN + cx.wn * TN * 32 + tn * 32 + col];
      tot[tn] = t;
      mean[tn] = t / (float)cnt;
    }
    __syncthreads();
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      float t = 0.f;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          int m = cx.mb + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          float d = acc[tm][tn][i] - mean[tn];
          t += (m < M) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 32, 64);
      s[tn] = t;
    }
    if (h == 0)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) red[cx.wm * BN + cx.wn * TN * 32 + tn * 32 + col] = s[tn];
    __syncthreads();
    if (cx.wm == w0 && h == 0 && cnt > 0) {
      float* pr = e.stats + ((size_t)cx.mblk * G + g) * 2 * N;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        int n = cx.nb + tn * 32 + col;
        if (n >= N) continue;
        float q = 0.f;
#pragma unroll
        for (int w = 0; w < WG; ++w) q += red[(w0 + w) * BN + cx.wn * TN * 32 + tn * 32 + col];
        pr[n] = tot[tn];
        pr[N + n] = q;
      }
    }
  }
};

// BN-backward epilogue of the 1x1 input-gradient GEMM of a DoubleConv
// (g = dA1 = dY2 W2, the gradient wrt the activated output of the block's
// first BN; Unetmodel.py:22-26). With y = Y1 (that BN's input):
//   dz = g * lrelu'(y*scale + shift) * mask[b][c]
// mode 0: partials {sum dz, sum dz*(y-mean)*invstd} per row chunk (the
//         nsm_bn_bwd_reduce format; chunk = nsm_conv_stat_rows rows), g not stored
// mode 1: mode 0 and g stored (nsm_bn_bwd_apply then reads it)
// mode 2: dy = k1*dz + k2*(y-mean) + k3 stored (coef from nsm_bn_bwd_finalize)
// Modes 0 then 2 run the same GEMM twice, so dA1 never goes through HBM.
struct BnBwdEpiP {
  void* out;
  int ldo;
  const void* y;
  int ldy;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* invstd;
  const float* coef;
  const float* mask;  // [B][N] or null
  FastDiv fdHW;
  float slope;
  float* partial;  // [nchunk][2][N]
  int mode;
  uint32_t* amax = nullptr;  // mode 2 (fp32): max|dy| written (an h2 scale source)
  uint32_t* k1dz = nullptr;  // modes 0/1 (fp32): max|scale * dz| (the dy bound's k1 term)
};

__device__ __forceinline__ f32x4 lrelu_grad_v4(f32x4 z, float slope) {
  return f32x4{lrelu_grad(z.x, slope), lrelu_grad(z.y, slope), lrelu_grad(z.z, slope),
               lrelu_grad(z.w, slope)};
}
__device__ __forceinline__ f32x4 shfl_xor_v4(f32x4 v, int o) {
  return f32x4{__shfl_xor(v.x, o, 64), __shfl_xor(v.y, o, 64), __shfl_xor(v.z, o, 64),
               __shfl_xor(v.w, o, 64)};
}

// Each wave stages its accumulator tile as rows in LDS (row stride WC + 4
// floats: the two row halves of a store land on different banks), then every
// lane keeps ONE 4-column group and walks the rows with 16-B accesses: all Y1
// loads of the lane issue back to back, the accumulators are dead by then, so
// the epilogue adds no register pressure to the GEMM loop.
struct EpiBnBwd {
  using P = BnBwdEpiP;
  // Y1 rows of the wave tile, loaded before the GEMM's K loop (gemm_h2_kernel:
  // with the short K of most 1x1 input gradients the epilogue's Y1 read is the
  // kernel's main traffic; issued first, it overlaps the operand DMA instead of
  // following the MFMAs). Lane layout of apply's loop: one 4-column group
  // (lane % CPR) per lane, rows (it * 64 + lane) / CPR.
  template <int TM, int TN>
  struct PreT {
    static constexpr int NIT = TM * 32 * (TN * 32 / 4) / 64;
    f32x4 yv[NIT];
  };
  template <int TM, int TN, int WM, int WN>
  __device__ static void prefetch(const P& e, PreT<TM, TN>& pre, int mb, int nb, int lane, int M,
                                  int N) {
    constexpr int CPR = TN * 32 / 4;
    const int n = nb + (lane % CPR) * 4, nc = n < N ? n : 0;
    const float* __restrict__ Y = (const float*)e.y;
#pragma unroll
    for (int it = 0; it < PreT<TM, TN>::NIT; ++it) {
      const int m = min(mb + (it * 64 + lane) / CPR, M - 1);
      pre.yv[it] = *(const f32x4*)(Y + (size_t)m * e.ldy + nc);
    }
  }
  // LDS of the h2 GEMMs' epilogue (gemm_h2_kernel): the staged wave tiles, then
  // the [WM][2][BNT] partial rows
  template <int TM, int TN, int WM, int WN>
  static constexpr int lds_bytes() {
    constexpr int a = WM * WN * TM * 32 * (TN * 32 + 4) * 4, b = WM * 2 * WN * TN * 32 * 4;
    return a > b ? a : b;
  }
  template <int TM, int TN, int WM, int WN>
  __device__ static void apply(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M, int N,
                               int) {
    apply_impl<TM, TN, WM, WN>(e, acc, cx, M, N, nullptr);
  }
  template <int TM, int TN, int WM, int WN>
  __device__ static void apply_pre(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M,
                                   int N, const PreT<TM, TN>& pre) {
    apply_impl<TM, TN, WM, WN>(e, acc, cx, M, N, &pre);
  }
  template <int TM, int TN, int WM, int WN>
  __device__ static void apply_impl(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M,
                                    int N, const PreT<TM, TN>* pre) {
    const int col = cx.lane & 31, h = cx.lane >> 5;
    constexpr int BNT = WN * TN * 32, WR = TM * 32, WC = TN * 32, WCP = WC + 4;
    constexpr int CPR = WC / 4;  // 16-B chunks per row
    constexpr int NIT = WR * CPR / 64;
    static_assert(64 % CPR == 0, "a lane keeps one column group");
    float* reg = cx.lds + (cx.wm * WN + cx.wn) * (WR * WCP);
    __syncthreads();  // the GEMM's last LDS reads are done everywhere
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          reg[(tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * WCP + tn * 32 + col] = acc[tm][tn][i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float* __restrict__ Y = (const float*)e.y;
    float* __restrict__ O = (float*)e.out;
    const float* __restrict__ mk = e.mask;
    const bool red = e.mode != 2;
    const int cc = cx.lane % CPR, n = cx.nb + cc * 4;
    const bool nok = n < N;
    const int nc = nok ? n : 0;
    f32x4 yv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      if (pre) {
        yv[it] = pre->yv[it];
      } else {
        const int m = min(cx.mb + (it * 64 + cx.lane) / CPR, M - 1);
        yv[it] = *(const f32x4*)(Y + (size_t)m * e.ldy + nc);
      }
    }
    const f32x4 sc = *(const f32x4*)(e.scale + nc), sh = *(const f32x4*)(e.shift + nc),
                mu = *(const f32x4*)(e.mean + nc);
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    const f32x4 is = red ? *(const f32x4*)(e.invstd + nc) : zero;
    const f32x4 k1 = red ? zero : *(const f32x4*)(e.coef + nc),
                k2 = red ? zero : *(const f32x4*)(e.coef + N + nc),
                k3 = red ? zero : *(const f32x4*)(e.coef + 2 * N + nc);
    f32x4 s1 = zero, s2 = zero;
    uint32_t am = 0;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (it * 64 + cx.lane) / CPR, m = cx.mb + r;
      const bool ok = m < M && nok;
      const f32x4 g = *(const f32x4*)&reg[r * WCP + cc * 4], v = yv[it];
      f32x4 dz = g * lrelu_grad_v4(v * sc + sh, e.slope);
      if (mk) dz = dz * *(const f32x4*)(mk + (size_t)fdiv((uint32_t)min(m, M - 1), e.fdHW) * N + nc);
      if (!red) {
        if (ok) {
          const f32x4 d = k1 * dz + k2 * (v - mu) + k3;
          *(f32x4*)(O + (size_t)m * e.ldo + n) = d;
          amax_fold(am, d);
        }
      } else if (ok) {
        s1 += dz;
        s2 += dz * ((v - mu) * is);
        if (e.mode == 1) *(f32x4*)(O + (size_t)m * e.ldo + n) = g;
        if (e.k1dz) amax_fold(am, sc * dz);
      }
    }
    if (!red) {
      amax_flush(am, e.amax);
      return;
    }
    amax_flush(am, e.k1dz);
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
      s1 += shfl_xor_v4(s1, o);
      s2 += shfl_xor_v4(s2, o);
    }
    // one partial row per block (RPP = BM = nsm_conv_stat_rows): the waves of
    // one column range meet in LDS, fixed order
    __syncthreads();
    float* lds = cx.lds;  // [WM][2][BNT]
    if (cx.lane < CPR) {
      *(f32x4*)(lds + (cx.wm * 2) * BNT + cx.wn * WC + cc * 4) = s1;
      *(f32x4*)(lds + (cx.wm * 2 + 1) * BNT + cx.wn * WC + cc * 4) = s2;
    }
    __syncthreads();
    if (cx.wm == 0) {
      float* pr = e.partial + (size_t)cx.mblk * 2 * N;
      for (int j = cx.lane; j < 2 * WC; j += 64) {
        const int k = j / WC, c = j - k * WC, nn = cx.nb + c;
        if (nn >= N) continue;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) t += lds[(w * 2 + k) * BNT + cx.wn * WC + c];
        pr[k * N + nn] = t;
      }
    }
  }
};

struct EpiSlabP {
  float* ws;
  int vec;  // EpiSlabV: 16-B row stores staged through LDS
};
struct EpiSlab {
  using P = EpiSlabP;
  template <int TM, int TN, int WM, int WN>
  __device__ static void apply(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M, int N,
                               int split) {
    const int col = cx.lane & 31, h = cx.lane >> 5;
    const int mb = cx.mb, nb = cx.nb;
    float* out = e.ws + (size_t)cx.zslab * M * N;  // slab per (batch, split)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      int n = nb + tn * 32 + col;
      if (n >= N) continue;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          int m = mb + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (m < M) out[(size_t)m * N + n] = acc[tm][tn][i];
        }
      }
    }
  }
};

// EpiSlab with the LDS-staged 16-B row stores of EpiStore (fp32 weight-
// gradient kernels only: their two K-major stages, 64 x (BM + BN + 8) floats,
// hold the BM x BN tile unpadded — the +4 row pad of EpiStore would not fit at
// 128x128; the bf16 kernels' LDS holds neither, they keep EpiSlab)
struct EpiSlabV {
  using P = EpiSlabP;
  template <int TM, int TN, int WM, int WN>
  __device__ static void apply(const P& e, f32x16 (&acc)[TM][TN], const EpiCtx& cx, int M, int N,
                               int split) {
    float* out = e.ws + (size_t)cx.zslab * M * N;
    if (!e.vec || (N & 3) || (((uintptr_t)e.ws) & 15)) {
      EpiSlab::apply<TM, TN, WM, WN>(e, acc, cx, M, N, split);
      return;
    }
    const int col = cx.lane & 31, h = cx.lane >> 5;
    constexpr int WR = TM * 32, WC = TN * 32, CPR = WC / 4;
    float* reg = cx.lds + (cx.wm * WN + cx.wn) * (WR * WC);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          reg[(tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h) * WC + tn * 32 + col] = acc[tm][tn][i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < WR * CPR / 64; ++it) {
      const int q = it * 64 + cx.lane, r = q / CPR, cc = q - r * CPR;
      const int m = cx.mb + r, n = cx.nb + cc * 4;
      if (m < M && n < N) *(f32x4*)(out + (size_t)m * N + n) = *(const f32x4*)&reg[r * WC + cc * 4];
    }
  }
};

// ---------------------------------------------------------------------------
// The GEMM kernel: block tile BM x BN, WM x WN waves, each wave TM x TN 32x32
// MFMA tiles; grid (ceil(M/BM), ceil(N/BN), splits); split z covers
// K range [z*kchunk, min(K,(z+1)*kchunk)).
// ---------------------------------------------------------------------------
// LDS (2 stages, ~74 KB at 128x128) caps residency at 2 blocks per CU, i.e.
// <= 2 waves per SIMD for 256-thread blocks: tell the compiler so it spends
// registers on keeping LDS reads in flight instead of maximising occupancy.
template <int BM, int BN, int WM, int WN, class AL, class BL, class EP, class AP, class BP>
__global__ void __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(1, 2)))
    gemm_f32_kernel(AP ap, BP bp, typename EP::P ep, int M, int N, int K, int kchunk, int zsplit) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int A_SZ = AL::LDS_FLOATS, B_SZ = BL::LDS_FLOATS, STAGE = A_SZ + B_SZ;
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // blockIdx.z = batch * zsplit + split (batch: Winograd xi; split: split-K slice)
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int split = blockIdx.z % zsplit, batch = blockIdx.z / zsplit;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;

  AL a;
  BL b;
  if constexpr (AL::KM) a.init(ap, m0, kbeg, kend, tid, batch);
  else a.init(ap, m0, kbeg, tid, batch);
  if constexpr (BL::KM) b.init(bp, n0, kbeg, kend, tid, batch);
  else b.init(bp, n0, kbeg, tid, batch);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  f32x4 ar[AL::NPT], br[BL::NPT];
  if (nk > 0) {
    a.load(ap, ar);
    b.load(bp, br);
    a.store(lds, ar);
    b.store(lds + A_SZ, br);
  }
  __syncthreads();

  const int arb = wm * TM * 32, brb = wn * TN * 32;
  // One basic block per K-slab: the next slab's loads are issued
  // unconditionally (on the last slab they hit the zero-fill / stay inside the
  // descriptor range and land in the idle LDS stage), so the scheduler can
  // interleave them, the LDS fragment reads and the MFMAs freely; the
  // sched_group_barrier sequence below pins that interleave.
  for (int it = 0; it < nk; ++it) {
    const float* As = lds + (it & 1) * STAGE;
    const float* Bs = As + A_SZ;
    a.advance(ap);
    b.advance(bp);
    float fa[2][TM][4], fb[2][TN][4];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) read_frag<AL::KM, BM>(As, arb + tm * 32, lane, 0, fa[0][tm]);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) read_frag<BL::KM, BN>(Bs, brb + tn * 32, lane, 0, fb[0][tn]);
    a.load(ap, ar);
    b.load(bp, br);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cur = j & 1;
      if (j < 3) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          read_frag<AL::KM, BM>(As, arb + tm * 32, lane, j + 1, fa[cur ^ 1][tm]);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          read_frag<BL::KM, BN>(Bs, brb + tn * 32, lane, j + 1, fb[cur ^ 1][tn]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[cur][tm][q], fb[cur][tn][q],
                                                               acc[tm][tn], 0, 0, 0);
    }
    float* An = lds + ((it + 1) & 1) * STAGE;
    a.store(An, ar);
    b.store(An + A_SZ, br);
    // ---- pinned interleave (LLVM SchedGroupMask: VALU 0x2, MFMA 0x8,
    //      VMEM_READ 0x20, DS_READ 0x100, DS_WRITE 0x200) ----
    constexpr int NMF = 4 * TM * TN;               // MFMAs per fragment group
    constexpr int NLD = AL::NPT + BL::NPT;         // global loads per slab
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // group-0 fragments
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int m = 0; m < NMF; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (j == 0 && m < NLD) {
          __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        if (j < 3 && m < 8) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x200, 16, 0);
    __syncthreads();
  }
  EpiCtx cx{m0, n0, m0 + arb, n0 + brb, wm, wn, lane, lds, (int)blockIdx.x, (int)blockIdx.z};
  EP::template apply<TM, TN, WM, WN>(ep, acc, cx, M, N, split);
}

#include "nsm_conv_split.inc"

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
// amax: the operands' maxima (f16x2 split); a prologue (PRO) transforms the
// operand after its producer recorded the maximum, so it runs the bf16 split
template <int BM, int BN, int WM, int WN, bool PRO, class EP = EpiStore>
static int launch_conv_fwd(const ConvActP& ap, const RowsKP& bp, const typename EP::P& ep, int M,
                           int N, int K, hipStream_t s, AmaxPair amax = AmaxPair{}) {
  constexpr int NT = WM * WN * 64;
  using AL = ConvActLoader<BM, NT, PRO>;
  using BL = RowsKLoader<BN, NT>;
  dim3 grid(ceil_div(M, BM), ceil_div(N, BN), 1);
  launch_f32_gemm<BM, BN, WM, WN, AL, BL, EP, ConvActP, RowsKP>(grid, s, ap, bp, ep, M, N, K, K, 1,
                                                                PRO ? AmaxPair{} : amax);
  NSM_LAUNCH_CHECK("conv_fwd");
  return 0;
}

// BM chosen by dispatch_conv_fwd (rows per BN-stat partial)
// 256-row tiles (4 waves of 64x32: 0.75 fragment reads per MFMA instead of
// 1) for the 32-channel fp32 convs with >= 2048 of them (conv2 at 256^2):
// conv2.0 fwd 127 -> 112 us, its dgrad 117 -> 101 us (NSM_N32_BM256=0: 128)
static bool n32_bm256() {
  static bool v = [] {
    const char* e = getenv("NSM_N32_BM256");
    return !e || atoi(e) != 0;
  }();
  return v;
}
// 256x64 tiles (4 waves of 64x64) for the 64-channel fp32 convs with >= 2048
// of them (conv2.4, conv8.4 at 256^2 and their input gradients): 118.5 ->
// 101.9, 78 -> 66-70, 59 -> 55 us per launch (NSM_N64_BM256=0: 128x64)
static bool n64_bm256() {
  static bool v = [] {
    const char* e = getenv("NSM_N64_BM256");
    return !e || atoi(e) != 0;
  }();
  return v;
}
static int conv_fwd_bm(long long M, int N) {
  long long mb128 = ceil_div(M, 128);
  if (N >= 128) return mb128 * ceil_div(N, 128) >= 512 ? 128 : 64;
  if (N >= 64) return mb128 * ceil_div(N, 64) >= 512 ? 128 : 64;
  return mb128 >= 512 ? 128 : 64;
}
// rows per BN-partial row of the fp32 direct-conv dispatch (dispatch_conv_fwd)
static int conv_fwd_bm_f(long long M, int N) {
  if (N < 64 && n32_bm256() && ceil_div(M, 128) >= 4096) return 256;
  if (N == 64 && n64_bm256() && ceil_div(M, 128) >= 4096) return 256;
  return conv_fwd_bm(M, N);
}

template <bool PRO, class EP = EpiStore>
static int dispatch_conv_fwd(const ConvActP& ap, const RowsKP& bp, const typename EP::P& ep, int M,
                             int N, int K, hipStream_t s, AmaxPair amax = AmaxPair{}) {
  // Tile choice: 128x128 (2x2 waves of 64x64) wherever N allows; narrower N
  // tiles for the 32/64-channel layers; BM=64 when the grid would not cover
  // the 256 CUs twice.
  long long mb128 = ceil_div(M, 128);
  if (N >= 128) {
    if (mb128 * ceil_div(N, 128) >= 512)
      return launch_conv_fwd<128, 128, 2, 2, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
    return launch_conv_fwd<64, 128, 2, 2, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
  }
  if (N >= 64) {
    if (n64_bm256() && mb128 >= 4096 && N == 64)
      return launch_conv_fwd<256, 64, 4, 1, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
    if (mb128 * ceil_div(N, 64) >= 512)
      return launch_conv_fwd<128, 64, 2, 2, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
    return launch_conv_fwd<64, 64, 2, 2, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
  }
  if (n32_bm256() && mb128 >= 4096)
    return launch_conv_fwd<256, 32, 4, 1, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
  if (mb128 >= 512) return launch_conv_fwd<128, 32, 4, 1, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
  return launch_conv_fwd<64, 32, 2, 1, PRO, EP>(ap, bp, ep, M, N, K, s, amax);
}

template <int BM, int BN, int WM, int WN, bool SHIFT, bool PRO>
static int launch_wgrad(const PixRowsP& ap, const PixRowsP& bp, const EpiSlabP& ep, int M, int N,
                        int K, int kchunk, int splits, hipStream_t s, AmaxPair amax) {
  constexpr int NT = WM * WN * 64;
  using AL = PixRowsLoader<BM, NT, false, false>;
  using BL = PixRowsLoader<BN, NT, SHIFT, PRO>;
  dim3 grid(ceil_div(M, BM), ceil_div(N, BN), splits);
  launch_f32_gemm<BM, BN, WM, WN, AL, BL, EpiSlabV, PixRowsP, PixRowsP>(grid, s, ap, bp, ep, M, N, K,
                                                                        kchunk, splits,
                                                                        PRO ? AmaxPair{} : amax);
  NSM_LAUNCH_CHECK("conv_wgrad");
  return 0;
}

template <bool SHIFT, bool PRO>
static int dispatch_wgrad(int BM, int BN, const PixRowsP& ap, const PixRowsP& bp,
                          const EpiSlabP& ep, int M, int N, int K, int kchunk, int splits,
                          hipStream_t s, AmaxPair amax = AmaxPair{}) {
#define NSM_WG(bm, bn, wm, wn) \
  if (BM == bm && BN == bn)    \
    return launch_wgrad<bm, bn, wm, wn, SHIFT, PRO>(ap, bp, ep, M, N, K, kchunk, splits, s, amax);
  NSM_WG(128, 128, 2, 2)
  NSM_WG(128, 64, 2, 2)
  NSM_WG(128, 32, 4, 1)
  NSM_WG(64, 128, 2, 2)
  NSM_WG(64, 64, 2, 2)
  NSM_WG(64, 32, 2, 1)
  NSM_WG(32, 128, 1, 4)
  NSM_WG(32, 64, 1, 2)
  NSM_WG(32, 32, 1, 1)
#undef NSM_WG
  return fail(NSM_E_ARG, "wgrad: no tile %dx%d", BM, BN);
}

struct WgradPlan {
  int BM, BN, splits, kchunk;
  size_t ws_floats;
};

// NSM_WGRAD_MULTITAP=0: one tap per weight-gradient N tile (register kernels)
static bool wgrad_multitap_f32() {
  static bool v = [] {
    const char* e = getenv("NSM_WGRAD_MULTITAP");
    return !e || atoi(e) != 0;
  }();
  return v;
}

static WgradPlan plan_wgrad(int B, int H, int W, int cin_p, int cout_p, int ksize) {
  WgradPlan pl;
  const int M = cout_p, N = ksize * ksize * cin_p;
  const long long K = (long long)B * H * W;
  pl.BM = cout_p >= 128 ? 128 : (cout_p >= 64 ? 64 : 32);
  // 3x3 with Cin < 128: N tiles of 128 columns spanning 2 (Cin 64) or 4
  // (Cin 32) taps: wider waves, the dy operand shared by more columns
  pl.BN = cin_p >= 128 || (ksize == 3 && wgrad_multitap_f32()) ? 128
                                                                : (cin_p >= 64 ? 64 : 32);
  long long tiles = (long long)ceil_div(M, pl.BM) * ceil_div(N, pl.BN);
  // ~512 blocks (one round of 2 blocks/CU; A/B 4096 / 1024 / 512: 657 / 663 / 665
  // frames/s); each split keeps >= 8 K-slabs,
  // and the fp32 partial slabs stay <= 512 MB. (4096 blocks, the round-1
  // policy, made the 1x1 weight gradients of the wide layers write and re-read
  // more partial slabs than operands: conv6.4 128 splits x 2 MB = 268 MB.)
  static const long long target = [] {
    const char* e = getenv("NSM_WGRAD_BLOCKS");
    return e ? atoll(e) : 512ll;
  }();
  // rounded DOWN: a grid just past the resident slots runs a second round for
  // its last few blocks (conv2.0's 3 N tiles x 171 = 513 blocks took 151.6 us)
  long long want = target / tiles;
  if (want < 1) want = 1;
  long long maxs = (K + 255) / 256;
  long long slab_cap = (128ll << 20) / ((long long)M * N);
  if (slab_cap < 1) slab_cap = 1;
  long long sp = want < maxs ? want : maxs;
  if (sp > slab_cap) sp = slab_cap;
  if (sp > 512) sp = 512;
  if (sp < 1) sp = 1;
  long long kc = (K + sp - 1) / sp;
  kc = (kc + BK - 1) / BK * BK;
  sp = (K + kc - 1) / kc;
  pl.splits = (int)sp;
  pl.kchunk = (int)kc;
  pl.ws_floats = (size_t)sp * M * N;
  if (sp > 16) pl.ws_floats += (size_t)((sp + 15) / 16) * M * N;  // stage-1 sums
  return pl;
}

// dw[co][ci][tap] (real dims) = sum_s ws[s][co][tap*cin_p + ci].
// Block = one output channel co x 64 input channels: split-K partials are read
// coalesced along ci (GEMM layout), summed in a fixed order, transposed through
// LDS, and written as one contiguous [64][taps] run of the reference layout.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, int splits,
                                                           int M, int N, int cin_p, int taps,
                                                           int cin, int cout,
                                                           float* __restrict__ dw) {
  __shared__ float tile[64 * 9];
  const int co = blockIdx.y, ci0 = blockIdx.x * 64;
  const int nci = min(64, cin - ci0);
  const size_t MN = (size_t)M * N;
  for (int i = threadIdx.x; i < 64 * taps; i += 256) {
    int tap = i / 64, cl = i % 64;
    float s = 0.f;
    if (cl < nci) {  // four splits' loads in flight (fixed order: deterministic)
      const float* src = ws + (size_t)co * N + tap * cin_p + ci0 + cl;
      float s1 = 0.f, s2 = 0.f, s3 = 0.f;
      int k = 0;
      for (; k + 3 < splits; k += 4) {
        s += src[k * MN];
        s1 += src[(k + 1) * MN];
        s2 += src[(k + 2) * MN];
        s3 += src[(k + 3) * MN];
      }
      for (; k < splits; ++k) s += src[k * MN];
      s = (s + s1) + (s2 + s3);
    }
    tile[cl * taps + tap] = s;
  }
  __syncthreads();
  float* dst = dw + ((size_t)co * cin + ci0) * taps;
  for (int j = threadIdx.x; j < nci * taps; j += 256) dst[j] = tile[j];
}

// First reduction stage for many splits: dst[g][i] = sum of src[s][i] over the
// splits s in group g (16 per group), float4 per thread, fixed order.
__global__ void __launch_bounds__(256) splitsum_kernel(const float* __restrict__ src, int splits,
                                                       long long L4, int per,
                                                       float* __restrict__ dst) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= L4) return;
  const int g = blockIdx.y;
  const int s0 = g * per, s1 = min(splits, s0 + per);
  const f32x4* p = (const f32x4*)src + i;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + 1 < s1; s += 2) {
    a += p[(size_t)s * L4];
    b += p[(size_t)(s + 1) * L4];
  }
  if (s < s1) a += p[(size_t)s * L4];
  ((f32x4*)dst)[(size_t)g * L4 + i] = a + b;
}

// split-K slabs -> dw (reference layout): optional 16-way first stage, then
// the transposing reduction
static int wgrad_finish(float* ws, const WgradPlan& pl, int M, int N, int cin_p, int taps, int cin,
                        int cout, float* dw, hipStream_t s) {
  const float* red_src = ws;
  int red_splits = pl.splits;
  if (pl.splits > 16) {
    const int per = 16, groups = ceil_div(pl.splits, per);
    long long L4 = (long long)M * N / 4;
    float* stage = ws + (size_t)pl.splits * M * N;
    hipLaunchKernelGGL(splitsum_kernel, dim3(ceil_div(L4, 256), groups), dim3(256), 0, s, ws,
                       pl.splits, L4, per, stage);
    NSM_LAUNCH_CHECK("conv_wgrad splitsum");
    red_src = stage;
    red_splits = groups;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(ceil_div(cin, 64), cout), dim3(256), 0, s, red_src,
                     red_splits, M, N, cin_p, taps, cin, cout, dw);
  NSM_LAUNCH_CHECK("conv_wgrad reduce");
  return 0;
}

__global__ void pack_weight_kernel(const float* __restrict__ w, int cout, int cin, int taps,
                                   int cout_p, int cin_p, int mode, float* __restrict__ out) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  int total = cout_p * cin_p * taps;
  if (idx >= total) return;
  if (mode == NSM_PACK_FWD) {  // out[co][tap][ci]
    int ci = idx % cin_p;
    int t = idx / cin_p;
    int tap = t % taps;
    int co = t / taps;
    out[idx] = (co < cout && ci < cin) ? w[((size_t)co * cin + ci) * taps + tap] : 0.f;
  } else {  // out[ci][tap'][co] = w[co][ci][taps-1-tap']
    int co = idx % cout_p;
    int t = idx / cout_p;
    int tap = t % taps;
    int ci = t / taps;
    out[idx] =
        (co < cout && ci < cin) ? w[((size_t)co * cin + ci) * taps + (taps - 1 - tap)] : 0.f;
  }
}

__global__ void pad_vec_kernel(const float* __restrict__ v, int n, int n_p, float* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_p) out[i] = i < n ? v[i] : 0.f;
}

// ===========================================================================
// Winograd F(m x m, 3x3), m in {2, 4}, for the deep 3x3 convolutions
// (forward, dgrad and wgrad). alpha = m + 2, tiles t = (b, ty, tx) of m x m outputs:
//   V[xi][t][c]  = (B^T d B)     input tile d = alpha x alpha window at (m ty-1, m tx-1)
//   U[xi][n][k]  = (G g G^T)     g = 3x3 filter of (out n, in k)
//   M[xi][t][n]  = sum_k V[xi][t][k] U[xi][n][k]   (alpha^2 batched MFMA GEMMs)
//   Y(m x m)     = A^T M A  (+ bias)
// F(2x2): 16 GEMMs per 4 outputs (2.25x fewer MFMA flops than direct);
// F(4x4): 36 per 16 (4x fewer). Matrices: exact Cook-Toom tables generated by
// tools/wino_coeffs.py (F(4x4) uses points 0, 1, -1, 1/2, -2 for lower fp32 error).
// ===========================================================================
// Bounds of the Winograd transforms, (max_i sum_j |T_ij|)^2 rounded up:
// which 0 = the input transform B^T d B, 1 = the output-gradient transform
// A dY A^T, 2 = the filter transform G g G^T. max|transform| <= beta * max|in|
// (the h2 operands' scale source, nsm_conv_h2.inc)
__host__ __device__ constexpr float wino_beta(int tile, int which) {
  return which == 0   ? (tile == 6 ? 225.f : tile == 4 ? 49.f : 4.f)
         : which == 1 ? (tile == 6 ? 3969.f : tile == 4 ? 225.f : 4.f)
                      : (tile == 6 ? 1.5625f : tile == 4 ? 3.5f : 2.25f);
}
template <int MT> struct WinoMats;
template <> struct WinoMats<2> {
  static constexpr int A = 4;
  __device__ static constexpr float at(int i, int j) {
    constexpr float t[2][4] = {{1.f, 1.f, 1.f, 0.f}, {0.f, 1.f, -1.f, 1.f}};
    return t[i][j];
  }
  __device__ static constexpr float g(int i, int j) {
    constexpr float t[4][3] = {{-1.f, 0.f, 0.f}, {0.5f, 0.5f, 0.5f}, {0.5f, -0.5f, 0.5f},
                               {0.f, 0.f, 1.f}};
    return t[i][j];
  }
  __device__ static constexpr float bt(int i, int j) {
    constexpr float t[4][4] = {{-1.f, 0.f, 1.f, 0.f}, {0.f, 1.f, 1.f, 0.f},
                               {0.f, -1.f, 1.f, 0.f}, {0.f, -1.f, 0.f, 1.f}};
    return t[i][j];
  }
};
template <> struct WinoMats<4> {
  static constexpr int A = 6;
  __device__ static constexpr float at(int i, int j) {
    constexpr float t[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                               {0.f, 1.f, -1.f, 0.5f, -2.f, 0.f},
                               {0.f, 1.f, 1.f, 0.25f, 4.f, 0.f},
                               {0.f, 1.f, -1.f, 0.125f, -8.f, 1.f}};
    return t[i][j];
  }
  __device__ static constexpr float g(int i, int j) {
    constexpr float t[6][3] = {{1.f, 0.f, 0.f},
                               {1.f / 3, 1.f / 3, 1.f / 3},
                               {-1.f / 3, 1.f / 3, -1.f / 3},
                               {-16.f / 15, -8.f / 15, -4.f / 15},
                               {1.f / 15, -2.f / 15, 4.f / 15},
                               {0.f, 0.f, 1.f}};
    return t[i][j];
  }
  __device__ static constexpr float bt(int i, int j) {
    constexpr float t[6][6] = {{1.f, -1.5f, -2.f, 1.5f, 1.f, 0.f},
                               {0.f, -1.f, 0.5f, 2.5f, 1.f, 0.f},
                               {0.f, 1.f, -2.5f, 0.5f, 1.f, 0.f},
                               {0.f, -2.f, -1.f, 2.f, 1.f, 0.f},
                               {0.f, 0.5f, -1.f, -0.5f, 1.f, 0.f},
                               {0.f, 1.f, -1.5f, -2.f, 1.5f, 1.f}};
    return t[i][j];
  }
};
// F(6x6): points 0, +-1, +-2, +-1/2 (+inf): 64 GEMMs per 36 outputs (5.06x
// fewer MFMA flops than direct); fp32 error 8.8e-6 rms vs 2.9e-6 for F(4x4)
// on a 512-channel layer with O(1) outputs (tools/wino_coeffs.py)
template <> struct WinoMats<6> {
  static constexpr int A = 8;
  __device__ static constexpr float at(int i, int j) {
    constexpr float t[6][8] = {
        {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
        {0.f, 1.f, -1.f, 2.f, -2.f, 0.5f, -0.5f, 0.f},
        {0.f, 1.f, 1.f, 4.f, 4.f, 0.25f, 0.25f, 0.f},
        {0.f, 1.f, -1.f, 8.f, -8.f, 0.125f, -0.125f, 0.f},
        {0.f, 1.f, 1.f, 16.f, 16.f, 0.0625f, 0.0625f, 0.f},
        {0.f, 1.f, -1.f, 32.f, -32.f, 0.03125f, -0.03125f, 1.f}};
    return t[i][j];
  }
  __device__ static constexpr float g(int i, int j) {
    constexpr float t[8][3] = {{-1.f, 0.f, 0.f},
                               {-2.f / 9, -2.f / 9, -2.f / 9},
                               {-2.f / 9, 2.f / 9, -2.f / 9},
                               {1.f / 90, 2.f / 90, 4.f / 90},
                               {1.f / 90, -2.f / 90, 4.f / 90},
                               {32.f / 45, 16.f / 45, 8.f / 45},
                               {32.f / 45, -16.f / 45, 8.f / 45},
                               {0.f, 0.f, 1.f}};
    return t[i][j];
  }
  __device__ static constexpr float bt(int i, int j) {
    constexpr float t[8][8] = {{-1.f, 0.f, 5.25f, 0.f, -5.25f, 0.f, 1.f, 0.f},
                               {0.f, 1.f, 1.f, -4.25f, -4.25f, 1.f, 1.f, 0.f},
                               {0.f, -1.f, 1.f, 4.25f, -4.25f, -1.f, 1.f, 0.f},
                               {0.f, 0.5f, 0.25f, -2.5f, -1.25f, 2.f, 1.f, 0.f},
                               {0.f, -0.5f, 0.25f, 2.5f, -1.25f, -2.f, 1.f, 0.f},
                               {0.f, 2.f, 4.f, -2.5f, -5.f, 0.5f, 1.f, 0.f},
                               {0.f, -2.f, 4.f, 2.5f, -5.f, -0.5f, 1.f, 0.f},
                               {0.f, -1.f, 0.f, 5.25f, 0.f, -5.25f, 0.f, 1.f}};
    return t[i][j];
  }
};
// per-thread channel vector of the transform kernels: 4 channels (f32x4) for
// F(2x2)/F(4x4); one for F(6x6), whose 8x8 tiles would not fit in registers x4
template <int MT> struct WinoVec {
  using T = f32x4;
  static constexpr int W = 4;
};
template <> struct WinoVec<6> {
  using T = float;
  static constexpr int W = 1;
};
__device__ __forceinline__ float vlrelu(float v, float s) { return lrelu(v, s); }
__device__ __forceinline__ f32x4 vlrelu(f32x4 v, float s) {
  return f32x4{lrelu(v.x, s), lrelu(v.y, s), lrelu(v.z, s), lrelu(v.w, s)};
}
__device__ __forceinline__ f32x2 vlrelu(f32x2 v, float s) { return f32x2{lrelu(v.x, s), lrelu(v.y, s)}; }
__device__ __forceinline__ float vrelu(float v) { return fmaxf(v, 0.f); }
__device__ __forceinline__ f32x4 vrelu(f32x4 v) {
  return f32x4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
}
// coefficient views: c(i, j) of B^T, A^T, G and the transposes used by the gradients
template <int MT> struct CBt { __device__ static constexpr float c(int i, int j) { return WinoMats<MT>::bt(i, j); } };
template <int MT> struct CAt { __device__ static constexpr float c(int i, int j) { return WinoMats<MT>::at(i, j); } };
template <int MT> struct CA  { __device__ static constexpr float c(int i, int j) { return WinoMats<MT>::at(j, i); } };
template <int MT> struct CG  { __device__ static constexpr float c(int i, int j) { return WinoMats<MT>::g(i, j); } };
template <int MT> struct CGt { __device__ static constexpr float c(int i, int j) { return WinoMats<MT>::g(j, i); } };

// y[i] = sum_j C(i, j) x[j] over the nonzero compile-time coefficients (after
// unrolling every coefficient is a constant: zeros vanish, +-1 become moves/negations)
__device__ __forceinline__ float vfma(float c, float x, float a) { return __builtin_fmaf(c, x, a); }
__device__ __forceinline__ f32x4 vfma(float c, f32x4 x, f32x4 a) {
  return __builtin_elementwise_fma(f32x4{c, c, c, c}, x, a);
}
__device__ __forceinline__ f32x2 vfma(float c, f32x2 x, f32x2 a) {
  return __builtin_elementwise_fma(f32x2{c, c}, x, a);
}

template <class C, int NO, int NI, typename T>
__device__ __forceinline__ void wmat(const T (&x)[NI], T (&y)[NO]) {
  // every rounding spelled out (fma where |c| != 1, no contraction left to the
  // compiler): the same transform inlined into different kernels gives the
  // same bits (tests/test_gpu_ops.py: dual transform == separate transforms)
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    T acc{};
    bool first = true;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const float c = C::c(i, j);
      if (c == 0.f) continue;
      if (first) acc = c == 1.f ? x[j] : (c == -1.f ? -x[j] : c * x[j]);
      else if (c == 1.f) acc = acc + x[j];
      else if (c == -1.f) acc = acc - x[j];
      else acc = vfma(c, x[j], acc);
      first = false;
    }
    y[i] = acc;
  }
}

// Y = C X C^T for a square tile X[NI][NI] -> Y[NO][NO]
template <class C, int NO, int NI, typename T>
__device__ __forceinline__ void wmat2(const T (&x)[NI][NI], T (&y)[NO][NO]) {
  T s[NO][NI];
#pragma unroll
  for (int e = 0; e < NI; ++e) {
    T col[NI], r[NO];
#pragma unroll
    for (int j = 0; j < NI; ++j) col[j] = x[j][e];
    wmat<C>(col, r);
#pragma unroll
    for (int i = 0; i < NO; ++i) s[i][e] = r[i];
  }
#pragma unroll
  for (int i = 0; i < NO; ++i) wmat<C>(s[i], y[i]);
}

// wmat2's column pass fed one input row at a time: s[i][e] accumulates
// C(i, a) x[a][e] over the rows a in increasing order with wmat's exact
// operation sequence (first nonzero term, then +, - or fma), so streaming a
// tile's rows gives wmat2's bits while one row, not the tile, is live (the
// F(6x6) input transform with the x2 upsample held 220 VGPRs = 2 waves / SIMD)
template <class C, int NI>
__device__ constexpr int wfirst(int i) {
  for (int j = 0; j < NI; ++j)
    if (C::c(i, j) != 0.f) return j;
  return NI;
}
template <class C, int NO, int NI, typename T>
__device__ __forceinline__ void wcol_row(T (&s)[NO][NI], const T (&row)[NI], int a) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    const float c = C::c(i, a);
    if (c == 0.f) continue;
    const bool first = a == wfirst<C, NI>(i);
#pragma unroll
    for (int e = 0; e < NI; ++e) {
      if (first) s[i][e] = c == 1.f ? row[e] : (c == -1.f ? -row[e] : c * row[e]);
      else if (c == 1.f) s[i][e] = s[i][e] + row[e];
      else if (c == -1.f) s[i][e] = s[i][e] - row[e];
      else s[i][e] = vfma(c, row[e], s[i][e]);
    }
  }
}

template <int MT>
__global__ void wino_weight_kernel(const float* __restrict__ w, int cout, int cin, int n_p, int k_p,
                                   int flip, float* __restrict__ U) {
  constexpr int A = MT + 2;
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_p * k_p) return;
  const int k = idx % k_p, n = idx / k_p;
  // fwd: n = co, k = ci, g = w[co][ci];  dgrad: n = ci, k = co, g = rot180(w[co][ci])
  const int co = flip ? k : n, ci = flip ? n : k;
  float g[3][3];
  const bool ok = co < cout && ci < cin;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int sa = flip ? 2 - a : a, sb = flip ? 2 - b : b;
      g[a][b] = ok ? w[((size_t)co * cin + ci) * 9 + sa * 3 + sb] : 0.f;
    }
  float u[A][A];
  wmat2<CG<MT>>(g, u);
  const size_t plane = (size_t)n_p * k_p;
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int b = 0; b < A; ++b) U[(a * A + b) * plane + (size_t)n * k_p + k] = u[a][b];
}

// components i*A .. i*A+A-1 (row i of the transform) of tile t, channel(s)
// c.. of one thread into an h2 tensor [alpha^2][T][2C]
template <int A, typename VT>
__device__ __forceinline__ void h2_write_row(bf16_t* __restrict__ out, long long T, int C,
                                             long long t, int c, int i, const VT (&v)[A], float s) {
  const size_t plane2 = (size_t)T * 2 * C;
  bf16_t* row = out + (size_t)t * 2 * C + (size_t)(i * A) * plane2;
#pragma unroll
  for (int e = 0; e < A; ++e) {
    if constexpr (std::is_same<VT, float>::value)
      *(uint32_t*)(row + e * plane2 + h2_pair_off(c)) = h2_pair_word(v[e], s);
    else
      h2_store4(row + e * plane2, c, v[e], s);
  }
}

// the alpha x alpha transform values of tile t, channel(s) c.. of one thread
// into an h2 tensor [alpha^2][T][2C] (one channel per thread: lane pairs
// exchange terms, h2_pair_word; four: h2_store4)
template <int A, typename VT>
__device__ __forceinline__ void h2_write(bf16_t* __restrict__ out, long long T, int C, long long t,
                                         int c, const VT (&v)[A][A], float s) {
  const size_t plane2 = (size_t)T * 2 * C;
  bf16_t* row = out + (size_t)t * 2 * C;
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int e = 0; e < A; ++e) {
      if constexpr (std::is_same<VT, float>::value)
        *(uint32_t*)(row + (a * A + e) * plane2 + h2_pair_off(c)) = h2_pair_word(v[a][e], s);
      else
        h2_store4(row + (a * A + e) * plane2, c, v[a][e], s);
    }
}

// RELU: the input is a pre-activation tensor whose consumer applies max(x, 0)
// (VGG19 feature stack: ReLU folded into the next conv's operand load).
// UP: x is the low-resolution tensor [B][hi][wi] of a bilinear align_corners
// resize to H x W (the decoder's x2 upsample, Unetmodel.py:122-130); every
// patch value is sampled from it as nsm_resize_fwd computes it, so the
// resized activation is never written to HBM.
// H2: V is written as an h2 tensor (nsm_conv_h2.inc) Vh [alpha^2][T][2C] with
// the scale of hsc (max|x| recorded by x's producer, beta = the transform's bound)
// UNI (with UP, host-checked: C / CW a multiple of 64): a wave covers 64
// channels of ONE tile, so the tile, its source taps and rows are
// wave-uniform and kept in scalar registers
// OCC: minimum waves per SIMD the register allocation must allow (the F(6x6)
// x2-upsample form with wave-uniform tiles: 3, i.e. <= 168 VGPRs instead of
// 218 — no spills, tools/asm_audit.py)
template <int MT, bool RELU, bool UP, bool H2 = false, bool UNI = false, int OCC = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8)))
    wino_input_kernel(const float* __restrict__ x, int ld, int H, int W, int C, int TH, int TW,
                      long long T, float* __restrict__ V, int hi, int wi, float sh, float sw,
                      uint32_t* __restrict__ amax, bf16_t* __restrict__ Vh = nullptr,
                      H2Scale hsc = H2Scale{}) {
  constexpr int A = MT + 2, CW = WinoVec<MT>::W;
  using VT = typename WinoVec<MT>::T;
  const int C4 = C / CW;
  const long long total = T * C4;
  uint32_t am = 0;  // max|V| of this thread (the f16x2 GEMM's operand scale)
  float hs = 1.f;
  if constexpr (H2) hs = exp2i(h2_exp(hsc));
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    long long t = i / C4;
    if constexpr (UNI) t = __builtin_amdgcn_readfirstlane((int)t);
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    // patch rows stream through the column pass (wcol_row): one row live
    VT sc[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) sc[a][e] = VT{};
    if constexpr (UP) {
      int x0[A], x1[A];
      float lx0[A], lx1[A];
#pragma unroll
      for (int e = 0; e < A; ++e)
        lin_idx(sw, min(max(MT * tx - 1 + e, 0), W - 1), wi, x0[e], x1[e], lx0[e], lx1[e]);
      // Separable: a patch row is ly0 * h(y0) + ly1 * h(y1), h(y) the
      // x-interpolated source row y. The (m+2) patch rows of a x2 upsample
      // touch only ~m/2 + 2 source rows, so h(y) is computed once per source
      // row and kept while consecutive patch rows reuse it (4 loads per
      // element -> ~1.5). The reuse tests depend on the tile only, which is
      // uniform over a wave whenever C / CW >= 64 (the decoder layers).
      VT h0[A], h1[A];
      int ya = -1, yb = -1;  // source rows held in h0, h1
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const int yy = MT * ty - 1 + a;
        int y0, y1;
        float ly0, ly1;
        lin_idx(sh, min(max(yy, 0), H - 1), hi, y0, y1, ly0, ly1);
        if (y0 != ya) {
          if (y0 == yb) {
#pragma unroll
            for (int e = 0; e < A; ++e) h0[e] = h1[e];
          } else {
            const float* r0 = x + ((size_t)b * hi + y0) * wi * ld + c;
#pragma unroll
            for (int e = 0; e < A; ++e)
              h0[e] = lx0[e] * *(const VT*)(r0 + (size_t)x0[e] * ld) +
                      lx1[e] * *(const VT*)(r0 + (size_t)x1[e] * ld);
          }
          ya = y0;
        }
        if (y1 != yb) {
          if (y1 == ya) {
#pragma unroll
            for (int e = 0; e < A; ++e) h1[e] = h0[e];
          } else {
            const float* r1 = x + ((size_t)b * hi + y1) * wi * ld + c;
#pragma unroll
            for (int e = 0; e < A; ++e)
              h1[e] = lx0[e] * *(const VT*)(r1 + (size_t)x0[e] * ld) +
                      lx1[e] * *(const VT*)(r1 + (size_t)x1[e] * ld);
          }
          yb = y1;
        }
        VT d[A];
#pragma unroll
        for (int e = 0; e < A; ++e) {
          const int xx = MT * tx - 1 + e;
          const VT v = ly0 * h0[e] + ly1 * h1[e];
          d[e] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) ? v : VT{};
        }
        wcol_row<CBt<MT>>(sc, d, a);
      }
    } else {
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const int yy = MT * ty - 1 + a;
        VT d[A];
#pragma unroll
        for (int e = 0; e < A; ++e) {
          const int xx = MT * tx - 1 + e;
          d[e] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                     ? *(const VT*)(x + ((size_t)(b * H + yy) * W + xx) * ld + c)
                     : VT{};
          if (RELU) d[e] = vrelu(d[e]);
        }
        wcol_row<CBt<MT>>(sc, d, a);
      }
    }
    // row pass, one output row at a time
#pragma unroll
    for (int a = 0; a < A; ++a) {
      VT v[A];
      wmat<CBt<MT>>(sc[a], v);
      if constexpr (H2) {
        h2_write_row<A>(Vh, T, C, t, c, a, v, hs);
      } else {
        const size_t plane = (size_t)T * C;
        float* out = V + (size_t)t * C + c;
#pragma unroll
        for (int e = 0; e < A; ++e) {
          *(VT*)(out + (a * A + e) * plane) = v[e];
          if (amax) amax_fold(am, v[e]);
        }
      }
    }
  }
  if constexpr (!H2) amax_flush(am, amax);
}

// STATS: also the BatchNorm batch statistics of the written values (the
// Winograd layers' BN input, Unetmodel.py:21-22), so no separate bn_stats pass
// re-reads Y. The grid is sized so each thread keeps ONE channel group for the
// whole grid-stride loop (gridDim.x * 256 = nslot * N4); it Chan-merges each
// tile's {count, mean, M2} into its own and writes partial[slot][3][N] =
// {sum, M2 about the slot mean, count}, slot = (global thread id) / N4 (the
// counted partial layout nsm_bn_finalize_train takes with rows_per_chunk 0).
// ACT (eval, no STATS): y = lrelu((o + bias) * act_scale + act_shift) (+ res),
// the following BatchNorm (running statistics) + LeakyReLU (+ skip) applied
// on the way out (Unetmodel.py:22-23,27-28,125-137)
struct WinoAct {
  const float* scale;
  const float* shift;
  float slope;
  const float* res;
  int ldres;
};

// M16: M is the f16 output of the O16 GEMM (nsm_wino_gemm_f16m), scaled by
// 2^(e_v + e_u + e_tile) against the true M, e_tile the exponent the GEMM
// chose for each 64 x 64 tile of each component ([alpha^2][rows][N / 64])
struct WinoM16 {
  H2Scale sv, su;
  const int* e;
  int rows;  // ceil(T / 64)
};

// The column pass streams M's rows (wcol_row: wmat2's bits with one row
// live): F(6x6) 138 -> 128 VGPRs, 3 -> 4 waves per SIMD
// BFO (the bf16 path, nsm_wino_output_bf16): y holds bf16; the BN partials are
// of the bf16-rounded outputs, as the direct bf16 convolution's epilogue
// CWX: channels per thread (0: WinoVec<MT>::W; 2: the bf16 path's f16-M form
// at half the accumulator registers, BfLane's reason, or fp32 F(6x6): 8-B
// loads of M instead of 4-B ones, f6_out_cw)
template <int MT, bool STATS, bool ACT = false, bool BFO = false, bool M16 = false, int CWX = 0>
__global__ void __launch_bounds__(256) wino_output_kernel(const float* __restrict__ Mb, int N, int H,
                                                          int W, int TH, int TW, long long T,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y, int ldy,
                                                          float* __restrict__ partial,
                                                          WinoAct act = WinoAct{},
                                                          WinoM16 m16 = WinoM16{}) {
  constexpr int A = MT + 2, CW = CWX ? CWX : WinoVec<MT>::W;
  using VT = std::conditional_t<CW == 2, f32x2, typename WinoVec<MT>::T>;
  static_assert(CWX == 0 || (BFO && M16 && (CW == 2 || CW == 4)) || (MT == 6 && CWX == 2 && !BFO && !M16),
                "CWX: the f16-M bf16 form, or fp32 F(6x6) at 2 channels per thread");
  static_assert(!M16 || (BFO && (CW == 4 || CW == 2)), "f16 M: the bf16 path's F(4x4)");
  int ev = 0, eu = 0;  // every lane reads the scale slots (wave reduction) before the loop
  if constexpr (M16) {
    ev = h2_exp(m16.sv);
    eu = h2_exp(m16.su);
  }
  const int N4 = N / CW;
  const long long total = T * N4;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  VT s_sum{}, s_mean{}, s_m2{};
  float s_n = 0.f;
  for (long long i = i0; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % N4) * CW;
    const long long t = i / N4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    const size_t plane = (size_t)T * N;
    const float* in = Mb + (size_t)t * N + c;
    const bf16_t* in16 = (const bf16_t*)Mb + (size_t)t * N + c;
    VT sc[MT][A], o[MT][MT];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      VT row[A];
#pragma unroll
      for (int e = 0; e < A; ++e) {
        if constexpr (M16) {
          const int et = m16.e[((size_t)(a * A + e) * m16.rows + t / 64) * (N / 64) + c / 64];
          int x = -et - ev;
          x = x < -126 ? -126 : (x > 126 ? 126 : x);
          if constexpr (CW == 2) {
            const f32x2 lo = unpack_h2(*(const uint32_t*)(in16 + (a * A + e) * plane));
            row[e] = VT{lo.x, lo.y} * (exp2i(x) * exp2i(-eu));
          } else {
            const u32x2 h = *(const u32x2*)(in16 + (a * A + e) * plane);
            const f32x2 lo = unpack_h2(h.x), hi = unpack_h2(h.y);
            row[e] = VT{lo.x, lo.y, hi.x, hi.y} * (exp2i(x) * exp2i(-eu));
          }
        } else {
          row[e] = *(const VT*)(in + (a * A + e) * plane);
        }
      }
      wcol_row<CAt<MT>>(sc, row, a);
    }
#pragma unroll
    for (int a = 0; a < MT; ++a) wmat<CAt<MT>>(sc[a], o[a]);
    const VT bv = bias ? *(const VT*)(bias + c) : VT{};
    VT asc{}, ash{};
    if (ACT) {
      asc = *(const VT*)(act.scale + c);
      ash = *(const VT*)(act.shift + c);
    }
    VT ts{};
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int yy = MT * ty + a;
      if (yy >= H) continue;
      const size_t ro = ((size_t)(b * H + yy) * W + MT * tx) * ldy + c;
      float* row = y + ro;
#pragma unroll
      for (int e = 0; e < MT; ++e)
        if (MT * tx + e < W) {
          o[a][e] = o[a][e] + bv;
          if constexpr (BFO) {
            static_assert(CW == 4 || CW == 2, "bf16 output: F(4x4) / F(2x2)");
            // ACT (the bf16 eval path): lrelu(BN(y)) from the running statistics,
            // rounded once to bf16 (the skip add is on the block output, not here)
            VT q = o[a][e];
            if constexpr (ACT) q = vlrelu(q * asc + ash, act.slope);
            if constexpr (CW == 2) {
              o[a][e] = VT{round_bf(q.x), round_bf(q.y)};
              *(uint32_t*)((bf16_t*)y + ro + (size_t)e * ldy) = pack_bf2(o[a][e].x, o[a][e].y);
            } else {
              o[a][e] = VT{round_bf(q.x), round_bf(q.y), round_bf(q.z), round_bf(q.w)};
              st4((bf16_t*)y + ro + (size_t)e * ldy, o[a][e]);
            }
            if (STATS) ts = ts + o[a][e];
            continue;
          }
          VT v = o[a][e];
          if (ACT) {
            v = vlrelu(v * asc + ash, act.slope);
            if (act.res)
              v = v + *(const VT*)(act.res + ((size_t)(b * H + yy) * W + MT * tx + e) * act.ldres + c);
          }
          *(VT*)(row + (size_t)e * ldy) = v;
          if (STATS) ts = ts + o[a][e];
        }
    }
    if (STATS) {
      const int nv = min(MT, H - MT * ty) * min(MT, W - MT * tx);
      const VT tmean = ts * (1.f / (float)nv);
      VT tq{};
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int e = 0; e < MT; ++e)
          if (MT * ty + a < H && MT * tx + e < W) {
            const VT d = o[a][e] - tmean;
            tq = tq + d * d;
          }
      const float n2 = s_n + (float)nv;
      const VT delta = tmean - s_mean;
      s_mean = s_mean + delta * ((float)nv / n2);
      s_m2 = s_m2 + tq + delta * delta * (s_n * (float)nv / n2);
      s_sum = s_sum + ts;
      s_n = n2;
    }
  }
  if (STATS && i0 < (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i0 % N4) * CW;
    float* pr = partial + (size_t)(i0 / N4) * 3 * N + c;
    *(VT*)pr = s_sum;
    *(VT*)(pr + N) = s_m2;
    *(VT*)(pr + 2 * N) = VT{} + s_n;
  }
}

// dM[xi][t][n] = (A dY_t A^T): transpose of the output transform, m x m -> alpha x alpha
template <int MT>
__global__ void __launch_bounds__(256) wino_dout_kernel(const float* __restrict__ dy, int ld, int H,
                                                        int W, int N, int TH, int TW, long long T,
                                                        float* __restrict__ dM) {
  constexpr int A = MT + 2, CW = WinoVec<MT>::W;
  using VT = typename WinoVec<MT>::T;
  const int N4 = N / CW;
  const long long total = T * N4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % N4) * CW;
    const long long t = i / N4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    VT g[MT][MT], s[A][A];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int e = 0; e < MT; ++e) {
        const int yy = MT * ty + a, xx = MT * tx + e;
        g[a][e] = (yy < H && xx < W) ? *(const VT*)(dy + ((size_t)(b * H + yy) * W + xx) * ld + c)
                                     : VT{};
      }
    wmat2<CA<MT>>(g, s);
    const size_t plane = (size_t)T * N;
    float* out = dM + (size_t)t * N + c;
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) *(VT*)(out + (a * A + e) * plane) = s[a][e];
  }
}

// Both Winograd transforms of one gradient dY (the input gradient of a 3x3
// conv whose dgrad AND weight gradient run in the Winograd domain) from ONE
// read of it: the (m+2)^2 patch of tile t gives V = B^T d B (the dgrad's input
// transform, as wino_input) and its m x m interior gives dM = A^T-side
// transform (as wino_dout). Saves a full read of dY per layer.
// BN: dy is not materialised — each patch element is the first BatchNorm's
// backward (Unetmodel.py:21-24) computed from its inputs, exactly as
// nsm_bn_bwd_apply would have stored it: dz = g * lrelu'(y*scale+shift) *
// mask[b][c], dy = k1*dz + k2*(y - mean) + k3 (coef of nsm_bn_bwd_finalize);
// zero outside the image (the dgrad's padding). Saves writing dY1 and
// reading it back (it has no other consumer on the Winograd path).
struct WinoBnSrc {
  const float* y;
  int ldy;
  const float* scale;
  const float* shift;
  const float* mean;
  const float* coef;
  const float* mask;  // [B][C] or null
  float slope;
};
__device__ __forceinline__ float vlrelu_grad(float z, float s) { return lrelu_grad(z, s); }
__device__ __forceinline__ f32x4 vlrelu_grad(f32x4 z, float s) { return lrelu_grad_v4(z, s); }

// H2: V and dM written as h2 tensors (Vh, dMh; scales of hv, hd: max|dy|
// recorded by dy's producer, beta = each transform's bound)
template <int MT, bool BN = false, bool H2 = false>
__global__ void __launch_bounds__(256) wino_dual_kernel(const float* __restrict__ dy, int ld, int H,
                                                        int W, int C, int TH, int TW, long long T,
                                                        float* __restrict__ V,
                                                        float* __restrict__ dM,
                                                        WinoBnSrc bn = WinoBnSrc{},
                                                        uint32_t* __restrict__ amax_v = nullptr,
                                                        uint32_t* __restrict__ amax_dm = nullptr,
                                                        bf16_t* __restrict__ Vh = nullptr,
                                                        bf16_t* __restrict__ dMh = nullptr,
                                                        H2Scale hv = H2Scale{},
                                                        H2Scale hd = H2Scale{}) {
  constexpr int A = MT + 2, CW = WinoVec<MT>::W;
  using VT = typename WinoVec<MT>::T;
  const int C4 = C / CW;
  const long long total = T * C4;
  uint32_t amv = 0, amd = 0;  // max|V|, max|dM| (the f16x2 GEMMs' operand scales)
  float hsv = 1.f, hsd = 1.f;
  if constexpr (H2) {
    hsv = exp2i(h2_exp(hv));
    hsd = exp2i(h2_exp(hd));
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    const long long t = i / C4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    VT d[A][A];
    VT sc{}, sh{}, mu{}, k1{}, k2{}, k3{}, mk{};
    if constexpr (BN) {
      sc = *(const VT*)(bn.scale + c);
      sh = *(const VT*)(bn.shift + c);
      mu = *(const VT*)(bn.mean + c);
      k1 = *(const VT*)(bn.coef + c);
      k2 = *(const VT*)(bn.coef + C + c);
      k3 = *(const VT*)(bn.coef + 2 * C + c);
      if (bn.mask) mk = *(const VT*)(bn.mask + (size_t)b * C + c);
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const int yy = MT * ty - 1 + a;
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const size_t p = (size_t)(b * H + yy) * W + xx;
        if constexpr (BN) {
          VT v{};
          if (in) {
            const VT gv = *(const VT*)(dy + p * ld + c);
            const VT yv = *(const VT*)(bn.y + p * bn.ldy + c);
            VT dz = gv * vlrelu_grad(yv * sc + sh, bn.slope);
            if (bn.mask) dz = dz * mk;
            v = k1 * dz + k2 * (yv - mu) + k3;
          }
          d[a][e] = v;
        } else {
          d[a][e] = in ? *(const VT*)(dy + p * ld + c) : VT{};
        }
      }
    }
    const size_t plane = (size_t)T * C;
    {
      VT v[A][A];
      wmat2<CBt<MT>>(d, v);
      if constexpr (H2) {
        h2_write<A>(Vh, T, C, t, c, v, hsv);
      } else {
        float* out = V + (size_t)t * C + c;
#pragma unroll
        for (int a = 0; a < A; ++a)
#pragma unroll
          for (int e = 0; e < A; ++e) {
            *(VT*)(out + (a * A + e) * plane) = v[a][e];
            if (amax_v) amax_fold(amv, v[a][e]);
          }
      }
    }
    VT g[MT][MT], sm[A][A];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int e = 0; e < MT; ++e) g[a][e] = d[a + 1][e + 1];
    wmat2<CA<MT>>(g, sm);
    if constexpr (H2) {
      h2_write<A>(dMh, T, C, t, c, sm, hsd);
    } else {
      float* out = dM + (size_t)t * C + c;
#pragma unroll
      for (int a = 0; a < A; ++a)
#pragma unroll
        for (int e = 0; e < A; ++e) {
          *(VT*)(out + (a * A + e) * plane) = sm[a][e];
          if (amax_dm) amax_fold(amd, sm[a][e]);
        }
    }
  }
  if constexpr (!H2) {
    amax_flush(amv, amax_v);
    amax_flush(amd, amax_dm);
  }
}

// wino_dual_kernel<MT, BN=true, H2=true> through LDS: the per-thread form
// loads every patch element of g and y itself — 2 x 64 4-B loads per thread
// over patches that overlap 1.78x, each element's BN backward recomputed per
// patch holding it — and is load-issue-bound (~230 us on conv7's dY1 beside
// ~150 us for the separate apply). Here a block covers TYB x TXB tiles x 32
// channels: its (m TYB + 2) x (m TXB + 2) pixel region of g and y is read once
// with 16-B loads (8 lanes per pixel, coalesced), dY1 = k1 dz + k2 (y - mean)
// + k3 formed once per element into LDS (zero outside the image: the dgrad's
// padding), then each thread (tile, channel) reads its (m+2)^2 patch from LDS
// and writes both transforms as h2, as wino_dual_kernel does.
template <int MT, int TYB, int TXB>
__global__ void __launch_bounds__(256) wino_dual_bn_lds_kernel(
    const float* __restrict__ g, int ldg, int H, int W, int C, int TH, int TW, long long T,
    WinoBnSrc bn, bf16_t* __restrict__ Vh, bf16_t* __restrict__ dMh, H2Scale hv, H2Scale hd) {
  constexpr int A = MT + 2, CB = 32, RH = MT * TYB + 2, RW = MT * TXB + 2;
  static_assert(TYB * TXB * CB == 256, "one (tile, channel) per thread");
  __shared__ __attribute__((aligned(16))) float reg[RH * RW * CB];
  const int tid = threadIdx.x;
  const int txb = blockIdx.x % ((TW + TXB - 1) / TXB), tyb = blockIdx.x / ((TW + TXB - 1) / TXB);
  const int b = blockIdx.y / (C / CB), c0 = (blockIdx.y % (C / CB)) * CB;
  const int ty0 = tyb * TYB, tx0 = txb * TXB;
  // the scales before any lane leaves: amax_read reduces over all 64 lanes
  const float hsv = exp2i(h2_exp(hv)), hsd = exp2i(h2_exp(hd));
  {
    // the region's rows: this lane's 4 channels are fixed (256 % 8 == 0)
    const int cg = (tid & 7) * 4, c = c0 + cg;
    const f32x4 sc = *(const f32x4*)(bn.scale + c), sh = *(const f32x4*)(bn.shift + c);
    const f32x4 mu = *(const f32x4*)(bn.mean + c);
    const f32x4 k1 = *(const f32x4*)(bn.coef + c), k2 = *(const f32x4*)(bn.coef + C + c);
    const f32x4 k3 = *(const f32x4*)(bn.coef + 2 * C + c);
    f32x4 mk = {1.f, 1.f, 1.f, 1.f};
    if (bn.mask) mk = *(const f32x4*)(bn.mask + (size_t)b * C + c);
    // every load of the region goes out before the first is used: the loads
    // are unconditional (a pixel outside the region or image reads the
    // batch's first pixel, its value then discarded), so hipcc issues all of
    // them back to back instead of one loop trip at a time
    constexpr int NIT = (RH * RW + 31) / 32;
    f32x4 gv[NIT], yv[NIT];
    bool ok[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int p = (tid >> 3) + 32 * k;
      const int py = p / RW, px = p - py * RW;
      const int yy = MT * ty0 - 1 + py, xx = MT * tx0 - 1 + px;
      ok[k] = p < RH * RW && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const size_t q = (size_t)b * H * W + (ok[k] ? (size_t)yy * W + xx : 0);
      gv[k] = *(const f32x4*)(g + q * ldg + c);
      yv[k] = *(const f32x4*)(bn.y + q * bn.ldy + c);
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int p = (tid >> 3) + 32 * k;
      if (p >= RH * RW) break;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (ok[k]) {
        f32x4 dz = gv[k] * vlrelu_grad(yv[k] * sc + sh, bn.slope);
        if (bn.mask) dz = dz * mk;
        v = k1 * dz + k2 * (yv[k] - mu) + k3;
      }
      *(f32x4*)&reg[p * CB + cg] = v;
    }
  }
  __syncthreads();
  const int cl = tid & (CB - 1), tl = tid / CB;
  const int ty = ty0 + tl / TXB, tx = tx0 + tl % TXB;
  if (ty >= TH || tx >= TW) return;  // (no barrier follows)
  const long long t = ((long long)b * TH + ty) * TW + tx;
  const int c = c0 + cl;
  const float* pr = reg + ((tl / TXB) * MT * RW + (tl % TXB) * MT) * CB + cl;
  float d[A][A];
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int e = 0; e < A; ++e) d[a][e] = pr[(a * RW + e) * CB];
  {
    float v[A][A];
    wmat2<CBt<MT>>(d, v);
    h2_write<A>(Vh, T, C, t, c, v, hsv);
  }
  float gi[MT][MT], sm[A][A];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int e = 0; e < MT; ++e) gi[a][e] = d[a + 1][e + 1];
  wmat2<CA<MT>>(gi, sm);
  h2_write<A>(dMh, T, C, t, c, sm, hsd);
}

// wino_input_kernel<MT, RELU=false, UP, H2=true> through LDS, in the layout of
// wino_dual_bn_lds_kernel: a block's (m TYB + 2) x (m TXB + 2) pixel region x
// 32 channels is formed once — read with 16-B loads, or (UP) sampled from the
// low-resolution source with the bilinear align_corners weights of
// nsm_resize_fwd, once per pixel instead of once per patch holding it — then
// each thread (tile, channel) transforms its patch from LDS and writes V as
// h2 (scale: max|x| of the source times beta, as nsm_wino_input_h2).
template <int MT, int TYB, int TXB, bool UP>
__global__ void __launch_bounds__(256) wino_input_lds_kernel(
    const float* __restrict__ x, int ld, int H, int W, int C, int TH, int TW, long long T, int hi,
    int wi, float sh, float sw, bf16_t* __restrict__ Vh, H2Scale hsc) {
  constexpr int A = MT + 2, CB = 32, RH = MT * TYB + 2, RW = MT * TXB + 2;
  static_assert(TYB * TXB * CB == 256, "one (tile, channel) per thread");
  __shared__ __attribute__((aligned(16))) float reg[RH * RW * CB];
  const int tid = threadIdx.x;
  const int txb = blockIdx.x % ((TW + TXB - 1) / TXB), tyb = blockIdx.x / ((TW + TXB - 1) / TXB);
  const int b = blockIdx.y / (C / CB), c0 = (blockIdx.y % (C / CB)) * CB;
  const int ty0 = tyb * TYB, tx0 = txb * TXB;
  const float hs = exp2i(h2_exp(hsc));  // before any lane leaves (amax_read: all 64 lanes)
  {
    const int c = c0 + (tid & 7) * 4;
#pragma unroll
    for (int k = 0; k < (RH * RW + 31) / 32; ++k) {
      const int p = (tid >> 3) + 32 * k;
      if (p >= RH * RW) break;
      const int py = p / RW, px = p - py * RW;
      const int yy = MT * ty0 - 1 + py, xx = MT * tx0 - 1 + px;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
        if constexpr (UP) {
          int y0, y1, x0, x1;
          float ly0, ly1, lx0, lx1;
          lin_idx(sh, yy, hi, y0, y1, ly0, ly1);
          lin_idx(sw, xx, wi, x0, x1, lx0, lx1);
          const float* r0 = x + ((size_t)b * hi + y0) * wi * ld + c;
          const float* r1 = x + ((size_t)b * hi + y1) * wi * ld + c;
          const f32x4 h0 = lx0 * *(const f32x4*)(r0 + (size_t)x0 * ld) +
                           lx1 * *(const f32x4*)(r0 + (size_t)x1 * ld);
          const f32x4 h1 = lx0 * *(const f32x4*)(r1 + (size_t)x0 * ld) +
                           lx1 * *(const f32x4*)(r1 + (size_t)x1 * ld);
          v = ly0 * h0 + ly1 * h1;
        } else {
          v = *(const f32x4*)(x + ((size_t)(b * H + yy) * W + xx) * ld + c);
        }
      }
      *(f32x4*)&reg[p * CB + (tid & 7) * 4] = v;
    }
  }
  __syncthreads();
  const int cl = tid & (CB - 1), tl = tid / CB;
  const int ty = ty0 + tl / TXB, tx = tx0 + tl % TXB;
  if (ty >= TH || tx >= TW) return;  // (no barrier follows; lane pairs share a tile)
  const long long t = ((long long)b * TH + ty) * TW + tx;
  const float* pr = reg + ((tl / TXB) * MT * RW + (tl % TXB) * MT) * CB + cl;
  float d[A][A], v[A][A];
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int e = 0; e < A; ++e) d[a][e] = pr[(a * RW + e) * CB];
  wmat2<CBt<MT>>(d, v);
  h2_write<A>(Vh, T, C, t, c0 + cl, v, hs);
}

// dst[b][i] = sum_s src[b][s][i] (float4 lanes, fixed order): the split-K
// partials of a batched GEMM, one batch entry per grid.y
__global__ void __launch_bounds__(256) batched_splitsum_kernel(const float* __restrict__ src,
                                                               int splits, long long L4,
                                                               float* __restrict__ dst) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= L4) return;
  const f32x4* p = (const f32x4*)src + (size_t)blockIdx.y * splits * L4 + i;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 1 < splits; k += 2) {
    a += p[(size_t)k * L4];
    b += p[(size_t)(k + 1) * L4];
  }
  if (k < splits) a += p[(size_t)k * L4];
  ((f32x4*)dst)[(size_t)blockIdx.y * L4 + i] = a + b;
}

// dw[co][ci][3][3] = G^T (sum_s dU[xi][s][co][ci]) G, one thread per (co, ci)
template <int MT>
__global__ void __launch_bounds__(256) wino_wgrad_out_kernel(const float* __restrict__ slab,
                                                             int splits, int M, int N, int cin,
                                                             int cout, float* __restrict__ dw) {
  constexpr int A = MT + 2;
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= cout * cin) return;
  const int ci = idx % cin, co = idx / cin;
  const size_t MN = (size_t)M * N;
  const float* src = slab + (size_t)co * N + ci;
  float u[A][A], o[3][3];
  // split loop outside, the (m+2)^2 components unrolled inside: all of a
  // split's loads are in flight together (the component-outer form waited on
  // each component's loads in turn: 2.2 TB/s)
#pragma unroll
  for (int x = 0; x < A * A; ++x) u[x / A][x % A] = src[(size_t)x * splits * MN];
  for (int k = 1; k < splits; ++k) {
#pragma unroll
    for (int x = 0; x < A * A; ++x) u[x / A][x % A] += src[((size_t)x * splits + k) * MN];
  }
  wmat2<CGt<MT>>(u, o);
  float* out = dw + ((size_t)co * cin + ci) * 9;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int e = 0; e < 3; ++e) out[r * 3 + e] = o[r][e];
}

// ---- all weight layouts of one step in ONE launch ----------------------------
// Jobs (include/nsm.h NsmPrepJob): 0 = pack fp32, 1 = pack bf16 (a[] = cout,
// cin, taps, cout_p, cin_p, mode), 2 = Winograd U (a[] = cout, cin, n_p, k_p,
// flip, tile), 3 = pad vector (a[] = n, n_p). Items are output elements
// (pack, pad) or (n, k) filter pairs (Winograd); `base` is the job's first
// item in the launch-wide numbering (ascending), found by binary search.
__host__ __device__ inline long long nsm_prep_items_dev(const NsmPrepJob& j) {
  switch (j.kind) {
    case 0:
    case 1:
    case 5:
    case 7: return (long long)j.a[3] * j.a[4] * j.a[2];
    case 2:
    case 4:
    case 6: return (long long)j.a[2] * j.a[3];
    case 3: return j.a[1];
    default: return -1;
  }
}

template <int MT>
__device__ __forceinline__ void wino_weight_item(const float* __restrict__ w, int cout, int cin,
                                                 int n_p, int k_p, int flip, float* __restrict__ U,
                                                 int idx, uint32_t& am) {
  constexpr int A = MT + 2;
  const int k = idx % k_p, n = idx / k_p;
  const int co = flip ? k : n, ci = flip ? n : k;
  float g[3][3];
  const bool ok = co < cout && ci < cin;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int sa = flip ? 2 - a : a, sb = flip ? 2 - b : b;
      g[a][b] = ok ? w[((size_t)co * cin + ci) * 9 + sa * 3 + sb] : 0.f;
    }
  float u[A][A];
  wmat2<CG<MT>>(g, u);
  const size_t plane = (size_t)n_p * k_p;
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int b = 0; b < A; ++b) {
      U[(a * A + b) * plane + (size_t)n * k_p + k] = u[a][b];
      amax_fold(am, u[a][b]);
    }
}

// Winograd U as an h2 tensor [alpha^2][n_p][2 k_p] (nsm_conv_h2.inc), scale s
template <int MT>
__device__ __forceinline__ void wino_weight_item_h2(const float* __restrict__ w, int cout, int cin,
                                                    int n_p, int k_p, int flip,
                                                    bf16_t* __restrict__ U, int idx, float s) {
  constexpr int A = MT + 2;
  const int k = idx % k_p, n = idx / k_p;
  const int co = flip ? k : n, ci = flip ? n : k;
  float g[3][3];
  const bool ok = co < cout && ci < cin;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int sa = flip ? 2 - a : a, sb = flip ? 2 - b : b;
      g[a][b] = ok ? w[((size_t)co * cin + ci) * 9 + sa * 3 + sb] : 0.f;
    }
  float u[A][A];
  wmat2<CG<MT>>(g, u);
  h2_write<A>(U, n_p, k_p, n, k, u, s);
}

#ifndef NSM_PREP_ITEMS
#define NSM_PREP_ITEMS 512
#endif
// Winograd U as a single-plane scaled f16 tensor [alpha^2][n_p][k_p] (the
// bf16 path's F(4x4) forward, nsm_wino_gemm_f16), scale s
template <int MT>
__device__ __forceinline__ void wino_weight_item_f16(const float* __restrict__ w, int cout, int cin,
                                                     int n_p, int k_p, int flip,
                                                     bf16_t* __restrict__ U, int idx, float s) {
  constexpr int A = MT + 2;
  const int k = idx % k_p, n = idx / k_p;
  const int co = flip ? k : n, ci = flip ? n : k;
  float g[3][3];
  const bool ok = co < cout && ci < cin;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int sa = flip ? 2 - a : a, sb = flip ? 2 - b : b;
      g[a][b] = ok ? w[((size_t)co * cin + ci) * 9 + sa * 3 + sb] : 0.f;
    }
  float u[A][A];
  wmat2<CG<MT>>(g, u);
  const size_t plane = (size_t)n_p * k_p;
#pragma unroll
  for (int a = 0; a < A; ++a)
#pragma unroll
    for (int b = 0; b < A; ++b)
      U[(a * A + b) * plane + (size_t)n * k_p + k] =
          __builtin_bit_cast(unsigned short, (_Float16)(u[a][b] * s));
}

constexpr int PREP_ITEMS = NSM_PREP_ITEMS;  // items per block, 2 per thread (8: -0.2 % step, more tail)

// U of one (n, k) item, unscaled (flip: the input gradient's filters)
template <int MT>
__device__ __forceinline__ void wino_weight_u(const float* __restrict__ w, int cout, int cin, int k_p,
                                              int flip, int idx, float (&u)[MT + 2][MT + 2]) {
  const int k = idx % k_p, n = idx / k_p;
  const int co = flip ? k : n, ci = flip ? n : k;
  float g[3][3];
  const bool ok = co < cout && ci < cin;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int sa = flip ? 2 - a : a, sb = flip ? 2 - b : b;
      g[a][b] = ok ? w[((size_t)co * cin + ci) * 9 + sa * 3 + sb] : 0.f;
    }
  wmat2<CG<MT>>(g, u);
}

// A block's U items (kinds 4 and 6, phase 1) with 16-B stores: each thread
// transforms its item, 16 planes at a time go through LDS ([plane][item]),
// then each store task takes 8 consecutive items (k) of one plane and writes
// their h and l chunks (h2, kind 4: the 8h / 8l of one channel chunk) or their
// 8 f16 (kind 6). One item per thread wrote 2-B (kind 6) or lane-paired 4-B
// (h2_write) words: 64 (36) store instructions per item. items % 8 == 0
// (k_p % 32), so a group of 8 is wholly inside or outside the job.
template <int MT, bool SPL>
__device__ void wino_weight_block(const NsmPrepJob& j, long long lbase, long long items, float s,
                                  float* __restrict__ stg) {
  constexpr int A = MT + 2, NPL = A * A, CH = 16;
  const int cout = j.a[0], cin = j.a[1], n_p = j.a[2], k_p = j.a[3], flip = j.a[4];
  bf16_t* U = (bf16_t*)j.dst;
  const int cols = SPL ? k_p : 2 * k_p;  // f16 row length of U
  const size_t plane = (size_t)n_p * cols;
  for (int r = 0; r < PREP_ITEMS / 256; ++r) {
    const long long lr = lbase + r * 256;
    if (lr >= items) break;  // uniform
    const long long li = lr + threadIdx.x;
    float u[A][A];
    wino_weight_u<MT>(j.src, cout, cin, k_p, flip, li < items ? (int)li : 0, u);
#pragma unroll
    for (int c0 = 0; c0 < NPL; c0 += CH) {
      __syncthreads();  // the previous chunk's LDS reads are done
#pragma unroll
      for (int q = 0; q < CH; ++q)
        if (c0 + q < NPL) stg[q * 256 + threadIdx.x] = u[(c0 + q) / A][(c0 + q) % A] * s;
      __syncthreads();
      for (int t = threadIdx.x; t < CH * 32; t += 256) {
        const int pl = t >> 5, grp = t & 31;
        const long long l0 = lr + 8 * grp;
        if (c0 + pl >= NPL || l0 >= items) continue;
        const int n = (int)(l0 / k_p), k0 = (int)(l0 - (long long)n * k_p);
        const f32x4 a = *(const f32x4*)&stg[pl * 256 + 8 * grp];
        const f32x4 b = *(const f32x4*)&stg[pl * 256 + 8 * grp + 4];
        bf16_t* o = U + (size_t)(c0 + pl) * plane + (size_t)n * cols + (SPL ? k0 : 2 * k0);
        if constexpr (SPL) {
          *(u32x4*)o = u32x4{pack_h2(f32x2{a.x, a.y}), pack_h2(f32x2{a.z, a.w}),
                             pack_h2(f32x2{b.x, b.y}), pack_h2(f32x2{b.z, b.w})};
        } else {
          u32x2 ha, la, hb, lb;
          split4h(a, 1.f, ha, la);
          split4h(b, 1.f, hb, lb);
          *(u32x4*)o = u32x4{ha.x, ha.y, hb.x, hb.y};
          *(u32x4*)(o + 8) = u32x4{la.x, la.y, lb.x, lb.y};
        }
      }
    }
  }
}

// blockIdx -> job by a (uniform) binary search over the jobs' first blocks
// (job.base / PREP_ITEMS: every job starts on a block boundary, see
// nsm_prep_items), then the block's items of that job, coalesced.
// phase 0: zeroes the step's operand-maximum slot buffers (z0, z1: the weight
// slots this launch fills, the forward's activation slots), and every block of
// an h2 / f16 job (kinds 4, 5, 6) stores max|w| of its filters as ONE word,
// pmax[blockIdx.x] (no atomics, so the slots need no zeroing before it);
// phase 1: such a job reduces the pmax words of its source job's blocks (its
// own, or those of the job whose filters it shares: a[6] = that job's first
// block + 1), the job's first block stores the maximum into line 0 of its slot
// (lines 1..63 stay 0: zeroed in phase 0) for the GEMMs, and all its blocks
// write with the scale derived from it; kinds 0 and 2 record max|written| by
// atomics (the slots zeroed in phase 0). Every other job waits for phase 1.
// (phase bit 1: the U jobs by wino_weight_block, NSM_PREP_WIDE)
__device__ __forceinline__ uint32_t block_max_u32(uint32_t m, uint32_t* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = max(max(red[0], red[1]), max(red[2], red[3]));
  __syncthreads();
  return m;
}

// the h2 exponent of a maximum held as a value (h2_exp's arithmetic)
__device__ __forceinline__ int h2_exp_of(uint32_t m, float beta) {
  uint32_t b = __float_as_uint(__uint_as_float(m) * beta);
  if (m < 0x7f800000u && b >= 0x7f800000u) b = 0x7f7fffffu;
  return pow2_scale_exp(b);
}

__global__ void __launch_bounds__(256) prep_weights_kernel(const NsmPrepJob* __restrict__ jobs,
                                                           int njobs, int phase,
                                                           uint32_t* __restrict__ pmax,
                                                           uint32_t* __restrict__ z0, long long nz0,
                                                           uint32_t* __restrict__ z1, long long nz1) {
  __shared__ uint32_t red[4];
  const bool wide = (phase & 2) != 0;
  phase &= 1;
  if (phase == 0) {  // the slot buffers of this step (uniform branch)
    const long long gs = (long long)gridDim.x * 256, i0 = (long long)blockIdx.x * 256 + threadIdx.x;
    for (long long i = i0; i < nz0; i += gs) z0[i] = 0u;
    for (long long i = i0; i < nz1; i += gs) z1[i] = 0u;
  }
  const long long blk0 = (long long)blockIdx.x * PREP_ITEMS;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].base <= blk0) lo = mid; else hi = mid - 1;
  }
  const NsmPrepJob& j = jobs[lo];
  const long long items = nsm_prep_items_dev(j);
  uint32_t am = 0;  // max|written| (the f16x2 GEMMs' operand scale, j.amax)
  const bool h2job = j.kind == 4 || j.kind == 5 || j.kind == 6;
  uint32_t wmax = 0;  // phase 1 of an h2 job: max|w| of its (source job's) filters
  if (h2job && phase == 1) {
    const long long first = j.a[6] ? (long long)j.a[6] - 1 : j.base / PREP_ITEMS;
    const long long nblk = (items + PREP_ITEMS - 1) / PREP_ITEMS;
    uint32_t m = 0;
    for (long long b = threadIdx.x; b < nblk; b += 256) m = max(m, pmax[first + b]);
    wmax = block_max_u32(m, red);
    if (blk0 == j.base && threadIdx.x == 0) j.amax[0] = wmax;  // line 0 of the slot
  }
  if (j.kind == 5) {  // h2 pack (uniform per block): max|w| (phase 0), then h + l (phase 1)
    const int cout = j.a[0], cin = j.a[1], taps = j.a[2], cout_p = j.a[3], cin_p = j.a[4];
    const bool fwd = j.a[5] == NSM_PACK_FWD;
    if (phase == 0 && j.a[6]) return;  // the FWD job over the same weight holds its maximum
    const float s = phase ? exp2i(h2_exp_of(wmax, 1.f)) : 0.f;
    const int K = taps * (fwd ? cin_p : cout_p);  // row length (fp32 elements)
    bf16_t* out = (bf16_t*)j.dst;
    for (int r = 0; r < PREP_ITEMS / 256; ++r) {
      const long long li = blk0 - j.base + r * 256 + threadIdx.x;
      if (li >= items) break;
      const int idx = (int)li;
      float v;
      if (fwd) {
        const int ci = idx % cin_p, t = idx / cin_p, tap = t % taps, co = t / taps;
        v = (co < cout && ci < cin) ? j.src[((size_t)co * cin + ci) * taps + tap] : 0.f;
      } else {
        const int co = idx % cout_p, t = idx / cout_p, tap = t % taps, ci = t / taps;
        v = (co < cout && ci < cin) ? j.src[((size_t)co * cin + ci) * taps + (taps - 1 - tap)] : 0.f;
      }
      if (phase == 0) {
        amax_fold(am, v);
      } else {
        const int row = idx / K, k = idx - row * K;
        const float a = v * s;
        const _Float16 h = (_Float16)a;
        bf16_t* o = out + (size_t)row * 2 * K + 16 * (k >> 3) + (k & 7);
        o[0] = __builtin_bit_cast(unsigned short, h);
        o[8] = __builtin_bit_cast(unsigned short, (_Float16)(a - (float)h));
      }
    }
    if (phase == 0) {
      am = block_max_u32(am, red);
      if (threadIdx.x == 0) pmax[blockIdx.x] = am;
    }
    return;
  }
  if (j.kind == 4 || j.kind == 6) {  // uniform per block (6: single-plane f16 U)
    const int cout = j.a[0], cin = j.a[1], n_p = j.a[2], k_p = j.a[3], flip = j.a[4];
    if (phase == 0) {
      if (j.a[6]) return;  // the un-flipped job over the same filters holds its maximum
      for (int r = 0; r < PREP_ITEMS / 256; ++r) {
        const long long li = blk0 - j.base + r * 256 + threadIdx.x;
        if (li >= items) break;
        const int k = (int)(li % k_p), n = (int)(li / k_p);
        const int co = flip ? k : n, ci = flip ? n : k;
        if (co < cout && ci < cin) {
          const float* g = j.src + ((size_t)co * cin + ci) * 9;
#pragma unroll
          for (int q = 0; q < 9; ++q) amax_fold(am, g[q]);
        }
      }
      am = block_max_u32(am, red);
      if (threadIdx.x == 0) pmax[blockIdx.x] = am;
      return;
    }
    const float s = exp2i(h2_exp_of(wmax, wino_beta(j.a[5], 2)));
    bf16_t* U = (bf16_t*)j.dst;
    if (wide) {
      __shared__ __attribute__((aligned(16))) float stg[16 * 256];
      const long long lb = blk0 - j.base;
      if (j.kind == 6) {
        if (j.a[5] == 4) wino_weight_block<4, true>(j, lb, items, s, stg);
        else wino_weight_block<2, true>(j, lb, items, s, stg);
      } else if (j.a[5] == 6) {
        wino_weight_block<6, false>(j, lb, items, s, stg);
      } else if (j.a[5] == 4) {
        wino_weight_block<4, false>(j, lb, items, s, stg);
      } else {
        wino_weight_block<2, false>(j, lb, items, s, stg);
      }
      return;
    }
    for (int r = 0; r < PREP_ITEMS / 256; ++r) {
      const long long li = blk0 - j.base + r * 256 + threadIdx.x;
      if (li >= items) break;
      if (j.kind == 6) {
        if (j.a[5] == 4) wino_weight_item_f16<4>(j.src, cout, cin, n_p, k_p, flip, U, (int)li, s);
        else wino_weight_item_f16<2>(j.src, cout, cin, n_p, k_p, flip, U, (int)li, s);
        continue;
      }
      if (j.a[5] == 6) wino_weight_item_h2<6>(j.src, cout, cin, n_p, k_p, flip, U, (int)li, s);
      else if (j.a[5] == 4) wino_weight_item_h2<4>(j.src, cout, cin, n_p, k_p, flip, U, (int)li, s);
      else wino_weight_item_h2<2>(j.src, cout, cin, n_p, k_p, flip, U, (int)li, s);
    }
    return;
  }
  if (phase == 0) return;
  for (int r = 0; r < PREP_ITEMS / 256; ++r) {
    const long long li = blk0 - j.base + r * 256 + threadIdx.x;
    if (li >= items) break;
    const int idx = (int)li;
    if (j.kind <= 1 || j.kind == 7) {
      const int cout = j.a[0], cin = j.a[1], taps = j.a[2], cout_p = j.a[3], cin_p = j.a[4];
      float v;
      if (j.a[5] == NSM_PACK_FWD) {
        const int ci = idx % cin_p, t = idx / cin_p, tap = t % taps, co = t / taps;
        v = (co < cout && ci < cin) ? j.src[((size_t)co * cin + ci) * taps + tap] : 0.f;
      } else {
        const int co = idx % cout_p, t = idx / cout_p, tap = t % taps, ci = t / taps;
        v = (co < cout && ci < cin) ? j.src[((size_t)co * cin + ci) * taps + (taps - 1 - tap)]
                                    : 0.f;
      }
      if (j.kind == 0) {
        ((float*)j.dst)[idx] = v;
        amax_fold(am, v);
      } else if (j.kind == 1) {
        ((bf16_t*)j.dst)[idx] = (bf16_t)(pack_bf2(v, 0.f) & 0xFFFFu);
      } else {  // 7: IEEE half
        ((bf16_t*)j.dst)[idx] = (bf16_t)(pack_hh(v, 0.f) & 0xFFFFu);
      }
    } else if (j.kind == 2) {
      float* U = (float*)j.dst;
      if (j.a[5] == 6) wino_weight_item<6>(j.src, j.a[0], j.a[1], j.a[2], j.a[3], j.a[4], U, idx, am);
      else if (j.a[5] == 4) wino_weight_item<4>(j.src, j.a[0], j.a[1], j.a[2], j.a[3], j.a[4], U, idx, am);
      else wino_weight_item<2>(j.src, j.a[0], j.a[1], j.a[2], j.a[3], j.a[4], U, idx, am);
    } else {
      ((float*)j.dst)[idx] = idx < j.a[0] ? j.src[idx] : 0.f;
    }
  }
  amax_flush(am, j.amax);  // uniform per block (a block serves one job)
}

template <int BM, int BN, int WM, int WN>
static int launch_wino_gemm(const RowsKP& ap, const RowsKP& bp, const EpiStoreP& ep, int M, int N,
                            int K, int nb, hipStream_t s, AmaxPair amax = AmaxPair{nullptr, nullptr}) {
  constexpr int NT = WM * WN * 64;
  using AL = RowsKLoader<BM, NT>;
  using BL = RowsKLoader<BN, NT>;
  dim3 grid(ceil_div(M, BM), ceil_div(N, BN), nb);
  launch_f32_gemm<BM, BN, WM, WN, AL, BL, EpiStore, RowsKP, RowsKP>(grid, s, ap, bp, ep, M, N, K, K, 1,
                                                                    amax);
  NSM_LAUNCH_CHECK("wino_gemm");
  return 0;
}

static int grid_1d(long long work) {
  long long g = (work + 255) / 256;
  if (g > 16384) g = 16384;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace nsm

using namespace nsm;

// NSM_F32_EPI_VEC=0: the fp32 store epilogue writes 4-byte elements directly
static int f32_epi_vec() {
  static int v = [] {
    const char* e = getenv("NSM_F32_EPI_VEC");
    return (!e || atoi(e) != 0) ? 1 : 0;
  }();
  return v;
}


extern "C" int nsm_pack_conv_weight(const float* w, int cout, int cin, int ksize, int cout_p,
                                    int cin_p, int mode, float* out, void* stream) {
  NSM_CHECK_ARG(w && out && cout > 0 && cin > 0 && cout_p >= cout && cin_p >= cin,
                "pack_conv_weight: bad args");
  NSM_CHECK_ARG(ksize == 1 || ksize == 3, "pack_conv_weight: ksize %d", ksize);
  int taps = ksize * ksize;
  int total = cout_p * cin_p * taps;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(ceil_div(total, 256)), dim3(256), 0,
                     as_stream(stream), w, cout, cin, taps, cout_p, cin_p, mode, out);
  NSM_LAUNCH_CHECK("pack_conv_weight");
  return 0;
}

extern "C" int nsm_pad_vec(const float* v, int n, int n_p, float* out, void* stream) {
  NSM_CHECK_ARG(v && out && n_p >= n, "pad_vec: bad args");
  hipLaunchKernelGGL(pad_vec_kernel, dim3(ceil_div(n_p, 256)), dim3(256), 0, as_stream(stream), v,
                     n, n_p, out);
  NSM_LAUNCH_CHECK("pad_vec");
  return 0;
}

// the job's item count ROUNDED UP to whole blocks of the launch, i.e. the
// amount to advance `base` by (jobs start on block boundaries)
extern "C" long long nsm_prep_items(const NsmPrepJob* j) {
  if (!j) return -1;
  const long long n = nsm_prep_items_dev(*j);
  return n < 0 ? -1 : (n + PREP_ITEMS - 1) / PREP_ITEMS * PREP_ITEMS;
}

extern "C" int nsm_prep_weights(const NsmPrepJob* jobs_dev, int njobs, long long total_items,
                                int max_pass, uint32_t* pmax, uint32_t* zero0, int64_t nzero0,
                                uint32_t* zero1, int64_t nzero1, void* stream) {
  NSM_CHECK_ARG(jobs_dev && njobs > 0 && total_items > 0 && total_items % PREP_ITEMS == 0,
                "prep_weights: bad args");
  NSM_CHECK_ARG(total_items / PREP_ITEMS < (1ll << 31), "prep_weights: too many items");
  NSM_CHECK_ARG(!max_pass || pmax, "prep_weights: the h2 / f16 jobs need pmax (one word per block)");
  NSM_CHECK_ARG((nzero0 == 0 || zero0) && (nzero1 == 0 || zero1) && nzero0 >= 0 && nzero1 >= 0,
                "prep_weights: zero ranges");
  static const bool wide = [] {  // NSM_PREP_WIDE=1: the U jobs by wino_weight_block
    const char* e = getenv("NSM_PREP_WIDE");
    return e && atoi(e) != 0;
  }();
  // phase 0 (the slot zeroing and the max|w| pass of the h2 / f16 jobs) where
  // there is something to do: otherwise every block of it would return
  const bool p0 = max_pass || nzero0 > 0 || nzero1 > 0;
  for (int phase = p0 ? 0 : 1; phase < 2; ++phase)
    hipLaunchKernelGGL(prep_weights_kernel, dim3((unsigned)(total_items / PREP_ITEMS)), dim3(256), 0,
                       as_stream(stream), jobs_dev, njobs, phase | (wide && phase ? 2 : 0), pmax,
                       zero0, (long long)nzero0, zero1, (long long)nzero1);
  NSM_LAUNCH_CHECK("prep_weights");
  return 0;
}

extern "C" int nsm_conv_fwd(const float* x, int ldx, int B, int H, int W, int cin_p,
                            const float* wpk, const float* bias, int cout_p, int ksize, float* y,
                            int ldy, const float* pro_scale, const float* pro_shift,
                            const float* pro_mask, float slope, void* stream) {
  return nsm_conv_fwd_stats(x, ldx, B, H, W, cin_p, wpk, bias, cout_p, ksize, y, ldy, pro_scale,
                            pro_shift, pro_mask, slope, nullptr, nullptr, nullptr, stream);
}

extern "C" int nsm_conv_stat_rows(int B, int H, int W, int cout_p) {
  long long M = (long long)B * H * W;
  return conv_fwd_bm_f(M, cout_p);
}

extern "C" int nsm_conv_fwd_stats(const float* x, int ldx, int B, int H, int W, int cin_p,
                                  const float* wpk, const float* bias, int cout_p, int ksize,
                                  float* y, int ldy, const float* pro_scale, const float* pro_shift,
                                  const float* pro_mask, float slope, float* stats,
                                  const uint32_t* amax_x, const uint32_t* amax_w, void* stream) {
  NSM_CHECK_ARG(x && wpk && y, "conv_fwd: null pointer");
  NSM_CHECK_ARG(B > 0 && H > 0 && W > 0, "conv_fwd: bad shape");
  NSM_CHECK_ARG(cin_p % 32 == 0 && cout_p % 32 == 0, "conv_fwd: channels must be multiples of 32");
  NSM_CHECK_ARG(ldx >= cin_p && ldx % 4 == 0 && ldy >= cout_p, "conv_fwd: bad leading dims");
  NSM_CHECK_ARG(ksize == 1 || ksize == 3, "conv_fwd: ksize %d", ksize);
  NSM_CHECK_ARG(!pro_scale || pro_shift, "conv_fwd: prologue needs scale and shift");
  NSM_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)wpk % 16) == 0, "conv_fwd: 16B alignment");
  long long Ml = (long long)B * H * W;
  NSM_CHECK_ARG(Ml < (1ll << 30), "conv_fwd: too many pixels");
  ConvActP ap;
  ap.x = x;
  ap.ld = ldx;
  ap.cin = cin_p;
  ap.H = H;
  ap.W = W;
  ap.M = (int)Ml;
  ap.ksize = ksize;
  ap.fdW = make_fastdiv(W);
  ap.fdH = make_fastdiv(H);
  ap.scale = pro_scale;
  ap.shift = pro_shift;
  ap.mask = pro_mask ? pro_mask : pro_scale;
  ap.mask_ld = pro_mask ? cin_p : 0;
  ap.mask_on = pro_mask != nullptr;
  ap.slope = slope;
  int K = ksize * ksize * cin_p;
  RowsKP bp{wpk, K, cout_p, 0};
  EpiStoreP ep{y, ldy, bias, stats, 0, nullptr, nullptr, 0.f, nullptr, 0, f32_epi_vec()};
  hipStream_t s = as_stream(stream);
  if (pro_scale) return dispatch_conv_fwd<true>(ap, bp, ep, (int)Ml, cout_p, K, s);
  return dispatch_conv_fwd<false>(ap, bp, ep, (int)Ml, cout_p, K, s, AmaxPair{amax_x, amax_w});
}

static int conv_fwd_act_f32(const float* x, int ldx, int B, int H, int W, int cin_p,
                            const float* wpk, const float* bias, int cout_p, int ksize, float* y,
                            int ldy, const float* act_scale, const float* act_shift, float slope,
                            const float* res, int ldres, hipStream_t s) {
  NSM_CHECK_ARG(x && wpk && y && act_scale && act_shift, "conv_fwd_act: null pointer");
  NSM_CHECK_ARG(B > 0 && H > 0 && W > 0 && cin_p % 32 == 0 && cout_p % 32 == 0,
                "conv_fwd_act: bad shape");
  NSM_CHECK_ARG(ldx >= cin_p && ldx % 4 == 0 && ldy >= cout_p && (!res || ldres >= cout_p),
                "conv_fwd_act: bad leading dims");
  NSM_CHECK_ARG(ksize == 1 || ksize == 3, "conv_fwd_act: ksize %d", ksize);
  NSM_CHECK_ARG(((uintptr_t)x % 16) == 0 && ((uintptr_t)wpk % 16) == 0, "conv_fwd_act: 16B alignment");
  const long long Ml = (long long)B * H * W;
  NSM_CHECK_ARG(Ml < (1ll << 30), "conv_fwd_act: too many pixels");
  ConvActP ap{};
  ap.x = x;
  ap.ld = ldx;
  ap.cin = cin_p;
  ap.H = H;
  ap.W = W;
  ap.M = (int)Ml;
  ap.ksize = ksize;
  ap.fdW = make_fastdiv(W);
  ap.fdH = make_fastdiv(H);
  const int K = ksize * ksize * cin_p;
  RowsKP bp{wpk, K, cout_p, 0};
  EpiStoreP ep{y, ldy, bias, nullptr, 0, act_scale, act_shift, slope, res, ldres, f32_epi_vec()};
  return dispatch_conv_fwd<false>(ap, bp, ep, (int)Ml, cout_p, K, s);
}

extern "C" size_t nsm_conv_wgrad_ws(int B, int H, int W, int cin_p, int cout_p, int ksize) {
  return plan_wgrad(B, H, W, cin_p, cout_p, ksize).ws_floats;
}

extern "C" int nsm_conv_wgrad(const float* dy, int lddy, const float* x, int ldx, int B, int H,
                              int W, int cin_p, int cout_p, int ksize, const float* pro_scale,
                              const float* pro_shift, const float* pro_mask, float slope,
                              float* ws, size_t ws_floats, int cin, int cout, float* dw,
                              const uint32_t* amax_dy, const uint32_t* amax_x, void* stream) {
  NSM_CHECK_ARG(dy && x && ws && dw, "conv_wgrad: null pointer");
  NSM_CHECK_ARG(cin_p % 32 == 0 && cout_p % 32 == 0, "conv_wgrad: channels must be x32");
  NSM_CHECK_ARG(ksize == 1 || ksize == 3, "conv_wgrad: ksize %d", ksize);
  NSM_CHECK_ARG(lddy >= cout_p && ldx >= cin_p && lddy % 4 == 0 && ldx % 4 == 0,
                "conv_wgrad: bad leading dims");
  NSM_CHECK_ARG(!pro_scale || (pro_shift && ksize == 1), "conv_wgrad: prologue needs 1x1");
  NSM_CHECK_ARG(cin <= cin_p && cout <= cout_p, "conv_wgrad: real dims exceed padded");
  WgradPlan pl = plan_wgrad(B, H, W, cin_p, cout_p, ksize);
  NSM_CHECK_ARG(cin_p % pl.BN == 0 || pl.BN % cin_p == 0, "conv_wgrad: N tile straddles taps");
  if (ws_floats < pl.ws_floats)
    return fail(NSM_E_WS, "conv_wgrad: workspace %zu < %zu floats", ws_floats, pl.ws_floats);
  const int M = cout_p, N = ksize * ksize * cin_p;
  const long long Kl = (long long)B * H * W;
  NSM_CHECK_ARG(Kl < (1ll << 30), "conv_wgrad: too many pixels");
  PixRowsP ap{};
  ap.x = dy;
  ap.ld = lddy;
  ap.ncols = cout_p;
  ap.cin = 0;
  ap.H = H;
  ap.W = W;
  ap.M = (int)Kl;
  ap.ksize = 1;
  ap.fdW = make_fastdiv(W);
  ap.fdH = make_fastdiv(H);
  PixRowsP bp = ap;
  bp.x = x;
  bp.ld = ldx;
  bp.ncols = cin_p;
  bp.cin = cin_p;
  bp.ksize = ksize;
  bp.scale = pro_scale;
  bp.shift = pro_shift;
  bp.mask = pro_mask ? pro_mask : pro_scale;
  bp.mask_ld = pro_mask ? cin_p : 0;
  bp.mask_on = pro_mask != nullptr;
  bp.slope = slope;
  EpiSlabP ep{ws, f32_epi_vec()};
  hipStream_t s = as_stream(stream);
  int rc;
  const AmaxPair am{amax_dy, amax_x};
  if (ksize == 3)
    rc = dispatch_wgrad<true, false>(pl.BM, pl.BN, ap, bp, ep, M, N, (int)Kl, pl.kchunk, pl.splits, s,
                                     am);
  else if (pro_scale)
    rc = dispatch_wgrad<false, true>(pl.BM, pl.BN, ap, bp, ep, M, N, (int)Kl, pl.kchunk, pl.splits, s);
  else
    rc = dispatch_wgrad<false, false>(pl.BM, pl.BN, ap, bp, ep, M, N, (int)Kl, pl.kchunk, pl.splits,
                                      s, am);
  if (rc) return rc;
  return wgrad_finish(ws, pl, M, N, cin_p, ksize * ksize, cin, cout, dw, s);
}

// ---- Winograd host side: tile in {2, 4} selects F(2x2,3x3) / F(4x4,3x3) -------
struct WinoGeom {
  int m, alpha2, TH, TW;
  long long T;
};

static bool wino_geom(int tile, int B, int H, int W, WinoGeom& g) {
  if (tile != 2 && tile != 4 && tile != 6) return false;
  g.m = tile;
  g.alpha2 = (tile + 2) * (tile + 2);
  g.TH = (H + tile - 1) / tile;
  g.TW = (W + tile - 1) / tile;
  g.T = (long long)B * g.TH * g.TW;
  return B > 0 && H > 0 && W > 0 && g.T < (1ll << 30);
}

extern "C" size_t nsm_wino_ws(int B, int H, int W, int cin_p, int cout_p, int tile) {
  WinoGeom g;
  if (!wino_geom(tile, B, H, W, g)) return 0;
  return (size_t)g.alpha2 * g.T * (cin_p + cout_p);
}

extern "C" int nsm_wino_weight(const float* w, int cout, int cin, int n_p, int k_p, int flip,
                               int tile, float* U, void* stream) {
  NSM_CHECK_ARG(w && U && n_p % 32 == 0 && k_p % 32 == 0, "wino_weight: bad args");
  NSM_CHECK_ARG(tile == 2 || tile == 4 || tile == 6, "wino_weight: tile must be 2, 4 or 6");
  NSM_CHECK_ARG(flip ? (n_p >= cin && k_p >= cout) : (n_p >= cout && k_p >= cin),
                "wino_weight: padded dims too small");
  dim3 grid(ceil_div(n_p * k_p, 256));
  if (tile == 2)
    hipLaunchKernelGGL(wino_weight_kernel<2>, grid, dim3(256), 0, as_stream(stream), w, cout, cin,
                       n_p, k_p, flip, U);
  else if (tile == 4)
    hipLaunchKernelGGL(wino_weight_kernel<4>, grid, dim3(256), 0, as_stream(stream), w, cout, cin,
                       n_p, k_p, flip, U);
  else
    hipLaunchKernelGGL(wino_weight_kernel<6>, grid, dim3(256), 0, as_stream(stream), w, cout, cin,
                       n_p, k_p, flip, U);
  NSM_LAUNCH_CHECK("wino_weight");
  return 0;
}

extern "C" int nsm_wino_input_resize(const float* x, int ldx, int B, int hi, int wi, int H, int W,
                                     int cin_p, int tile, int relu, float* V, uint32_t* amax,
                                     void* stream) {
  NSM_CHECK_ARG(x && V && cin_p % 32 == 0 && ldx % 4 == 0 && ldx >= cin_p, "wino_input: bad args");
  NSM_CHECK_ARG(hi > 0 && wi > 0, "wino_input: bad source shape");
  NSM_CHECK_ARG(!(relu && (hi != H || wi != W)), "wino_input: relu with a resize");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_input: bad tile or shape");
  dim3 grid(grid_1d(g.T * cin_p / (tile == 6 ? 1 : 4)));
  hipStream_t s = as_stream(stream);
  const bool up = hi != H || wi != W;
  const float sh = ac_scale(hi, H), sw = ac_scale(wi, W);
#define NSM_WI(m, r, u)                                                                           \
  hipLaunchKernelGGL((wino_input_kernel<m, r, u>), grid, dim3(256), 0, s, x, ldx, H, W, cin_p,     \
                     g.TH, g.TW, g.T, V, hi, wi, sh, sw, amax)
  if (tile == 2) {
    if (up) NSM_WI(2, false, true); else if (relu) NSM_WI(2, true, false); else NSM_WI(2, false, false);
  } else if (tile == 4) {
    if (up) NSM_WI(4, false, true); else if (relu) NSM_WI(4, true, false); else NSM_WI(4, false, false);
  } else {
    if (up) NSM_WI(6, false, true); else if (relu) NSM_WI(6, true, false); else NSM_WI(6, false, false);
  }
#undef NSM_WI
  NSM_LAUNCH_CHECK("wino_input");
  return 0;
}

extern "C" int nsm_wino_input(const float* x, int ldx, int B, int H, int W, int cin_p, int tile,
                              int relu, float* V, void* stream) {
  return nsm_wino_input_resize(x, ldx, B, H, W, H, W, cin_p, tile, relu, V, nullptr, stream);
}

// 256x64 tiles for the 64-channel Winograd GEMMs (conv9 at 256^2: fwd 122 ->
// 109 us, dgrad 116 -> 105 us); NSM_WINO_N64_BM256=0: 128x64
static bool wino_n64_bm256() {
  static bool v = [] {
    const char* e = getenv("NSM_WINO_N64_BM256");
    return !e || atoi(e) != 0;
  }();
  return v;
}

extern "C" int nsm_wino_gemm(const float* V, const float* U, int B, int H, int W, int cin_p,
                             int cout_p, int tile, float* Mb, void* stream) {
  return nsm_wino_gemm_s(V, U, B, H, W, cin_p, cout_p, tile, Mb, nullptr, nullptr, stream);
}

extern "C" int nsm_absmax(const float* x, int64_t n, uint32_t* out, void* stream) {
  NSM_CHECK_ARG(x && out && n > 0, "absmax: bad args");
  const long long g = std::min<long long>(ceil_div(n, 1024), 2048);
  hipLaunchKernelGGL(absmax_kernel, dim3((int)g), dim3(256), 0, as_stream(stream), x,
                     (long long)n, out);
  NSM_LAUNCH_CHECK("absmax");
  return 0;
}

extern "C" int nsm_absmax_bf16(const void* x, int64_t n, uint32_t* out, void* stream) {
  NSM_CHECK_ARG(x && out && n > 0 && ((uintptr_t)x % 16) == 0, "absmax_bf16: bad args");
  const long long g = std::min<long long>(ceil_div(n, 2048), 2048);
  hipLaunchKernelGGL(absmax_bf16_kernel, dim3((int)g), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)x, (long long)n, out);
  NSM_LAUNCH_CHECK("absmax_bf16");
  return 0;
}

extern "C" int nsm_wino_gemm_s(const float* V, const float* U, int B, int H, int W, int cin_p,
                               int cout_p, int tile, float* Mb, const uint32_t* amax_v,
                               const uint32_t* amax_u, void* stream) {
  NSM_CHECK_ARG(V && U && Mb && cin_p % 32 == 0 && cout_p % 32 == 0, "wino_gemm: bad args");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_gemm: bad tile or shape");
  hipStream_t s = as_stream(stream);
  RowsKP ap{V, cin_p, (int)g.T, g.T * cin_p};
  RowsKP bp{U, cin_p, cout_p, (long long)cout_p * cin_p};
  EpiStoreP ep{Mb, cout_p, nullptr, nullptr, g.T * cout_p, nullptr, nullptr, 0.f, nullptr, 0,
               f32_epi_vec()};
  const int M = (int)g.T, N = cout_p, K = cin_p, nb = g.alpha2;
  long long mb128 = ceil_div(M, 128);
  // the split kernel runs two blocks per CU (one stage of LDS): 128x128 from
  // two dispatch rounds on
  if (N >= 128)
    return (mb128 * ceil_div(N, 128) * nb >= (f32_split() ? 512 : 1024))
               ? launch_wino_gemm<128, 128, 2, 2>(ap, bp, ep, M, N, K, nb, s, AmaxPair{amax_v, amax_u})
               : launch_wino_gemm<64, 128, 2, 2>(ap, bp, ep, M, N, K, nb, s, AmaxPair{amax_v, amax_u});
  if (N >= 64) {
    // 256x64 (4 waves of 64x64) where the batched grid still has >= 2048 blocks
    if (N == 64 && wino_n64_bm256() && f32_split() && ceil_div(M, 256) * nb >= 2048)
      return launch_wino_gemm<256, 64, 4, 1>(ap, bp, ep, M, N, K, nb, s, AmaxPair{amax_v, amax_u});
    return launch_wino_gemm<128, 64, 2, 2>(ap, bp, ep, M, N, K, nb, s, AmaxPair{amax_v, amax_u});
  }
  return launch_wino_gemm<128, 32, 4, 1>(ap, bp, ep, M, N, K, nb, s, AmaxPair{amax_v, amax_u});
}

// thread slots per channel of the statistics form of the output transform:
// nslot * N4 must fill whole 256-thread blocks (nslot a multiple of
// wino_stat_step). The policy: ~1024 blocks, and 0 (= separate bn_stats pass)
// under 2 tiles per thread, where the grid-stride form loses more parallelism
// than the extra pass costs (measured: conv3-conv5 slower, conv6 even).
// NSM_F6_OUT_CW: channels per thread of the fp32 F(6x6) output transform. 2
// (default): 8-B loads of M — a wave's 64 plane reads carry 512 B each instead
// of 256 B (tools/ubench/plane_read.hip: the 64-plane read of the transform at
// 3.84 TB/s with 4-B lanes, 5.69 with 8-B ones); 1: one channel per thread
static int f6_out_cw() {
  static int v = [] {
    const char* e = getenv("NSM_F6_OUT_CW");
    return (e && atoi(e) == 1) ? 1 : 2;
  }();
  return v;
}
static int wino_out_cw(int tile) { return tile == 6 ? f6_out_cw() : 4; }

static int wino_stat_step(int cout_p, int tile) {
  int a = cout_p / wino_out_cw(tile), b = 256;
  while (b) {
    const int r = a % b;
    a = b;
    b = r;
  }
  return 256 / a;
}
// blocks of the statistics kernel resident at once on the device (every block
// does the same grid-stride work, so a grid past one round leaves a tail:
// F(6x6)'s 128 VGPRs hold 4 blocks per CU, i.e. 1024 blocks)
static int wino_stat_resident(int tile) {
  static int cache[7] = {0, 0, 0, 0, 0, 0, 0};
  if (tile < 0 || tile > 6) return 1024;
  if (cache[tile]) return cache[tile];
  int per = 0, dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) {
    const void* k = tile == 6   ? (f6_out_cw() == 2
                                       ? (const void*)wino_output_kernel<6, true, false, false, false, 2>
                                       : (const void*)wino_output_kernel<6, true>)
                    : tile == 4 ? (const void*)wino_output_kernel<4, true>
                                : (const void*)wino_output_kernel<2, true>;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, 0);
  }
  cache[tile] = (e == hipSuccess && per > 0 && cus > 0) ? per * cus : 1024;
  return cache[tile];
}
// NSM_WINO_STAT_SMALL=0: layers with fewer tiles than the policy's slot count
// (conv3-conv6 of the fp32 step) write Y without statistics and a separate
// bn_stats pass re-reads it; default: the statistics form at one slot per
// tile (the plain form's grid), capped at one resident round as below.
// Interleaved A/B, fp32 B=8 step: conv6 71.8 + 46 (bn_stats) -> 77.9 us
static bool wino_stat_small() {
  static bool v = [] {
    const char* e = getenv("NSM_WINO_STAT_SMALL");
    return !e || atoi(e) != 0;
  }();
  return v;
}
static long long wino_stat_slots(long long T, int cout_p, int tile) {
  const int N4 = cout_p / wino_out_cw(tile), step = wino_stat_step(cout_p, tile);
  // the policy (stats form where a thread covers >= 2 tiles) is judged on
  // ~1024 blocks of one channel per thread for F(6x6) (its decisions as
  // before the 2-channel form); the grid itself is one resident round
  long long ns = (1024ll * 256) / (cout_p / (tile == 6 ? 1 : 4));
  if (ns < 512) ns = 512;
  ns = ns / step * step;
  if (ns < step) ns = step;
  if (T < 2 * ns) {
    if (!wino_stat_small()) return 0;
    ns = T / step * step;
    if (ns < step) return 0;
  }
  long long nr = ((long long)wino_stat_resident(tile) * 256) / N4;
  nr = nr / step * step;
  if (nr >= step && nr < ns) ns = nr;
  return ns;
}

extern "C" int nsm_wino_stat_step(int cout_p, int tile) {
  if (cout_p <= 0 || cout_p % 32 != 0 || (tile != 2 && tile != 4 && tile != 6)) return 0;
  return wino_stat_step(cout_p, tile);
}

extern "C" int nsm_wino_stat_slots(int B, int H, int W, int cout_p, int tile) {
  WinoGeom g;
  if (!wino_geom(tile, B, H, W, g) || cout_p % 32 != 0) return 0;
  return (int)wino_stat_slots(g.T, cout_p, tile);
}

template <int MT, int CWX = 0>
static void launch_wino_output(dim3 grid, hipStream_t s, const float* Mb, int cout_p, int H, int W,
                               const WinoGeom& g, const float* bias, float* y, int ldy,
                               float* partial, const WinoAct* act = nullptr) {
  if (act)
    hipLaunchKernelGGL((wino_output_kernel<MT, false, true, false, false, CWX>), grid, dim3(256), 0, s,
                       Mb, cout_p, H, W, g.TH, g.TW, g.T, bias, y, ldy, nullptr, *act);
  else if (partial)
    hipLaunchKernelGGL((wino_output_kernel<MT, true, false, false, false, CWX>), grid, dim3(256), 0, s,
                       Mb, cout_p, H, W, g.TH, g.TW, g.T, bias, y, ldy, partial);
  else
    hipLaunchKernelGGL((wino_output_kernel<MT, false, false, false, false, CWX>), grid, dim3(256), 0, s,
                       Mb, cout_p, H, W, g.TH, g.TW, g.T, bias, y, ldy, partial);
}
// wino_output_kernel<6, STATS, false, false, false, 2> (the fp32 step's F(6x6)
// output transform) on 32-bit buffer offsets (host-checked: M under 4 GiB, y
// under 2 GiB, T x N / 2 under 2^31): M's plane in the scalar offset of one
// descriptor, y's rows through another. Same arithmetic and order.
template <bool STATS>
__global__ void __launch_bounds__(256) wino_output6_buf_kernel(const float* __restrict__ Mb, int N,
                                                               int H, int W, int TH, int TW, int T,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ y, int ldy,
                                                               float* __restrict__ partial) {
  constexpr int MT = 6, A = 8, CW = 2;
  using VT = f32x2;
  const int N4 = N / CW;
  const int total = T * N4;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = T / (TH * TW);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)Mb, (short)0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(y, (long long)nb * H * W * ldy);
  const uint32_t pbytes = (uint32_t)T * (uint32_t)N * 4u;
  VT s_sum{}, s_mean{}, s_m2{};
  float s_n = 0.f;
  for (int i = i0; i < total; i += gridDim.x * blockDim.x) {
    const int c = (i % N4) * CW;
    const int t = i / N4;
    const int tx = t % TW;
    const int r = t / TW;
    const int ty = r % TH;
    const int b = r / TH;
    const uint32_t mo = (uint32_t)(t * N + c) * 4u;
    VT sc[MT][A], o[MT][MT];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      VT row[A];
#pragma unroll
      for (int e = 0; e < A; ++e)
        row[e] = __builtin_bit_cast(VT, __builtin_amdgcn_raw_buffer_load_b64(
                                            mr, mo, (int)((uint32_t)(a * A + e) * pbytes), 0));
      wcol_row<CAt<MT>>(sc, row, a);
    }
#pragma unroll
    for (int a = 0; a < MT; ++a) wmat<CAt<MT>>(sc[a], o[a]);
    const VT bv = bias ? *(const VT*)(bias + c) : VT{};
    VT ts{};
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int yy = MT * ty + a;
      if (yy >= H) continue;
      const uint32_t ro = (uint32_t)(((b * H + yy) * W + MT * tx) * ldy + c) * 4u;
#pragma unroll
      for (int e = 0; e < MT; ++e)
        if (MT * tx + e < W) {
          o[a][e] = o[a][e] + bv;
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(mr, 0u, 0, 0)), o[a][e]),
              yr, ro + (uint32_t)(e * ldy) * 4u, 0, 0);
          if (STATS) ts = ts + o[a][e];
        }
    }
    if (STATS) {
      const int nv = min(MT, H - MT * ty) * min(MT, W - MT * tx);
      const VT tmean = ts * (1.f / (float)nv);
      VT tq{};
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int e = 0; e < MT; ++e)
          if (MT * ty + a < H && MT * tx + e < W) {
            const VT d = o[a][e] - tmean;
            tq = tq + d * d;
          }
      const float n2 = s_n + (float)nv;
      const VT delta = tmean - s_mean;
      s_mean = s_mean + delta * ((float)nv / n2);
      s_m2 = s_m2 + tq + delta * delta * (s_n * (float)nv / n2);
      s_sum = s_sum + ts;
      s_n = n2;
    }
  }
  if (STATS && i0 < (int)(gridDim.x * blockDim.x)) {
    const int c = (i0 % N4) * CW;
    float* pr = partial + (size_t)(i0 / N4) * 3 * N + c;
    *(VT*)pr = s_sum;
    *(VT*)(pr + N) = s_m2;
    *(VT*)(pr + 2 * N) = VT{} + s_n;
  }
}

// NSM_F6_OUT_BUF=0: the generic kernel for the fp32 F(6x6) output transform
static bool f6_out_buf() {
  static bool v = [] {
    const char* e = getenv("NSM_F6_OUT_BUF");
    return !e || atoi(e) != 0;
  }();
  return v;
}

static void launch_wino_output6(dim3 grid, hipStream_t s, const float* Mb, int cout_p, int H, int W,
                                const WinoGeom& g, const float* bias, float* y, int ldy,
                                float* partial, const WinoAct* act = nullptr) {
  const long long B = g.T / ((long long)g.TH * g.TW);
  if (f6_out_cw() == 2 && !act && f6_out_buf() && 64ll * g.T * cout_p * 4 < 0xFFFFFFFFll &&
      B * H * W * ldy * 4 < 0x7FFFFFFFll && g.T * (cout_p / 2) < (1ll << 31)) {
    if (partial)
      hipLaunchKernelGGL(wino_output6_buf_kernel<true>, grid, dim3(256), 0, s, Mb, cout_p, H, W, g.TH,
                         g.TW, (int)g.T, bias, y, ldy, partial);
    else
      hipLaunchKernelGGL(wino_output6_buf_kernel<false>, grid, dim3(256), 0, s, Mb, cout_p, H, W, g.TH,
                         g.TW, (int)g.T, bias, y, ldy, nullptr);
    return;
  }
  if (f6_out_cw() == 2)
    launch_wino_output<6, 2>(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, partial, act);
  else
    launch_wino_output<6>(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, partial, act);
}

extern "C" int nsm_wino_output_stats(const float* Mb, int B, int H, int W, int cout_p, int tile,
                                     const float* bias, float* y, int ldy, float* partial,
                                     int nslot, void* stream) {
  NSM_CHECK_ARG(Mb && y && cout_p % 32 == 0 && ldy % 4 == 0, "wino_output: bad args");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_output: bad tile or shape");
  const int N4 = cout_p / wino_out_cw(tile);
  dim3 grid(grid_1d(g.T * N4));
  if (partial) {
    NSM_CHECK_ARG(nslot > 0 && nslot % wino_stat_step(cout_p, tile) == 0 && nslot <= (1 << 20),
                  "wino_output: nslot %d not a multiple of %d", nslot,
                  wino_stat_step(cout_p, tile));
    grid = dim3((unsigned)((long long)nslot * N4 / 256));
  }
  hipStream_t s = as_stream(stream);
  if (tile == 2) launch_wino_output<2>(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, partial);
  else if (tile == 4) launch_wino_output<4>(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, partial);
  else launch_wino_output6(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, partial);
  NSM_LAUNCH_CHECK("wino_output");
  return 0;
}

extern "C" int nsm_wino_output_act(const float* Mb, int B, int H, int W, int cout_p, int tile,
                                   const float* bias, float* y, int ldy, const float* act_scale,
                                   const float* act_shift, float slope, const float* res,
                                   int ldres, void* stream) {
  NSM_CHECK_ARG(Mb && y && act_scale && act_shift && cout_p % 32 == 0 && ldy % 4 == 0 &&
                    (!res || (ldres % 4 == 0 && ldres >= cout_p)),
                "wino_output_act: bad args");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_output_act: bad tile or shape");
  const WinoAct act{act_scale, act_shift, slope, res, ldres};
  dim3 grid(grid_1d(g.T * (cout_p / wino_out_cw(tile))));
  hipStream_t s = as_stream(stream);
  if (tile == 2) launch_wino_output<2>(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, nullptr, &act);
  else if (tile == 4) launch_wino_output<4>(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, nullptr, &act);
  else launch_wino_output6(grid, s, Mb, cout_p, H, W, g, bias, y, ldy, nullptr, &act);
  NSM_LAUNCH_CHECK("wino_output_act");
  return 0;
}

extern "C" int nsm_wino_output(const float* Mb, int B, int H, int W, int cout_p, int tile,
                               const float* bias, float* y, int ldy, void* stream) {
  return nsm_wino_output_stats(Mb, B, H, W, cout_p, tile, bias, y, ldy, nullptr, 0, stream);
}

extern "C" int nsm_conv3x3_wino(const float* x, int ldx, int B, int H, int W, int cin_p,
                                const float* U, const float* bias, int cout_p, int tile, int relu,
                                float* y, int ldy, float* ws, size_t ws_floats, void* stream) {
  NSM_CHECK_ARG(x && U && y && ws, "conv3x3_wino: null pointer");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "conv3x3_wino: bad tile or shape");
  if (ws_floats < nsm_wino_ws(B, H, W, cin_p, cout_p, tile))
    return fail(NSM_E_WS, "conv3x3_wino: workspace too small");
  float* V = ws;
  float* Mb = ws + (size_t)g.alpha2 * g.T * cin_p;
  int rc = nsm_wino_input(x, ldx, B, H, W, cin_p, tile, relu, V, stream);
  if (!rc) rc = nsm_wino_gemm(V, U, B, H, W, cin_p, cout_p, tile, Mb, stream);
  if (!rc) rc = nsm_wino_output(Mb, B, H, W, cout_p, tile, bias, y, ldy, stream);
  return rc;
}

// ---- Winograd weight gradient -------------------------------------------------
struct WinoWgradPlan {
  int BM, BN, splits, kchunk;
  size_t slab_floats, dm_floats;
};

static WinoWgradPlan plan_wino_wgrad(long long T, int cin_p, int cout_p, int nb) {
  WinoWgradPlan p;
  p.BM = cout_p >= 128 ? 128 : (cout_p >= 64 ? 64 : 32);
  p.BN = cin_p >= 128 ? 128 : (cin_p >= 64 ? 64 : 32);
  long long tiles = (long long)ceil_div(cout_p, p.BM) * ceil_div(cin_p, p.BN) * nb;
  long long want = (4096 + tiles - 1) / tiles;
  long long maxs = (T + 255) / 256;
  long long sp = want < maxs ? want : maxs;
  if (sp > 64) sp = 64;
  if (sp < 1) sp = 1;
  long long kc = (T + sp - 1) / sp;
  kc = (kc + BK - 1) / BK * BK;
  sp = (T + kc - 1) / kc;
  p.splits = (int)sp;
  p.kchunk = (int)kc;
  p.slab_floats = (size_t)nb * sp * cout_p * cin_p;
  if (sp > 1) p.slab_floats += (size_t)nb * cout_p * cin_p;  // split-summed dU
  p.dm_floats = (size_t)nb * T * cout_p;
  return p;
}

extern "C" size_t nsm_wino_wgrad_ws(int B, int H, int W, int cin_p, int cout_p, int tile) {
  WinoGeom g;
  if (!wino_geom(tile, B, H, W, g)) return 0;
  WinoWgradPlan p = plan_wino_wgrad(g.T, cin_p, cout_p, g.alpha2);
  return p.slab_floats + p.dm_floats;
}

template <int BM, int BN, int WM, int WN>
static int launch_wino_wgrad(const PixRowsP& ap, const PixRowsP& bp, const EpiSlabP& ep, int M,
                             int N, int K, int kchunk, int splits, int nb, hipStream_t s,
                             AmaxPair amax) {
  constexpr int NT = WM * WN * 64;
  using AL = PixRowsLoader<BM, NT, false, false>;
  using BL = PixRowsLoader<BN, NT, false, false>;
  dim3 grid(ceil_div(M, BM), ceil_div(N, BN), nb * splits);
  launch_f32_gemm<BM, BN, WM, WN, AL, BL, EpiSlabV, PixRowsP, PixRowsP>(grid, s, ap, bp, ep, M, N, K,
                                                                        kchunk, splits, amax);
  NSM_LAUNCH_CHECK("wino_wgrad_gemm");
  return 0;
}

extern "C" int nsm_wino_dual_input(const float* dy, int lddy, int B, int H, int W, int c_p,
                                   int tile, float* V, float* dM, uint32_t* amax_v,
                                   uint32_t* amax_dm, void* stream) {
  NSM_CHECK_ARG(dy && V && dM && c_p % 32 == 0 && lddy % 4 == 0 && lddy >= c_p,
                "wino_dual_input: bad args");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_dual_input: bad tile or shape");
  dim3 grid(grid_1d(g.T * c_p / (tile == 6 ? 1 : 4)));
  hipStream_t s = as_stream(stream);
  if (tile == 2)
    hipLaunchKernelGGL(wino_dual_kernel<2>, grid, dim3(256), 0, s, dy, lddy, H, W, c_p, g.TH, g.TW,
                       g.T, V, dM, WinoBnSrc{}, amax_v, amax_dm);
  else if (tile == 4)
    hipLaunchKernelGGL(wino_dual_kernel<4>, grid, dim3(256), 0, s, dy, lddy, H, W, c_p, g.TH, g.TW,
                       g.T, V, dM, WinoBnSrc{}, amax_v, amax_dm);
  else
    hipLaunchKernelGGL(wino_dual_kernel<6>, grid, dim3(256), 0, s, dy, lddy, H, W, c_p, g.TH, g.TW,
                       g.T, V, dM, WinoBnSrc{}, amax_v, amax_dm);
  NSM_LAUNCH_CHECK("wino_dual_input");
  return 0;
}

extern "C" int nsm_wino_dual_input_bn(const float* g, int ldg, const float* y, int ldy, int B,
                                      int H, int W, int c_p, int tile, const float* scale,
                                      const float* shift, float slope, const float* mask,
                                      const float* mean, const float* coef, float* V, float* dM,
                                      uint32_t* amax_v, uint32_t* amax_dm, void* stream) {
  NSM_CHECK_ARG(g && y && V && dM && scale && shift && mean && coef && c_p % 32 == 0 &&
                    ldg % 4 == 0 && ldg >= c_p && ldy % 4 == 0 && ldy >= c_p,
                "wino_dual_input_bn: bad args");
  WinoGeom geo;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, geo), "wino_dual_input_bn: bad tile or shape");
  dim3 grid(grid_1d(geo.T * c_p / (tile == 6 ? 1 : 4)));
  hipStream_t s = as_stream(stream);
  const WinoBnSrc bn{y, ldy, scale, shift, mean, coef, mask, slope};
#define A_ g, ldg, H, W, c_p, geo.TH, geo.TW, geo.T, V, dM, bn, amax_v, amax_dm
  if (tile == 2) hipLaunchKernelGGL((wino_dual_kernel<2, true>), grid, dim3(256), 0, s, A_);
  else if (tile == 4) hipLaunchKernelGGL((wino_dual_kernel<4, true>), grid, dim3(256), 0, s, A_);
  else hipLaunchKernelGGL((wino_dual_kernel<6, true>), grid, dim3(256), 0, s, A_);
#undef A_
  NSM_LAUNCH_CHECK("wino_dual_input_bn");
  return 0;
}

static int wgrad_wino(const float* dy, int lddy, const float* dM_in, const float* V, int B, int H,
                      int W, int cin_p, int cout_p, int cin, int cout, int tile, float* dw,
                      float* ws, size_t ws_floats, void* stream, AmaxPair amax = AmaxPair{});
static int wgrad_wino_finish(float* slab, const WinoWgradPlan& pl, int nb, int M, int N, int cin,
                             int cout, int tile, float* dw, hipStream_t s);

extern "C" int nsm_conv3x3_wgrad_wino(const float* dy, int lddy, const float* V, int B, int H,
                                      int W, int cin_p, int cout_p, int cin, int cout, int tile,
                                      float* dw, float* ws, size_t ws_floats, void* stream) {
  return wgrad_wino(dy, lddy, nullptr, V, B, H, W, cin_p, cout_p, cin, cout, tile, dw, ws,
                    ws_floats, stream);
}

// the weight gradient from a dM nsm_wino_dual_input already wrote (no dY read)
extern "C" int nsm_conv3x3_wgrad_wino_dm(const float* dM, const float* V, int B, int H, int W,
                                         int cin_p, int cout_p, int cin, int cout, int tile,
                                         float* dw, float* ws, size_t ws_floats,
                                         const uint32_t* amax_dm, const uint32_t* amax_v,
                                         void* stream) {
  NSM_CHECK_ARG(dM, "conv3x3_wgrad_wino_dm: null dM");
  return wgrad_wino(nullptr, cout_p, dM, V, B, H, W, cin_p, cout_p, cin, cout, tile, dw, ws,
                    ws_floats, stream, AmaxPair{amax_dm, amax_v});
}

static int wgrad_wino(const float* dy, int lddy, const float* dM_in, const float* V, int B, int H,
                      int W, int cin_p, int cout_p, int cin, int cout, int tile, float* dw,
                      float* ws, size_t ws_floats, void* stream, AmaxPair amax) {
  NSM_CHECK_ARG((dy || dM_in) && V && dw && ws, "conv3x3_wgrad_wino: null pointer");
  NSM_CHECK_ARG(cin_p % 32 == 0 && cout_p % 32 == 0 && lddy % 4 == 0 && cin <= cin_p &&
                    cout <= cout_p, "conv3x3_wgrad_wino: bad channels");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "conv3x3_wgrad_wino: bad tile or shape");
  const int nb = g.alpha2;
  WinoWgradPlan pl = plan_wino_wgrad(g.T, cin_p, cout_p, nb);
  if (ws_floats < pl.slab_floats + pl.dm_floats)
    return fail(NSM_E_WS, "conv3x3_wgrad_wino: workspace too small");
  hipStream_t s = as_stream(stream);
  float* slab = ws;
  float* dM = ws + pl.slab_floats;
  dim3 g1(grid_1d(g.T * cout_p / (tile == 6 ? 1 : 4)));
  if (dM_in)
    dM = (float*)dM_in;
  else if (tile == 2)
    hipLaunchKernelGGL(wino_dout_kernel<2>, g1, dim3(256), 0, s, dy, lddy, H, W, cout_p, g.TH, g.TW,
                       g.T, dM);
  else if (tile == 4)
    hipLaunchKernelGGL(wino_dout_kernel<4>, g1, dim3(256), 0, s, dy, lddy, H, W, cout_p, g.TH, g.TW,
                       g.T, dM);
  else
    hipLaunchKernelGGL(wino_dout_kernel<6>, g1, dim3(256), 0, s, dy, lddy, H, W, cout_p, g.TH, g.TW,
                       g.T, dM);
  NSM_LAUNCH_CHECK("wino_dout");
  PixRowsP ap{};
  ap.x = dM;
  ap.ld = cout_p;
  ap.ncols = cout_p;
  ap.cin = 0;
  ap.H = 1;
  ap.W = 1;
  ap.M = (int)g.T;
  ap.ksize = 1;
  ap.fdW = make_fastdiv(1);
  ap.fdH = make_fastdiv(1);
  ap.bstride = g.T * cout_p;
  PixRowsP bp = ap;
  bp.x = V;
  bp.ld = cin_p;
  bp.ncols = cin_p;
  bp.bstride = g.T * cin_p;
  EpiSlabP ep{slab, f32_epi_vec()};
  const int M = cout_p, N = cin_p, K = (int)g.T;
  int rc;
#define NSM_WW(bm, bn, wm, wn) \
  if (pl.BM == bm && pl.BN == bn) \
    rc = launch_wino_wgrad<bm, bn, wm, wn>(ap, bp, ep, M, N, K, pl.kchunk, pl.splits, nb, s, amax); \
  else
  NSM_WW(128, 128, 2, 2)
  NSM_WW(128, 64, 2, 2)
  NSM_WW(64, 128, 2, 2)
  NSM_WW(64, 64, 2, 2)
  NSM_WW(128, 32, 4, 1)
  NSM_WW(32, 128, 1, 4)
  NSM_WW(64, 32, 2, 1)
  NSM_WW(32, 64, 1, 2)
  rc = launch_wino_wgrad<32, 32, 1, 1>(ap, bp, ep, M, N, K, pl.kchunk, pl.splits, nb, s, amax);
#undef NSM_WW
  if (rc) return rc;
  return wgrad_wino_finish(slab, pl, nb, M, N, cin, cout, tile, dw, s);
}

// split-K partials -> one dU per xi with a parallel, fixed-order sum (the
// transform kernel then reads alpha^2 values per output weight) -> dw
static int wgrad_wino_finish(float* slab, const WinoWgradPlan& pl, int nb, int M, int N, int cin,
                             int cout, int tile, float* dw, hipStream_t s) {
  const float* du = slab;
  int du_splits = pl.splits;
  if (pl.splits > 1) {
    float* sum = slab + (size_t)nb * pl.splits * M * N;
    const long long L4 = (long long)M * N / 4;
    hipLaunchKernelGGL(batched_splitsum_kernel, dim3(ceil_div(L4, 256), nb), dim3(256), 0, s, slab,
                       pl.splits, L4, sum);
    NSM_LAUNCH_CHECK("wino_wgrad splitsum");
    du = sum;
    du_splits = 1;
  }
  dim3 g2(ceil_div(cout * cin, 256));
  if (tile == 2)
    hipLaunchKernelGGL(wino_wgrad_out_kernel<2>, g2, dim3(256), 0, s, du, du_splits, M, N, cin,
                       cout, dw);
  else if (tile == 4)
    hipLaunchKernelGGL(wino_wgrad_out_kernel<4>, g2, dim3(256), 0, s, du, du_splits, M, N, cin,
                       cout, dw);
  else
    hipLaunchKernelGGL(wino_wgrad_out_kernel<6>, g2, dim3(256), 0, s, du, du_splits, M, N, cin,
                       cout, dw);
  NSM_LAUNCH_CHECK("wino_wgrad_out");
  return 0;
}

// The 16-bit conv body twice: bf16 (namespace nsm_bf) and f16 (nsm_h). Not
// nested in nsm: argument-dependent lookup on nsm's types (F8) would otherwise
// see nsm's bf16 helpers beside nsm_h's f16 ones.
namespace nsm_bf {
using namespace nsm;
__device__ __forceinline__ f32x16 mfma_s16_32(bf16x8 a, bf16x8 b, f32x16 c, int, int, int) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_s16_16(bf16x8 a, bf16x8 b, f32x4 c, int, int, int) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// bits of a value already rounded to bf16 (round_bf)
__device__ __forceinline__ bf16_t s16_bits(float v) { return (bf16_t)(__float_as_uint(v) >> 16); }
__device__ __forceinline__ void st8s(bf16_t* p, F8 v) { nsm::st8(p, v); }
#include "nsm_conv_s16.inc"
}  // namespace nsm_bf
namespace nsm_h {
using namespace nsm;
#include "nsm_fmt_f16.h"
#include "nsm_conv_s16.inc"
}  // namespace nsm_h

using namespace nsm;
using namespace nsm_bf;

#include "nsm_conv_bf16.inc"
#include "nsm_conv_h2.inc"
#include "nsm_conv_h2d.inc"

extern "C" float nsm_wino_beta(int tile, int which) {
  return (tile == 2 || tile == 4 || tile == 6) && which >= 0 && which <= 2 ? wino_beta(tile, which)
                                                                          : 0.f;
}

// NSM_WINO_IN_LDS=1: the F(6x6) h2 input transform on the LDS-region kernel
// (wino_input_lds_kernel) instead of the per-thread one. Measured (B=8 step,
// one box): conv7 170.6 -> 208.5 us, conv8 157.4 -> 189.0, conv6 81.8 ->
// 100.6; step 723 -> 716 frames/s — off: the per-thread kernel's source-row
// reuse already keeps its loads cheap, and the region phase serialises the
// block's reads before its writes at 3 blocks per CU
static bool wino_in_lds() {
  static bool v = [] {
    const char* e = getenv("NSM_WINO_IN_LDS");
    return e && atoi(e) != 0;
  }();
  return v;
}

extern "C" int nsm_wino_input_h2(const float* x, int ldx, int B, int hi, int wi, int H, int W,
                                 int cin_p, int tile, void* Vh, const uint32_t* amax_x,
                                 void* stream) {
  NSM_CHECK_ARG(x && Vh && amax_x && cin_p % 32 == 0 && ldx % 4 == 0 && ldx >= cin_p,
                "wino_input_h2: bad args");
  NSM_CHECK_ARG(hi > 0 && wi > 0 && ((uintptr_t)Vh % 16) == 0, "wino_input_h2: bad source / alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_input_h2: bad tile or shape");
  dim3 grid(grid_1d(g.T * cin_p / (tile == 6 ? 1 : 4)));
  hipStream_t s = as_stream(stream);
  const bool up = hi != H || wi != W;
  const float sh = ac_scale(hi, H), sw = ac_scale(wi, W);
  const H2Scale sc{amax_x, wino_beta(tile, 0)};
  bf16_t* V = (bf16_t*)Vh;
  if (tile == 6 && wino_in_lds() && B * (cin_p / 32) <= 65535) {
    const dim3 grid2(ceil_div(g.TW, 4) * ceil_div(g.TH, 2), B * (cin_p / 32));
    if (up)
      hipLaunchKernelGGL((wino_input_lds_kernel<6, 2, 4, true>), grid2, dim3(256), 0, s, x, ldx, H, W,
                         cin_p, g.TH, g.TW, g.T, hi, wi, sh, sw, V, sc);
    else
      hipLaunchKernelGGL((wino_input_lds_kernel<6, 2, 4, false>), grid2, dim3(256), 0, s, x, ldx, H,
                         W, cin_p, g.TH, g.TW, g.T, hi, wi, sh, sw, V, sc);
    NSM_LAUNCH_CHECK("wino_input_h2");
    return 0;
  }
  const bool uni = (cin_p / (tile == 6 ? 1 : 4)) % 64 == 0;
#define NSM_WI(m, u, un)                                                                          \
  hipLaunchKernelGGL((wino_input_kernel<m, false, u, true, un>), grid, dim3(256), 0, s, x, ldx, H, \
                     W, cin_p, g.TH, g.TW, g.T, nullptr, hi, wi, sh, sw, nullptr, V, sc)
  if (tile == 2) {
    if (up && uni) NSM_WI(2, true, true); else if (up) NSM_WI(2, true, false); else NSM_WI(2, false, false);
  } else if (tile == 4) {
    if (up && uni) NSM_WI(4, true, true); else if (up) NSM_WI(4, true, false); else NSM_WI(4, false, false);
  } else {
    if (up && uni)
      hipLaunchKernelGGL((wino_input_kernel<6, false, true, true, true, 3>), grid, dim3(256), 0, s,
                         x, ldx, H, W, cin_p, g.TH, g.TW, g.T, nullptr, hi, wi, sh, sw, nullptr, V, sc);
    else if (up) NSM_WI(6, true, false); else NSM_WI(6, false, false);
  }
#undef NSM_WI
  NSM_LAUNCH_CHECK("wino_input_h2");
  return 0;
}

extern "C" int nsm_wino_dual_input_h2(const float* dy, int lddy, int B, int H, int W, int c_p,
                                      int tile, void* Vh, void* dMh, const uint32_t* amax_dy,
                                      void* stream) {
  NSM_CHECK_ARG(dy && Vh && dMh && amax_dy && c_p % 32 == 0 && lddy % 4 == 0 && lddy >= c_p,
                "wino_dual_input_h2: bad args");
  NSM_CHECK_ARG(((uintptr_t)Vh % 16) == 0 && ((uintptr_t)dMh % 16) == 0, "wino_dual_input_h2: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_dual_input_h2: bad tile or shape");
  dim3 grid(grid_1d(g.T * c_p / (tile == 6 ? 1 : 4)));
  hipStream_t s = as_stream(stream);
  const H2Scale hv{amax_dy, wino_beta(tile, 0)}, hd{amax_dy, wino_beta(tile, 1)};
#define A_ dy, lddy, H, W, c_p, g.TH, g.TW, g.T, nullptr, nullptr, WinoBnSrc{}, nullptr, nullptr, \
           (bf16_t*)Vh, (bf16_t*)dMh, hv, hd
  if (tile == 2) hipLaunchKernelGGL((wino_dual_kernel<2, false, true>), grid, dim3(256), 0, s, A_);
  else if (tile == 4) hipLaunchKernelGGL((wino_dual_kernel<4, false, true>), grid, dim3(256), 0, s, A_);
  else hipLaunchKernelGGL((wino_dual_kernel<6, false, true>), grid, dim3(256), 0, s, A_);
#undef A_
  NSM_LAUNCH_CHECK("wino_dual_input_h2");
  return 0;
}

// NSM_DUAL_LDS=0: the F(6x6) BN-fused h2 dual transform on the per-thread
// kernel (wino_dual_kernel) instead of the LDS-region one
static bool dual_lds() {
  static bool v = [] {
    const char* e = getenv("NSM_DUAL_LDS");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// wino_dual_input_h2 of a BN backward whose apply pass was not run
// (nsm_wino_dual_input_bn's operands): dY1 = k1 dz + k2 (y - mean) + k3 is
// formed per patch element and never stored; the h2 scale source is `bound`,
// the dY1 bound nsm_bn_bwd_finalize derives from max|k1 dz| (its amax_k1dz),
// which the GEMMs reading Vd / dM take as their operand scale source too
extern "C" int nsm_wino_dual_input_bn_h2(const float* g, int ldg, const float* y, int ldy, int B,
                                         int H, int W, int c_p, int tile, const float* scale,
                                         const float* shift, float slope, const float* mask,
                                         const float* mean, const float* coef, void* Vh, void* dMh,
                                         const uint32_t* bound, void* stream) {
  NSM_CHECK_ARG(g && y && Vh && dMh && scale && shift && mean && coef && bound && c_p % 32 == 0 &&
                    ldg % 4 == 0 && ldg >= c_p && ldy % 4 == 0 && ldy >= c_p,
                "wino_dual_input_bn_h2: bad args");
  NSM_CHECK_ARG(((uintptr_t)Vh % 16) == 0 && ((uintptr_t)dMh % 16) == 0,
                "wino_dual_input_bn_h2: alignment");
  WinoGeom geo;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, geo), "wino_dual_input_bn_h2: bad tile or shape");
  dim3 grid(grid_1d(geo.T * c_p / (tile == 6 ? 1 : 4)));
  hipStream_t s = as_stream(stream);
  const WinoBnSrc bn{y, ldy, scale, shift, mean, coef, mask, slope};
  const H2Scale hv{bound, wino_beta(tile, 0)}, hd{bound, wino_beta(tile, 1)};
  if (tile == 6 && dual_lds()) {
    NSM_CHECK_ARG(B * (c_p / 32) <= 65535, "wino_dual_input_bn_h2: grid");
    const dim3 grid2(ceil_div(geo.TW, 4) * ceil_div(geo.TH, 2), B * (c_p / 32));
    hipLaunchKernelGGL((wino_dual_bn_lds_kernel<6, 2, 4>), grid2, dim3(256), 0, s, g, ldg, H, W, c_p,
                       geo.TH, geo.TW, geo.T, bn, (bf16_t*)Vh, (bf16_t*)dMh, hv, hd);
    NSM_LAUNCH_CHECK("wino_dual_input_bn_h2");
    return 0;
  }
#define A_ g, ldg, H, W, c_p, geo.TH, geo.TW, geo.T, nullptr, nullptr, bn, nullptr, nullptr, \
           (bf16_t*)Vh, (bf16_t*)dMh, hv, hd
  if (tile == 2) hipLaunchKernelGGL((wino_dual_kernel<2, true, true>), grid, dim3(256), 0, s, A_);
  else if (tile == 4) hipLaunchKernelGGL((wino_dual_kernel<4, true, true>), grid, dim3(256), 0, s, A_);
  else hipLaunchKernelGGL((wino_dual_kernel<6, true, true>), grid, dim3(256), 0, s, A_);
#undef A_
  NSM_LAUNCH_CHECK("wino_dual_input_bn_h2");
  return 0;
}

// NSM_H2_WG256=0: the h2 weight gradients keep 128x128 tiles where 256x256 fit
static bool h2_wg256() {
  static bool v = [] {
    const char* e = getenv("NSM_H2_WG256");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// the h2 weight-gradient plan: plan_wino_wgrad's, or 256x256 tiles (8 waves,
// the forward's tile) where both channel counts are multiples of 256, with the
// split count that brings the grid to ~1024 blocks (4 rounds of one block per CU)
// splits of a batched weight-gradient GEMM over T tiles for ~target blocks
static void wino_wgrad_resplit(WinoWgradPlan& p, long long T, int cin_p, int cout_p, int nb,
                               long long target) {
  const long long tiles = (long long)ceil_div(cout_p, p.BM) * ceil_div(cin_p, p.BN) * nb;
  long long sp = (target + tiles - 1) / tiles, maxs = (T + 255) / 256;
  if (sp > maxs) sp = maxs;
  if (sp > 64) sp = 64;
  if (sp < 1) sp = 1;
  long long kc = (T + sp - 1) / sp;
  kc = (kc + BK - 1) / BK * BK;
  sp = (T + kc - 1) / kc;
  p.splits = (int)sp;
  p.kchunk = (int)kc;
  p.slab_floats = (size_t)nb * sp * cout_p * cin_p;
  if (sp > 1) p.slab_floats += (size_t)nb * cout_p * cin_p;
}

static WinoWgradPlan plan_wino_wgrad_h2(long long T, int cin_p, int cout_p, int nb) {
  WinoWgradPlan p = plan_wino_wgrad(T, cin_p, cout_p, nb);
  // the 128 / 64 tiles run two blocks per CU: one round of ~512 blocks
  // (plan_wino_wgrad's ~4096 wrote 64 x 57 partial dU slabs at conv8; A/B
  // 4096 / 1024 / 512: 658-659 / 661-663 / 664 frames/s)
  static const long long target = [] {
    const char* e = getenv("NSM_H2_WG_BLOCKS");
    return e ? atoll(e) : 512ll;
  }();
  wino_wgrad_resplit(p, T, cin_p, cout_p, nb, target);
  if (!h2_wg256() || cin_p % 256 || cout_p % 256) return p;
  p.BM = p.BN = 256;
  const long long tiles = (long long)(cout_p / 256) * (cin_p / 256) * nb;
  static const long long target256 = [] {
    const char* e = getenv("NSM_H2_WG256_BLOCKS");
    return e ? atoll(e) : 1024ll;
  }();
  long long sp = (target256 + tiles - 1) / tiles, maxs = (T + 255) / 256;
  // a full round of unsplit blocks stays unsplit (conv7: 256 tiles x K = 3872,
  // no partial slabs, no split sum; A/B 694 -> 698 frames/s against 4 splits)
  if (tiles >= cu_count()) sp = 1;
  if (sp > maxs) sp = maxs;
  if (sp > 64) sp = 64;
  if (sp < 1) sp = 1;
  long long kc = (T + sp - 1) / sp;
  kc = (kc + BK - 1) / BK * BK;
  sp = (T + kc - 1) / kc;
  // (conv5's F(4x4) at 32x32: 144 tiles x 2 splits = 288 blocks, measured
  // 52.5 -> 63.5 us: keep the 128x128 plan under three rounds of blocks)
  if (tiles * sp < 768 && !(sp == 1 && tiles >= cu_count()))
    return plan_wino_wgrad(T, cin_p, cout_p, nb);
  p.splits = (int)sp;
  p.kchunk = (int)kc;
  p.slab_floats = (size_t)nb * sp * cout_p * cin_p;
  if (sp > 1) p.slab_floats += (size_t)nb * cout_p * cin_p;
  return p;
}

extern "C" size_t nsm_wino_wgrad_h2_ws(int B, int H, int W, int cin_p, int cout_p, int tile) {
  WinoGeom g;
  if (!wino_geom(tile, B, H, W, g)) return 0;
  return plan_wino_wgrad_h2(g.T, cin_p, cout_p, g.alpha2).slab_floats;
}

extern "C" int nsm_conv3x3_wgrad_wino_h2(const void* dMh, const void* Vh, int B, int H, int W,
                                         int cin_p, int cout_p, int cin, int cout, int tile,
                                         float* dw, float* ws, size_t ws_floats,
                                         const uint32_t* amax_dy, const uint32_t* amax_x,
                                         void* stream) {
  NSM_CHECK_ARG(dMh && Vh && dw && ws && amax_dy && amax_x, "conv3x3_wgrad_wino_h2: null pointer");
  NSM_CHECK_ARG(cin_p % 32 == 0 && cout_p % 32 == 0 && cin <= cin_p && cout <= cout_p,
                "conv3x3_wgrad_wino_h2: bad channels");
  NSM_CHECK_ARG(((uintptr_t)dMh % 16) == 0 && ((uintptr_t)Vh % 16) == 0 && ((uintptr_t)ws % 16) == 0,
                "conv3x3_wgrad_wino_h2: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "conv3x3_wgrad_wino_h2: bad tile or shape");
  const int nb = g.alpha2;
  WinoWgradPlan pl = plan_wino_wgrad_h2(g.T, cin_p, cout_p, nb);
  if (ws_floats < pl.slab_floats) return fail(NSM_E_WS, "conv3x3_wgrad_wino_h2: workspace too small");
  NSM_CHECK_ARG(g.T * 2 * (long long)std::max(cin_p, cout_p) < (1ll << 30),
                "conv3x3_wgrad_wino_h2: operand too large");
  hipStream_t s = as_stream(stream);
  const int M = cout_p, N = cin_p;
  const int rc = wino_wgrad_gemm_h2((const bf16_t*)dMh, (const bf16_t*)Vh, g.T, cin_p, cout_p, nb,
                                    pl.BM, pl.BN, pl.kchunk, pl.splits, ws,
                                    H2Scale{amax_dy, wino_beta(tile, 1)},
                                    H2Scale{amax_x, wino_beta(tile, 0)}, s);
  if (rc) return rc;
  return wgrad_wino_finish(ws, pl, nb, M, N, cin, cout, tile, dw, s);
}

extern "C" int nsm_to_h2(const float* x, int64_t rows, int C, const uint32_t* amax, float beta,
                         void* out, void* stream) {
  NSM_CHECK_ARG(x && out && amax && rows > 0 && C > 0 && C % 8 == 0 && beta > 0.f,
                "to_h2: bad args");
  const long long g = std::min<long long>(ceil_div(rows * (C / 4), 256), 8192);
  hipLaunchKernelGGL(to_h2_kernel, dim3((int)g), dim3(256), 0, as_stream(stream), x,
                     (long long)rows, C, H2Scale{amax, beta}, (bf16_t*)out);
  NSM_LAUNCH_CHECK("to_h2");
  return 0;
}

extern "C" int nsm_wino_gemm_h2(const void* V, const void* U, int B, int H, int W, int cin_p,
                                int cout_p, int tile, float* Mb, const uint32_t* amax_v,
                                float beta_v, const uint32_t* amax_u, float beta_u,
                                void* stream) {
  NSM_CHECK_ARG(V && U && Mb && amax_v && amax_u && cin_p % 32 == 0 && cout_p % 32 == 0,
                "wino_gemm_h2: bad args");
  NSM_CHECK_ARG(((uintptr_t)V % 16) == 0 && ((uintptr_t)U % 16) == 0 && ((uintptr_t)Mb % 16) == 0,
                "wino_gemm_h2: 16B alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_gemm_h2: bad tile or shape");
  NSM_CHECK_ARG(g.T * 2 * cin_p < (1ll << 30) && (long long)cout_p * 2 * cin_p < (1ll << 30),
                "wino_gemm_h2: operand too large");
  return wino_gemm_h2((const bf16_t*)V, (const bf16_t*)U, g.T, cin_p, cout_p, g.alpha2, Mb,
                      H2Scale{amax_v, beta_v}, H2Scale{amax_u, beta_u}, as_stream(stream));
}

// ---- bf16 path: Winograd F(4x4) forward on single-plane scaled f16 operands ----
// The bf16 configuration's direct 3x3 implicit GEMM (gemm_bf16_dma_kernel) is
// ~75 % of its step. F(4x4, 3x3) does the same convolution with 4x fewer
// multiplies; its operands V = B^T d B and U = G g G^T are written ONCE as f16
// scaled by a power of two (max|source| x the transform's bound, as the h2
// tensors: no overflow, 11-bit significands), the batched GEMM runs the f16
// MFMA on them (gemm_h2p/h2q_kernel, single-plane mode), M stays fp32 and the
// output transform writes Y in bf16 with the BN partials of the rounded
// values. Rounding: V and U to f16 (2^-11), amplified ~7x by the F(4x4)
// transforms (tools/wino_coeffs.py: F(4x4) / direct rms 7.3 in fp32) — the
// size of the direct path's bf16 operand rounding (2^-9 x 2). Unetmodel.py:21.
typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 bf4_to_f32(u32x2 w) {
  return f32x4{bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)};
}
// Channels per thread of the bf16 path's F(4x4) transforms (BfLane<CW>): the
// 6x6 tile's column-pass accumulators are 36 lane vectors, 144 VGPRs at 4
// channels (1-2 waves / SIMD, the x2-upsample form spilling to AGPRs) and 72
// at 2 (3-4 waves / SIMD). Same per-channel arithmetic either way.
template <int CW> struct BfLane;
template <> struct BfLane<4> {
  using V = f32x4;
  using W = u32x2;  // 4 bf16
  __device__ static W raw(const bf16_t* p) { return *(const W*)p; }
  __device__ static V cvt(W w) { return bf4_to_f32(w); }
  __device__ static V ld(const bf16_t* p) { return cvt(raw(p)); }
  __device__ static V rbf(V v) { return V{round_bf(v.x), round_bf(v.y), round_bf(v.z), round_bf(v.w)}; }
  __device__ static void st16(bf16_t* p, V v) {  // IEEE half
    *(u32x2*)p = __builtin_bit_cast(u32x2, __builtin_convertvector(v, f16x4v));
  }
  __device__ static W pack(V v) { return W{pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)}; }  // bf16
  __device__ static V lrg(V z, float s) { return lrelu_grad_v4(z, s); }
};
template <> struct BfLane<2> {
  using V = f32x2;
  using W = uint32_t;  // 2 bf16
  __device__ static W raw(const bf16_t* p) { return *(const W*)p; }
  __device__ static V cvt(W w) { return V{bf_lo(w), bf_hi(w)}; }
  __device__ static V ld(const bf16_t* p) { return cvt(raw(p)); }
  __device__ static V rbf(V v) { return V{round_bf(v.x), round_bf(v.y)}; }
  __device__ static void st16(bf16_t* p, V v) { *(uint32_t*)p = pack_h2(v); }
  __device__ static W pack(V v) { return pack_bf2(v.x, v.y); }  // bf16
  __device__ static V lrg(V z, float s) { return V{lrelu_grad(z.x, s), lrelu_grad(z.y, s)}; }
};
// NSM_F16_TX_CW: 2 (default) or 4 channels per thread in those transforms
static int f16_tx_cw() {
  static int v = [] {
    const char* e = getenv("NSM_F16_TX_CW");
    return e && atoi(e) == 4 ? 4 : 2;
  }();
  return v;
}
// NSM_F16_OUT_CW: channels per thread of the training step's f16-M output
// transform alone (4, default: M read as 8-B words; 2: as 4-B ones).
// Interleaved A/B (bf16 B=64 kernel traces, two rounds): the step's output
// transforms 2818 / 2818 -> 2397 / 2401 us, bench 1637.8 / 1619.2 -> 1643.7 /
// 1632.7 frames/s — the 8-B reads outweigh the halved occupancy here, unlike
// the input and dual transforms (NSM_F16_TX_CW)
static int f16_out_cw() {
  static int v = [] {
    const char* e = getenv("NSM_F16_OUT_CW");
    return (e && atoi(e) == 2) ? 2 : 4;
  }();
  return v;
}

// V [alpha^2][T][C] f16 = s B^T d B of the bf16 NHWC input x (zero padding), 4
// channels per thread, the column pass streamed over the patch rows
template <int MT, int CW>
__global__ void __launch_bounds__(256) wino_input_f16_kernel(const bf16_t* __restrict__ x, int ld,
                                                             int H, int W, int C, int TH, int TW,
                                                             long long T, bf16_t* __restrict__ V,
                                                             H2Scale hsc) {
  constexpr int A = MT + 2;
  using L = BfLane<CW>;
  using LV = typename L::V;
  const int C4 = C / CW;
  const long long total = T * C4;
  const float hs = exp2i(h2_exp(hsc));  // every lane (amax_read: a wave reduction)
  const size_t plane = (size_t)T * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    const long long t = i / C4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    // the whole patch's loads go out first: unconditional (an element outside
    // the image reads the image's first pixel, then counts as 0)
    typename L::W raw[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int yy = MT * ty - 1 + a, xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        raw[a][e] = L::raw(x + ((size_t)b * H * W + (in ? (size_t)yy * W + xx : 0)) * ld + c);
        if (!in) raw[a][e] = typename L::W{};
      }
    LV sc[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV d[A];
#pragma unroll
      for (int e = 0; e < A; ++e) d[e] = L::cvt(raw[a][e]);
      wcol_row<CBt<MT>>(sc, d, a);
    }
    bf16_t* out = V + (size_t)t * C + c;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CBt<MT>>(sc[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)
        L::st16(out + (a * A + e) * plane, v[e] * hs);
    }
  }
}

// wino_input_f16_kernel of the decoder's x2 upsample of x (bf16 [B][hi][wi][C]
// NHWC, align_corners bilinear, Unetmodel.py:122-130) sampled per patch
// element: each value is interpolated in fp32 as resize_fwd8_kernel does and
// rounded to bf16 (what the materialised upsample would hold), then
// transformed; the upsampled tensor is never written or re-read. Source rows
// are x-interpolated once and kept while consecutive patch rows reuse them
// (a tile's 6 patch rows of a x2 upsample touch ~4 source rows).
template <int MT, int CW>
__global__ void __launch_bounds__(256) wino_input_f16_up_kernel(
    const bf16_t* __restrict__ x, int ld, int hi, int wi, float sh, float sw, int H, int W, int C,
    int TH, int TW, long long T, bf16_t* __restrict__ V, H2Scale hsc) {
  constexpr int A = MT + 2;
  using L = BfLane<CW>;
  using LV = typename L::V;
  const int C4 = C / CW;
  const long long total = T * C4;
  const float hs = exp2i(h2_exp(hsc));  // every lane (amax_read: a wave reduction)
  const size_t plane = (size_t)T * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    const long long t = i / C4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    int x0[A], x1[A];
    float lx0[A], lx1[A];
#pragma unroll
    for (int e = 0; e < A; ++e)
      lin_idx(sw, min(max(MT * tx - 1 + e, 0), W - 1), wi, x0[e], x1[e], lx0[e], lx1[e]);
    LV h0[A], h1[A];
    int ya = -1, yb = -1;  // source rows held in h0, h1
    LV sc[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const int yy = MT * ty - 1 + a;
      int y0, y1;
      float ly0, ly1;
      lin_idx(sh, min(max(yy, 0), H - 1), hi, y0, y1, ly0, ly1);
      if (y0 != ya) {
        if (y0 == yb) {
#pragma unroll
          for (int e = 0; e < A; ++e) h0[e] = h1[e];
        } else {
          const bf16_t* r0 = x + ((size_t)b * hi + y0) * wi * ld + c;
#pragma unroll
          for (int e = 0; e < A; ++e)
            h0[e] = lx0[e] * L::ld(r0 + (size_t)x0[e] * ld) + lx1[e] * L::ld(r0 + (size_t)x1[e] * ld);
        }
        ya = y0;
      }
      if (y1 != yb) {
        if (y1 == ya) {
#pragma unroll
          for (int e = 0; e < A; ++e) h1[e] = h0[e];
        } else {
          const bf16_t* r1 = x + ((size_t)b * hi + y1) * wi * ld + c;
#pragma unroll
          for (int e = 0; e < A; ++e)
            h1[e] = lx0[e] * L::ld(r1 + (size_t)x0[e] * ld) + lx1[e] * L::ld(r1 + (size_t)x1[e] * ld);
        }
        yb = y1;
      }
      const bool rin = (unsigned)yy < (unsigned)H;
      LV d[A];
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const bool in = rin && (unsigned)(MT * tx - 1 + e) < (unsigned)W;
        const LV v = ly0 * h0[e] + ly1 * h1[e];
        d[e] = in ? L::rbf(v) : LV{};
      }
      wcol_row<CBt<MT>>(sc, d, a);
    }
    bf16_t* out = V + (size_t)t * C + c;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CBt<MT>>(sc[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)
        L::st16(out + (a * A + e) * plane, v[e] * hs);
    }
  }
}

// wino_input_f16_up_kernel at 2 channels per thread on 32-bit buffer offsets
// (host-checked: x under 2 GiB, all of V under 4 GiB, T x C / 2 under 2^31):
// the source taps' column offsets are formed once per tile, a source row adds
// one offset, and V is stored through one descriptor, the plane in the scalar
// offset and the thread's in-plane offset in the vector one — the 64-bit
// address arithmetic of ~150 global loads and 36 stores per tile (the kernel
// is VALU-bound: 78 % VALU-busy SIMDs at B=64) is gone. Same values, bits and
// order as the generic kernel.
template <int MT>
__global__ void __launch_bounds__(256) wino_input_f16_up_buf_kernel(
    const bf16_t* __restrict__ x, int ld, int hi, int wi, float sh, float sw, int H, int W, int C,
    int TH, int TW, int T, bf16_t* __restrict__ V, H2Scale hsc) {
  constexpr int A = MT + 2;
  using L = BfLane<2>;
  using LV = L::V;
  const int C4 = C / 2;
  const int total = T * C4;
  const float hs = exp2i(h2_exp(hsc));  // every lane (amax_read: a wave reduction)
  const int nb = T / (TH * TW);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc_b(x, (long long)nb * hi * wi * ld);
  // all of V through one descriptor (4 GiB range: host-checked under it), the
  // plane in the scalar offset
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, -1, 0x00020000);
  const uint32_t pbytes = (uint32_t)T * (uint32_t)C * 2u;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = (i % C4) * 2;
    const int t = i / C4;
    const int tx = t % TW;
    const int r = t / TW;
    const int ty = r % TH;
    const int b = r / TH;
    uint32_t o0[A], o1[A];  // byte offsets of the taps' source columns (+ channel)
    float lx0[A], lx1[A];
#pragma unroll
    for (int e = 0; e < A; ++e) {
      int x0, x1;
      lin_idx(sw, min(max(MT * tx - 1 + e, 0), W - 1), wi, x0, x1, lx0[e], lx1[e]);
      o0[e] = (uint32_t)(x0 * ld + c) * 2u;
      o1[e] = (uint32_t)(x1 * ld + c) * 2u;
    }
    auto src_row = [&](int y, LV(&h)[A]) {
      const uint32_t ro = (uint32_t)((b * hi + y) * wi) * (uint32_t)ld * 2u;
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(xr, ro + o0[e], 0, 0);
        const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(xr, ro + o1[e], 0, 0);
        h[e] = lx0[e] * L::cvt(w0) + lx1[e] * L::cvt(w1);
      }
    };
    LV h0[A], h1[A];
    int ya = -1, yb = -1;  // source rows held in h0, h1
    LV sc[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const int yy = MT * ty - 1 + a;
      int y0, y1;
      float ly0, ly1;
      lin_idx(sh, min(max(yy, 0), H - 1), hi, y0, y1, ly0, ly1);
      if (y0 != ya) {
        if (y0 == yb) {
#pragma unroll
          for (int e = 0; e < A; ++e) h0[e] = h1[e];
        } else {
          src_row(y0, h0);
        }
        ya = y0;
      }
      if (y1 != yb) {
        if (y1 == ya) {
#pragma unroll
          for (int e = 0; e < A; ++e) h1[e] = h0[e];
        } else {
          src_row(y1, h1);
        }
        yb = y1;
      }
      const bool rin = (unsigned)yy < (unsigned)H;
      LV d[A];
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const bool in = rin && (unsigned)(MT * tx - 1 + e) < (unsigned)W;
        const LV v = ly0 * h0[e] + ly1 * h1[e];
        d[e] = in ? L::rbf(v) : LV{};
      }
      wcol_row<CBt<MT>>(sc, d, a);
    }
    const uint32_t vo = (uint32_t)(t * C + c) * 2u;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CBt<MT>>(sc[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)  // plane a A + e at the (uniform) scalar offset
        __builtin_amdgcn_raw_buffer_store_b32(pack_h2(v[e] * hs), vr, vo,
                                              (int)((uint32_t)(a * A + e) * pbytes), 0);
    }
  }
}

// NSM_F16_UP_BUF=0: the generic kernels for the bf16 x2-upsample input
// transform and the lazy dual transform (their buffer-offset forms otherwise)
static bool f16_up_buf() {
  static bool v = [] {
    const char* e = getenv("NSM_F16_UP_BUF");
    return !e || atoi(e) != 0;
  }();
  return v;
}

extern "C" int nsm_wino_input_f16_resize(const void* x, int ldx, int B, int hi, int wi, int H, int W,
                                         int cin_p, int tile, void* V, const uint32_t* amax_x,
                                         void* stream) {
  NSM_CHECK_ARG(x && V && amax_x && tile == 4 && cin_p % 32 == 0 && ldx % 4 == 0 && ldx >= cin_p &&
                    hi > 0 && wi > 0,
                "wino_input_f16_resize: bad args (tile 4 only)");
  NSM_CHECK_ARG(((uintptr_t)x % 8) == 0 && ((uintptr_t)V % 16) == 0, "wino_input_f16_resize: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_input_f16_resize: bad shape");
  const int cw = f16_tx_cw();
  const long long xbytes = (long long)B * hi * wi * ldx * 2, vbytes = 36ll * g.T * cin_p * 2;
  if (cw == 2 && f16_up_buf() && xbytes < 0x7FFFFFFFll && vbytes < 0xFFFFFFFFll &&
      g.T * (cin_p / 2) < (1ll << 31)) {
    hipLaunchKernelGGL(wino_input_f16_up_buf_kernel<4>, dim3(grid_1d(g.T * cin_p / 2)), dim3(256), 0,
                       as_stream(stream), (const bf16_t*)x, ldx, hi, wi, ac_scale(hi, H), ac_scale(wi, W),
                       H, W, cin_p, g.TH, g.TW, (int)g.T, (bf16_t*)V, H2Scale{amax_x, wino_beta(4, 0)});
    NSM_LAUNCH_CHECK("wino_input_f16_resize");
    return 0;
  }
  hipLaunchKernelGGL((cw == 2 ? wino_input_f16_up_kernel<4, 2> : wino_input_f16_up_kernel<4, 4>),
                     dim3(grid_1d(g.T * cin_p / cw)), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)x, ldx, hi, wi, ac_scale(hi, H), ac_scale(wi, W), H, W, cin_p,
                     g.TH, g.TW, g.T, (bf16_t*)V, H2Scale{amax_x, wino_beta(4, 0)});
  NSM_LAUNCH_CHECK("wino_input_f16_resize");
  return 0;
}

extern "C" int nsm_wino_input_f16(const void* x, int ldx, int B, int H, int W, int cin_p, int tile,
                                  void* V, const uint32_t* amax_x, void* stream) {
  NSM_CHECK_ARG(x && V && amax_x && tile == 4 && cin_p % 32 == 0 && ldx % 4 == 0 && ldx >= cin_p,
                "wino_input_f16: bad args (tile 4 only)");
  NSM_CHECK_ARG(((uintptr_t)x % 8) == 0 && ((uintptr_t)V % 16) == 0, "wino_input_f16: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_input_f16: bad shape");
  const int cw = f16_tx_cw();
  hipLaunchKernelGGL((cw == 2 ? wino_input_f16_kernel<4, 2> : wino_input_f16_kernel<4, 4>),
                     dim3(grid_1d(g.T * cin_p / cw)), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)x, ldx, H, W, cin_p, g.TH, g.TW, g.T, (bf16_t*)V,
                     H2Scale{amax_x, wino_beta(4, 0)});
  NSM_LAUNCH_CHECK("wino_input_f16");
  return 0;
}

extern "C" int nsm_wino_gemm_f16(const void* V, const void* U, int B, int H, int W, int cin_p,
                                 int cout_p, int tile, float* Mb, const uint32_t* amax_v,
                                 float beta_v, const uint32_t* amax_u, float beta_u, void* stream) {
  NSM_CHECK_ARG(V && U && Mb && amax_v && amax_u && cin_p % 128 == 0 && cout_p % 128 == 0,
                "wino_gemm_f16: bad args (cin_p, cout_p multiples of 128)");
  NSM_CHECK_ARG(((uintptr_t)V % 16) == 0 && ((uintptr_t)U % 16) == 0 && ((uintptr_t)Mb % 16) == 0,
                "wino_gemm_f16: 16B alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_gemm_f16: bad tile or shape");
  NSM_CHECK_ARG(g.T * cin_p < (1ll << 30) && (long long)cout_p * cin_p < (1ll << 30),
                "wino_gemm_f16: operand too large");
  return wino_gemm_f16((const bf16_t*)V, (const bf16_t*)U, g.T, cin_p, cout_p, g.alpha2, Mb,
                       H2Scale{amax_v, beta_v}, H2Scale{amax_u, beta_u}, as_stream(stream));
}

// the same GEMM writing M as f16 (O16: scale 2^-(15 + ceil log2 cin_p) in the
// operands' scaled units; M16 [alpha^2][T][cout_p] f16, half of Mb's bytes)
extern "C" int nsm_wino_gemm_f16m(const void* V, const void* U, int B, int H, int W, int cin_p,
                                  int cout_p, int tile, void* M16, int* m16e, const uint32_t* amax_v,
                                  float beta_v, const uint32_t* amax_u, float beta_u, void* stream) {
  NSM_CHECK_ARG(V && U && M16 && m16e && amax_v && amax_u && cin_p % 128 == 0 && cout_p % 128 == 0,
                "wino_gemm_f16m: bad args (cin_p, cout_p multiples of 128)");
  NSM_CHECK_ARG(((uintptr_t)V % 16) == 0 && ((uintptr_t)U % 16) == 0 && ((uintptr_t)M16 % 16) == 0,
                "wino_gemm_f16m: 16B alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_gemm_f16m: bad tile or shape");
  NSM_CHECK_ARG(g.T * cin_p < (1ll << 30) && g.T * cout_p < (1ll << 30) &&
                    (long long)cout_p * cin_p < (1ll << 30),
                "wino_gemm_f16m: operand too large");
  return wino_gemm_f16((const bf16_t*)V, (const bf16_t*)U, g.T, cin_p, cout_p, g.alpha2, (float*)M16,
                       H2Scale{amax_v, beta_v}, H2Scale{amax_u, beta_u}, as_stream(stream), true, m16e);
}

// the output transform of nsm_wino_gemm_f16m's f16 M (same scale slots / bounds
// as the GEMM call, cin_p its K) writing bf16 Y (+ the BN partials)
// wino_output_kernel<4, STATS, false, true, true, 4> (the training step's
// f16-M output transform) on 32-bit buffer offsets (host-checked: M under
// 4 GiB, y under 2 GiB, T x N / 4 under 2^31): M's plane in the scalar offset
// of one descriptor, y's pixel rows through another. Same arithmetic and
// order, so the same bits and BN partials.
template <bool STATS>
__global__ void __launch_bounds__(256) wino_output_f16m_buf_kernel(
    const bf16_t* __restrict__ M, int N, int H, int W, int TH, int TW, int T,
    const float* __restrict__ bias, bf16_t* __restrict__ y, int ldy, float* __restrict__ partial,
    WinoM16 m16) {
  constexpr int MT = 4, A = 6, CW = 4;
  using VT = f32x4;
  const int ev = h2_exp(m16.sv), eu = h2_exp(m16.su);
  const int N4 = N / CW;
  const int total = T * N4;
  const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = T / (TH * TW);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)M, (short)0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc_b(y, (long long)nb * H * W * ldy);
  const uint32_t pbytes = (uint32_t)T * (uint32_t)N * 2u;
  const float ieu = exp2i(-eu);
  VT s_sum{}, s_mean{}, s_m2{};
  float s_n = 0.f;
  for (int i = i0; i < total; i += gridDim.x * blockDim.x) {
    const int c = (i % N4) * CW;
    const int t = i / N4;
    const int tx = t % TW;
    const int r = t / TW;
    const int ty = r % TH;
    const int b = r / TH;
    const uint32_t mo = (uint32_t)(t * N + c) * 2u;
    const int* et0 = m16.e + (t / 64) * (N / 64) + c / 64;
    const int estep = m16.rows * (N / 64);
    VT sc[MT][A], o[MT][MT];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      VT row[A];
#pragma unroll
      for (int e = 0; e < A; ++e) {
        int x = -et0[(a * A + e) * estep] - ev;
        x = x < -126 ? -126 : (x > 126 ? 126 : x);
        const u32x2 h = __builtin_bit_cast(
            u32x2, __builtin_amdgcn_raw_buffer_load_b64(mr, mo, (int)((uint32_t)(a * A + e) * pbytes), 0));
        const f32x2 lo = unpack_h2(h.x), hi = unpack_h2(h.y);
        row[e] = VT{lo.x, lo.y, hi.x, hi.y} * (exp2i(x) * ieu);
      }
      wcol_row<CAt<MT>>(sc, row, a);
    }
#pragma unroll
    for (int a = 0; a < MT; ++a) wmat<CAt<MT>>(sc[a], o[a]);
    const VT bv = bias ? *(const VT*)(bias + c) : VT{};
    VT ts{};
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      const int yy = MT * ty + a;
      if (yy >= H) continue;
      const uint32_t ro = (uint32_t)(((b * H + yy) * W + MT * tx) * ldy + c) * 2u;
#pragma unroll
      for (int e = 0; e < MT; ++e)
        if (MT * tx + e < W) {
          o[a][e] = o[a][e] + bv;
          const VT q = o[a][e];
          o[a][e] = VT{round_bf(q.x), round_bf(q.y), round_bf(q.z), round_bf(q.w)};
          const u32x2 w = u32x2{pack_bf2(o[a][e].x, o[a][e].y), pack_bf2(o[a][e].z, o[a][e].w)};
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(mr, 0u, 0, 0)), w),
                                                yr, ro + (uint32_t)(e * ldy) * 2u, 0, 0);
          if (STATS) ts = ts + o[a][e];
        }
    }
    if (STATS) {
      const int nv = min(MT, H - MT * ty) * min(MT, W - MT * tx);
      const VT tmean = ts * (1.f / (float)nv);
      VT tq{};
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int e = 0; e < MT; ++e)
          if (MT * ty + a < H && MT * tx + e < W) {
            const VT d = o[a][e] - tmean;
            tq = tq + d * d;
          }
      const float n2 = s_n + (float)nv;
      const VT delta = tmean - s_mean;
      s_mean = s_mean + delta * ((float)nv / n2);
      s_m2 = s_m2 + tq + delta * delta * (s_n * (float)nv / n2);
      s_sum = s_sum + ts;
      s_n = n2;
    }
  }
  if (STATS && i0 < (int)(gridDim.x * blockDim.x)) {
    const int c = (i0 % N4) * CW;
    float* pr = partial + (size_t)(i0 / N4) * 3 * N + c;
    *(VT*)pr = s_sum;
    *(VT*)(pr + N) = s_m2;
    *(VT*)(pr + 2 * N) = VT{} + s_n;
  }
}

extern "C" int nsm_wino_output_bf16m(const void* M16, const int* m16e, int B, int H, int W, int cin_p,
                                     int cout_p, int tile, const uint32_t* amax_v, float beta_v,
                                     const uint32_t* amax_u, float beta_u, const float* bias,
                                     void* y, int ldy, float* partial, int nslot, void* stream) {
  NSM_CHECK_ARG(M16 && m16e && y && amax_v && amax_u && tile == 4 && cin_p > 0 && cout_p % 64 == 0 &&
                    ldy % 4 == 0,
                "wino_output_bf16m: bad args (tile 4 only)");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_output_bf16m: bad shape");
  // (the partial slots: nslot x N channels whatever the width; the grid's
  // threads, nslot x N / cw, each keep one channel group)
  const int cw = f16_out_cw();
  dim3 grid(grid_1d(g.T * (cout_p / cw)));
  if (partial) {
    NSM_CHECK_ARG(nslot > 0 && nslot % wino_stat_step(cout_p, tile) == 0 && nslot <= (1 << 20),
                  "wino_output_bf16m: nslot %d not a multiple of %d", nslot,
                  wino_stat_step(cout_p, tile));
    grid = dim3((unsigned)((long long)nslot * (cout_p / cw) / 256));
  }
  const WinoM16 m16{H2Scale{amax_v, beta_v}, H2Scale{amax_u, beta_u}, m16e, (int)((g.T + 63) / 64)};
  hipStream_t s = as_stream(stream);
  const long long mbytes = 36ll * g.T * cout_p * 2, ybytes = (long long)B * H * W * ldy * 2;
  if (cw == 4 && f16_up_buf() && mbytes < 0xFFFFFFFFll && ybytes < 0x7FFFFFFFll &&
      g.T * (cout_p / 4) < (1ll << 31)) {
    if (partial)
      hipLaunchKernelGGL(wino_output_f16m_buf_kernel<true>, grid, dim3(256), 0, s, (const bf16_t*)M16,
                         cout_p, H, W, g.TH, g.TW, (int)g.T, bias, (bf16_t*)y, ldy, partial, m16);
    else
      hipLaunchKernelGGL(wino_output_f16m_buf_kernel<false>, grid, dim3(256), 0, s, (const bf16_t*)M16,
                         cout_p, H, W, g.TH, g.TW, (int)g.T, bias, (bf16_t*)y, ldy, nullptr, m16);
    NSM_LAUNCH_CHECK("wino_output_bf16m");
    return 0;
  }
#define NSM_OUT16(STATS_, CW_)                                                                      \
  hipLaunchKernelGGL((wino_output_kernel<4, STATS_, false, true, true, CW_>), grid, dim3(256), 0, s, \
                     (const float*)M16, cout_p, H, W, g.TH, g.TW, g.T, bias, (float*)y, ldy,        \
                     STATS_ ? partial : nullptr, WinoAct{}, m16)
  if (partial) {
    if (cw == 2) NSM_OUT16(true, 2);
    else NSM_OUT16(true, 4);
  } else {
    if (cw == 2) NSM_OUT16(false, 2);
    else NSM_OUT16(false, 4);
  }
#undef NSM_OUT16
  NSM_LAUNCH_CHECK("wino_output_bf16m");
  return 0;
}

// eval: the output transform of nsm_wino_gemm_f16m's f16 M writing
// lrelu(BN(y)) in bf16, BN from the running statistics (act_scale, act_shift:
// nsm_bn_eval's folded vectors) — the bf16 eval forward's first BatchNorm +
// LeakyReLU of a DoubleConv (Unetmodel.py:21-23) in the 3x3 conv's epilogue
extern "C" int nsm_wino_output_bf16m_act(const void* M16, const int* m16e, int B, int H, int W,
                                         int cin_p, int cout_p, int tile, const uint32_t* amax_v,
                                         float beta_v, const uint32_t* amax_u, float beta_u,
                                         const float* bias, void* y, int ldy, const float* act_scale,
                                         const float* act_shift, float slope, void* stream) {
  NSM_CHECK_ARG(M16 && m16e && y && amax_v && amax_u && act_scale && act_shift && tile == 4 &&
                    cin_p > 0 && cout_p % 64 == 0 && ldy % 4 == 0 && ldy >= cout_p,
                "wino_output_bf16m_act: bad args (tile 4 only)");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_output_bf16m_act: bad shape");
  const WinoM16 m16{H2Scale{amax_v, beta_v}, H2Scale{amax_u, beta_u}, m16e, (int)((g.T + 63) / 64)};
  const WinoAct act{act_scale, act_shift, slope, nullptr, 0};
  const int cw = f16_tx_cw();
  if (cw == 2)
    hipLaunchKernelGGL((wino_output_kernel<4, false, true, true, true, 2>),
                       dim3(grid_1d(g.T * (cout_p / 2))), dim3(256), 0, as_stream(stream),
                       (const float*)M16, cout_p, H, W, g.TH, g.TW, g.T, bias, (float*)y, ldy, nullptr,
                       act, m16);
  else
    hipLaunchKernelGGL((wino_output_kernel<4, false, true, true, true, 4>),
                       dim3(grid_1d(g.T * (cout_p / 4))), dim3(256), 0, as_stream(stream),
                       (const float*)M16, cout_p, H, W, g.TH, g.TW, g.T, bias, (float*)y, ldy, nullptr,
                       act, m16);
  NSM_LAUNCH_CHECK("wino_output_bf16m_act");
  return 0;
}

// the output transform writing bf16 Y (+ the BN partials of the rounded values)
extern "C" int nsm_wino_output_bf16(const float* Mb, int B, int H, int W, int cout_p, int tile,
                                    const float* bias, void* y, int ldy, float* partial, int nslot,
                                    void* stream) {
  NSM_CHECK_ARG(Mb && y && tile == 4 && cout_p % 32 == 0 && ldy % 4 == 0,
                "wino_output_bf16: bad args (tile 4 only)");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_output_bf16: bad shape");
  dim3 grid(grid_1d(g.T * (cout_p / 4)));
  if (partial) {
    NSM_CHECK_ARG(nslot > 0 && nslot % wino_stat_step(cout_p, tile) == 0 && nslot <= (1 << 20),
                  "wino_output_bf16: nslot %d not a multiple of %d", nslot,
                  wino_stat_step(cout_p, tile));
    grid = dim3((unsigned)((long long)nslot * (cout_p / 4) / 256));
  }
  hipStream_t s = as_stream(stream);
  if (partial)
    hipLaunchKernelGGL((wino_output_kernel<4, true, false, true>), grid, dim3(256), 0, s, Mb, cout_p,
                       H, W, g.TH, g.TW, g.T, bias, (float*)y, ldy, partial, WinoAct{});
  else
    hipLaunchKernelGGL((wino_output_kernel<4, false, false, true>), grid, dim3(256), 0, s, Mb,
                       cout_p, H, W, g.TH, g.TW, g.T, bias, (float*)y, ldy, nullptr, WinoAct{});
  NSM_LAUNCH_CHECK("wino_output_bf16");
  return 0;
}

// dM [alpha^2][T][C] f16 = s (A dY A^T) of the bf16 output gradient (the
// weight gradient's transform of dY, as wino_dout_kernel), 4 channels per
// thread, the interior's loads first, the column pass streamed
template <int MT, int CW>
__global__ void __launch_bounds__(256) wino_dout_f16_kernel(const bf16_t* __restrict__ dy, int ld,
                                                            int H, int W, int C, int TH, int TW,
                                                            long long T, bf16_t* __restrict__ dM,
                                                            H2Scale hsc) {
  constexpr int A = MT + 2;
  using L = BfLane<CW>;
  using LV = typename L::V;
  const int C4 = C / CW;
  const long long total = T * C4;
  const float hs = exp2i(h2_exp(hsc));  // every lane (amax_read: a wave reduction)
  const size_t plane = (size_t)T * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    const long long t = i / C4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    typename L::W raw[MT][MT];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int e = 0; e < MT; ++e) {
        const int yy = MT * ty + a, xx = MT * tx + e;
        const bool in = yy < H && xx < W;
        raw[a][e] = L::raw(dy + ((size_t)b * H * W + (in ? (size_t)yy * W + xx : 0)) * ld + c);
        if (!in) raw[a][e] = typename L::W{};
      }
    LV sc[A][MT];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      LV d[MT];
#pragma unroll
      for (int e = 0; e < MT; ++e) d[e] = L::cvt(raw[a][e]);
      wcol_row<CA<MT>>(sc, d, a);
    }
    bf16_t* out = dM + (size_t)t * C + c;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CA<MT>>(sc[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)
        L::st16(out + (a * A + e) * plane, v[e] * hs);
    }
  }
}

extern "C" int nsm_wino_dout_f16(const void* dy, int lddy, int B, int H, int W, int c_p, int tile,
                                 void* dM, const uint32_t* amax_dy, void* stream) {
  NSM_CHECK_ARG(dy && dM && amax_dy && tile == 4 && c_p % 32 == 0 && lddy % 4 == 0 && lddy >= c_p,
                "wino_dout_f16: bad args (tile 4 only)");
  NSM_CHECK_ARG(((uintptr_t)dy % 8) == 0 && ((uintptr_t)dM % 16) == 0, "wino_dout_f16: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_dout_f16: bad shape");
  const int cw = f16_tx_cw();
  hipLaunchKernelGGL((cw == 2 ? wino_dout_f16_kernel<4, 2> : wino_dout_f16_kernel<4, 4>),
                     dim3(grid_1d(g.T * c_p / cw)), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)dy, lddy, H, W, c_p, g.TH, g.TW, g.T, (bf16_t*)dM,
                     H2Scale{amax_dy, wino_beta(4, 1)});
  NSM_LAUNCH_CHECK("wino_dout_f16");
  return 0;
}

// both F(4x4) transforms of the bf16 output gradient dY from one read of its
// patches (the fp32 path's wino_dual_kernel): V [alpha^2][T][C] f16 = s_v B^T
// d B of the 6x6 patch (the input gradient's operand, zero padding) and dM =
// s_d A dY A^T of its 4x4 interior (the weight gradient's), both scales from
// max|dY| (betas 0 and 1). wino_input_f16 + wino_dout_f16 read dY twice.
template <int MT, int CW>
__global__ void __launch_bounds__(256) wino_dual_f16_kernel(const bf16_t* __restrict__ dy, int ld,
                                                            int H, int W, int C, int TH, int TW,
                                                            long long T, bf16_t* __restrict__ V,
                                                            bf16_t* __restrict__ dM, H2Scale hv,
                                                            H2Scale hd) {
  constexpr int A = MT + 2;
  using L = BfLane<CW>;
  using LV = typename L::V;
  const int C4 = C / CW;
  const long long total = T * C4;
  // every lane (amax_read: a wave reduction)
  const float sv = exp2i(h2_exp(hv)), sd = exp2i(h2_exp(hd));
  const size_t plane = (size_t)T * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    const long long t = i / C4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    typename L::W raw[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int yy = MT * ty - 1 + a, xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        raw[a][e] = L::raw(dy + ((size_t)b * H * W + (in ? (size_t)yy * W + xx : 0)) * ld + c);
        if (!in) raw[a][e] = typename L::W{};
      }
    {
      LV sc[A][A];
#pragma unroll
      for (int a = 0; a < A; ++a) {
        LV d[A];
#pragma unroll
        for (int e = 0; e < A; ++e) d[e] = L::cvt(raw[a][e]);
        wcol_row<CBt<MT>>(sc, d, a);
      }
      bf16_t* out = V + (size_t)t * C + c;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        LV v[A];
        wmat<CBt<MT>>(sc[a], v);
#pragma unroll
        for (int e = 0; e < A; ++e)
          L::st16(out + (a * A + e) * plane, v[e] * sv);
      }
    }
    LV sc[A][MT];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      LV d[MT];
#pragma unroll
      for (int e = 0; e < MT; ++e) d[e] = L::cvt(raw[a + 1][e + 1]);
      wcol_row<CA<MT>>(sc, d, a);
    }
    bf16_t* out = dM + (size_t)t * C + c;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CA<MT>>(sc[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)
        L::st16(out + (a * A + e) * plane, v[e] * sd);
    }
  }
}

extern "C" int nsm_wino_dual_f16(const void* dy, int lddy, int B, int H, int W, int c_p, int tile,
                                 void* V, void* dM, const uint32_t* amax_dy, void* stream) {
  NSM_CHECK_ARG(dy && V && dM && amax_dy && tile == 4 && c_p % 32 == 0 && lddy % 4 == 0 &&
                    lddy >= c_p,
                "wino_dual_f16: bad args (tile 4 only)");
  NSM_CHECK_ARG(((uintptr_t)dy % 8) == 0 && ((uintptr_t)V % 16) == 0 && ((uintptr_t)dM % 16) == 0,
                "wino_dual_f16: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "wino_dual_f16: bad shape");
  const int cw = f16_tx_cw();
  hipLaunchKernelGGL((cw == 2 ? wino_dual_f16_kernel<4, 2> : wino_dual_f16_kernel<4, 4>),
                     dim3(grid_1d(g.T * c_p / cw)), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)dy, lddy, H, W, c_p, g.TH, g.TW, g.T, (bf16_t*)V, (bf16_t*)dM,
                     H2Scale{amax_dy, wino_beta(4, 0)}, H2Scale{amax_dy, wino_beta(4, 1)});
  NSM_LAUNCH_CHECK("wino_dual_f16");
  return 0;
}

// wino_dual_f16_kernel of a dY formed per element from the BN backward's
// deferred form (nsm_wino_dual_bn_f16): each patch element's dY = k1 dz + k2
// (y - mean) + k3 is rounded to bf16 exactly where nsm_bn_bwd_apply would
// store it, then transformed as a loaded dY is
template <int MT, int CW>
__global__ void __launch_bounds__(256) wino_dual_bn_f16_kernel(
    const bf16_t* __restrict__ g, int ldg, const bf16_t* __restrict__ y, int ldy, int H, int W, int C,
    int TH, int TW, long long T, const float* __restrict__ scale, const float* __restrict__ shift,
    float slope, const float* __restrict__ mask, const float* __restrict__ mean,
    const float* __restrict__ coef, bf16_t* __restrict__ V, bf16_t* __restrict__ dM, H2Scale hv,
    H2Scale hd) {
  constexpr int A = MT + 2;
  using L = BfLane<CW>;
  using LV = typename L::V;
  const int C4 = C / CW;
  const long long total = T * C4;
  const float sv = exp2i(h2_exp(hv)), sd = exp2i(h2_exp(hd));  // every lane
  const size_t plane = (size_t)T * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * CW;
    const long long t = i / C4;
    const int tx = (int)(t % TW);
    const long long r = t / TW;
    const int ty = (int)(r % TH);
    const long long b = r / TH;
    typename L::W raw[A][A], yr[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int yy = MT * ty - 1 + a, xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const size_t p = (size_t)b * H * W + (in ? (size_t)yy * W + xx : 0);
        raw[a][e] = L::raw(g + p * ldg + c);
        yr[a][e] = L::raw(y + p * ldy + c);
      }
    const LV sc = *(const LV*)(scale + c), sh = *(const LV*)(shift + c);
    const LV mu = *(const LV*)(mean + c);
    const LV k1 = *(const LV*)(coef + c), k2 = *(const LV*)(coef + C + c),
                k3 = *(const LV*)(coef + 2 * C + c);
    const LV mk = mask ? *(const LV*)(mask + (size_t)b * C + c) : LV{} + 1.f;
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int yy = MT * ty - 1 + a, xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const LV v = L::cvt(yr[a][e]);
        LV dz = L::cvt(raw[a][e]) * L::lrg(v * sc + sh, slope);
        if (mask) dz = dz * mk;
        const LV d = k1 * dz + k2 * (v - mu) + k3;
        raw[a][e] = in ? L::pack(d) : typename L::W{};
      }
    {
      LV scv[A][A];
#pragma unroll
      for (int a = 0; a < A; ++a) {
        LV d[A];
#pragma unroll
        for (int e = 0; e < A; ++e) d[e] = L::cvt(raw[a][e]);
        wcol_row<CBt<MT>>(scv, d, a);
      }
      bf16_t* out = V + (size_t)t * C + c;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        LV v[A];
        wmat<CBt<MT>>(scv[a], v);
#pragma unroll
        for (int e = 0; e < A; ++e)
          L::st16(out + (a * A + e) * plane, v[e] * sv);
      }
    }
    LV scm[A][MT];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      LV d[MT];
#pragma unroll
      for (int e = 0; e < MT; ++e) d[e] = L::cvt(raw[a + 1][e + 1]);
      wcol_row<CA<MT>>(scm, d, a);
    }
    bf16_t* out = dM + (size_t)t * C + c;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CA<MT>>(scm[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)
        L::st16(out + (a * A + e) * plane, v[e] * sd);
    }
  }
}

// wino_dual_bn_f16_kernel at 2 channels per thread on 32-bit buffer offsets
// (host-checked: g and y under 2 GiB, V and dM under 4 GiB, T x C / 2 under
// 2^31): the patch's 72 loads add a per-pixel offset to one descriptor each,
// the 72 stores put the plane in the scalar offset of one descriptor per
// output (as wino_input_f16_up_buf_kernel). Same values and bits as the
// generic kernel.
template <int MT>
__global__ void __launch_bounds__(256) wino_dual_bn_f16_buf_kernel(
    const bf16_t* __restrict__ g, int ldg, const bf16_t* __restrict__ y, int ldy, int H, int W, int C,
    int TH, int TW, int T, const float* __restrict__ scale, const float* __restrict__ shift,
    float slope, const float* __restrict__ mask, const float* __restrict__ mean,
    const float* __restrict__ coef, bf16_t* __restrict__ V, bf16_t* __restrict__ dM, H2Scale hv,
    H2Scale hd) {
  constexpr int A = MT + 2;
  using L = BfLane<2>;
  using LV = L::V;
  const int C4 = C / 2;
  const int total = T * C4;
  const float sv = exp2i(h2_exp(hv)), sd = exp2i(h2_exp(hd));  // every lane
  const int nb = T / (TH * TW);
  const __amdgpu_buffer_rsrc_t gr = make_rsrc_b(g, (long long)nb * H * W * ldg);
  const __amdgpu_buffer_rsrc_t yr_ = make_rsrc_b(y, (long long)nb * H * W * ldy);
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc((void*)V, (short)0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t mr = __builtin_amdgcn_make_buffer_rsrc((void*)dM, (short)0, -1, 0x00020000);
  const uint32_t pbytes = (uint32_t)T * (uint32_t)C * 2u;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = (i % C4) * 2;
    const int t = i / C4;
    const int tx = t % TW;
    const int r = t / TW;
    const int ty = r % TH;
    const int b = r / TH;
    uint32_t raw[A][A], yv[A][A];
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int yy = MT * ty - 1 + a, xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const uint32_t p = (uint32_t)(b * H * W + (in ? yy * W + xx : 0));
        raw[a][e] = __builtin_amdgcn_raw_buffer_load_b32(gr, (p * (uint32_t)ldg + c) * 2u, 0, 0);
        yv[a][e] = __builtin_amdgcn_raw_buffer_load_b32(yr_, (p * (uint32_t)ldy + c) * 2u, 0, 0);
      }
    const LV sc = *(const LV*)(scale + c), sh = *(const LV*)(shift + c);
    const LV mu = *(const LV*)(mean + c);
    const LV k1 = *(const LV*)(coef + c), k2 = *(const LV*)(coef + C + c),
             k3 = *(const LV*)(coef + 2 * C + c);
    const LV mk = mask ? *(const LV*)(mask + (size_t)b * C + c) : LV{} + 1.f;
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int e = 0; e < A; ++e) {
        const int yy = MT * ty - 1 + a, xx = MT * tx - 1 + e;
        const bool in = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const LV v = L::cvt(yv[a][e]);
        LV dz = L::cvt(raw[a][e]) * L::lrg(v * sc + sh, slope);
        if (mask) dz = dz * mk;
        const LV d = k1 * dz + k2 * (v - mu) + k3;
        raw[a][e] = in ? L::pack(d) : 0u;
      }
    const uint32_t vo = (uint32_t)(t * C + c) * 2u;
    {
      LV scv[A][A];
#pragma unroll
      for (int a = 0; a < A; ++a) {
        LV d[A];
#pragma unroll
        for (int e = 0; e < A; ++e) d[e] = L::cvt(raw[a][e]);
        wcol_row<CBt<MT>>(scv, d, a);
      }
#pragma unroll
      for (int a = 0; a < A; ++a) {
        LV v[A];
        wmat<CBt<MT>>(scv[a], v);
#pragma unroll
        for (int e = 0; e < A; ++e)
          __builtin_amdgcn_raw_buffer_store_b32(pack_h2(v[e] * sv), vr, vo,
                                                (int)((uint32_t)(a * A + e) * pbytes), 0);
      }
    }
    LV scm[A][MT];
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      LV d[MT];
#pragma unroll
      for (int e = 0; e < MT; ++e) d[e] = L::cvt(raw[a + 1][e + 1]);
      wcol_row<CA<MT>>(scm, d, a);
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
      LV v[A];
      wmat<CA<MT>>(scm[a], v);
#pragma unroll
      for (int e = 0; e < A; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(pack_h2(v[e] * sd), mr, vo,
                                              (int)((uint32_t)(a * A + e) * pbytes), 0);
    }
  }
}

extern "C" int nsm_wino_dual_bn_f16(const void* g, int ldg, const void* y, int ldy, int B, int H, int W,
                                    int c_p, int tile, const float* scale, const float* shift,
                                    float slope, const float* mask, const float* mean,
                                    const float* coef, void* V, void* dM, const uint32_t* bound,
                                    void* stream) {
  NSM_CHECK_ARG(g && y && V && dM && scale && shift && mean && coef && bound && tile == 4 &&
                    c_p % 32 == 0 && ldg % 4 == 0 && ldg >= c_p && ldy % 4 == 0 && ldy >= c_p,
                "wino_dual_bn_f16: bad args (tile 4 only)");
  NSM_CHECK_ARG(((uintptr_t)g % 8) == 0 && ((uintptr_t)y % 8) == 0 && ((uintptr_t)V % 16) == 0 &&
                    ((uintptr_t)dM % 16) == 0,
                "wino_dual_bn_f16: alignment");
  WinoGeom gm;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, gm), "wino_dual_bn_f16: bad shape");
  const int cw = f16_tx_cw();
  const long long gbytes = (long long)B * H * W * ldg * 2, ybytes = (long long)B * H * W * ldy * 2,
                  obytes = 36ll * gm.T * c_p * 2;
  if (cw == 2 && f16_up_buf() && gbytes < 0x7FFFFFFFll && ybytes < 0x7FFFFFFFll &&
      obytes < 0xFFFFFFFFll && gm.T * (c_p / 2) < (1ll << 31)) {
    hipLaunchKernelGGL(wino_dual_bn_f16_buf_kernel<4>, dim3(grid_1d(gm.T * c_p / 2)), dim3(256), 0,
                       as_stream(stream), (const bf16_t*)g, ldg, (const bf16_t*)y, ldy, H, W, c_p, gm.TH,
                       gm.TW, (int)gm.T, scale, shift, slope, mask, mean, coef, (bf16_t*)V, (bf16_t*)dM,
                       H2Scale{bound, wino_beta(4, 0)}, H2Scale{bound, wino_beta(4, 1)});
    NSM_LAUNCH_CHECK("wino_dual_bn_f16");
    return 0;
  }
  hipLaunchKernelGGL((cw == 2 ? wino_dual_bn_f16_kernel<4, 2> : wino_dual_bn_f16_kernel<4, 4>),
                     dim3(grid_1d(gm.T * c_p / cw)), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)g, ldg, (const bf16_t*)y, ldy, H, W, c_p, gm.TH, gm.TW, gm.T,
                     scale, shift, slope, mask, mean, coef, (bf16_t*)V, (bf16_t*)dM,
                     H2Scale{bound, wino_beta(4, 0)}, H2Scale{bound, wino_beta(4, 1)});
  NSM_LAUNCH_CHECK("wino_dual_bn_f16");
  return 0;
}

// the weight-gradient plan of the f16 path: the h2 plan's, on its 256 / 128 tiles
static WinoWgradPlan plan_wino_wgrad_f16(long long T, int cin_p, int cout_p, int nb) {
  WinoWgradPlan p = plan_wino_wgrad_h2(T, cin_p, cout_p, nb);
  // NSM_F16_WG_SPLITS: K splits of the 256x256 tiles (A/B)
  static const long long force = [] {
    const char* e = getenv("NSM_F16_WG_SPLITS");
    return e ? atoll(e) : 0ll;
  }();
  if (force > 0 && p.BM == 256 && p.BN == 256) {
    long long sp = force, maxs = (T + 255) / 256;
    if (sp > maxs) sp = maxs;
    long long kc = (T + sp - 1) / sp;
    kc = (kc + BK - 1) / BK * BK;
    sp = (T + kc - 1) / kc;
    p.splits = (int)sp;
    p.kchunk = (int)kc;
    p.slab_floats = (size_t)nb * sp * cout_p * cin_p;
    if (sp > 1) p.slab_floats += (size_t)nb * cout_p * cin_p;
  }
  if (force <= 0 && p.BM == 256 && p.BN == 256 && f16_wg_kt64()) {
    // K splits by a round model of the 256x256 blocks (one per CU): rounds x
    // (K / s x a + b) + the split sum's slab traffic c (s + 1) per tile, a, b,
    // c fitted on the B=64 step's conv5-conv7 weight gradients (kernel traces,
    // s = 1..8: conv6 1465 / 1299 / 1296 / 1345 us at s = 1..4, split sum
    // included; conv5 204 at s = 8 vs 136 at s = 3). The h2 planner's ~4
    // rounds left conv6 unsplit at 2.25 rounds and conv5 at 512-row splits
    const long long tiles = (long long)(cout_p / 256) * (cin_p / 256) * nb, cus = cu_count();
    const double a = 26.4e-3, b = 27.5, c = 0.0524;
    long long best = 1;
    double bt = 1e30;
    for (long long s = 1; s <= 8; ++s) {
      long long kc = (T + s - 1) / s;
      kc = (kc + BK - 1) / BK * BK;
      const long long se = (T + kc - 1) / kc;
      if (se != s) continue;
      const double t = (double)((tiles * s + cus - 1) / cus) * ((double)kc * a + b) +
                       (s > 1 ? c * (double)(s + 1) * (double)tiles : 0.0);
      if (t < bt) {
        bt = t;
        best = s;
      }
    }
    long long kc = (T + best - 1) / best;
    kc = (kc + BK - 1) / BK * BK;
    const long long sp = (T + kc - 1) / kc;
    p.splits = (int)sp;
    p.kchunk = (int)kc;
    p.slab_floats = (size_t)nb * sp * cout_p * cin_p;
    if (sp > 1) p.slab_floats += (size_t)nb * cout_p * cin_p;
  }
  if ((p.BM == 256 && p.BN == 256) || (p.BM == 128 && p.BN == 128)) return p;
  // (the h2 planner's smaller tiles: 128 x 128 with its ~512-block split)
  p.BM = p.BN = 128;
  const long long tiles = (long long)ceil_div(cout_p, 128) * ceil_div(cin_p, 128) * nb;
  long long sp = (512 + tiles - 1) / tiles, maxs = (T + 255) / 256;
  if (sp > maxs) sp = maxs;
  if (sp > 64) sp = 64;
  if (sp < 1) sp = 1;
  long long kc = (T + sp - 1) / sp;
  kc = (kc + BK - 1) / BK * BK;
  sp = (T + kc - 1) / kc;
  p.splits = (int)sp;
  p.kchunk = (int)kc;
  p.slab_floats = (size_t)nb * sp * cout_p * cin_p;
  if (sp > 1) p.slab_floats += (size_t)nb * cout_p * cin_p;
  return p;
}

extern "C" size_t nsm_wino_wgrad_f16_ws(int B, int H, int W, int cin_p, int cout_p, int tile) {
  WinoGeom g;
  if (!wino_geom(tile, B, H, W, g)) return 0;
  return plan_wino_wgrad_f16(g.T, cin_p, cout_p, g.alpha2).slab_floats;
}

// dw[co][ci][3][3] (reference layout) of the bf16 path's Winograd F(4x4) 3x3
// from dM (nsm_wino_dout_f16, scale source amax_dy) and the forward's V
// (nsm_wino_input_f16, scale source amax_x): batched split-K GEMMs on the f16
// matrix cores, then the filter transform (wgrad_wino_finish)
extern "C" int nsm_conv3x3_wgrad_wino_f16(const void* dM, const void* V, int B, int H, int W,
                                          int cin_p, int cout_p, int cin, int cout, int tile,
                                          float* dw, float* ws, size_t ws_floats,
                                          const uint32_t* amax_dy, const uint32_t* amax_x,
                                          void* stream) {
  NSM_CHECK_ARG(dM && V && dw && ws && amax_dy && amax_x && tile == 4,
                "conv3x3_wgrad_wino_f16: bad args");
  NSM_CHECK_ARG(cin_p % 128 == 0 && cout_p % 128 == 0 && cin <= cin_p && cout <= cout_p,
                "conv3x3_wgrad_wino_f16: channels (multiples of 128)");
  NSM_CHECK_ARG(((uintptr_t)dM % 16) == 0 && ((uintptr_t)V % 16) == 0 && ((uintptr_t)ws % 16) == 0,
                "conv3x3_wgrad_wino_f16: alignment");
  WinoGeom g;
  NSM_CHECK_ARG(wino_geom(tile, B, H, W, g), "conv3x3_wgrad_wino_f16: bad shape");
  NSM_CHECK_ARG(g.T * (long long)std::max(cin_p, cout_p) < (1ll << 30),
                "conv3x3_wgrad_wino_f16: operand too large");
  const int nb = g.alpha2;
  const WinoWgradPlan pl = plan_wino_wgrad_f16(g.T, cin_p, cout_p, nb);
  if (ws_floats < pl.slab_floats)
    return fail(NSM_E_WS, "conv3x3_wgrad_wino_f16: workspace too small");
  hipStream_t s = as_stream(stream);
  const int rc = wino_wgrad_gemm_f16((const bf16_t*)dM, (const bf16_t*)V, g.T, cin_p, cout_p, nb,
                                     pl.BM, pl.BN, pl.kchunk, pl.splits, ws,
                                     H2Scale{amax_dy, wino_beta(tile, 1)},
                                     H2Scale{amax_x, wino_beta(tile, 0)}, s);
  if (rc) return rc;
  return wgrad_wino_finish(ws, pl, nb, cout_p, cin_p, cin, cout, tile, dw, s);
}

// 1: fp32 GEMMs on the bf16 matrix cores by the exact split (default), 0: on
// v_mfma_f32_32x32x2_f32; returns the previous mode
extern "C" int nsm_set_f32_split(int mode) {
  const int prev = f32_split_mode();
  g_f32_split = mode < 0 ? 0 : (mode > 2 ? 2 : mode);
  return prev;
}

// ---- PMC calibration (tools/pmc_calib.py) -----------------------------------
// Launches of KNOWN byte counts in the access patterns of this library's
// kernels, so a rocprofv3 counter (WRITE_SIZE, FETCH_SIZE, TCC_EA0_RDREQ*) can
// be read against the bytes it should report before it is used on them
// (MI355X_MICROARCH.md §HBM calibrates only 16-B/lane global loads/stores).
// kind 0: read-only, global_load_dwordx4 (16 B/lane)
//      1: read-only, buffer_load ... lds (LDS-DMA, 16 B/lane; the GEMM loaders)
//      2: write-only, global_store_dwordx4
//      3: write-only, rows staged in LDS then raw_buffer_store_b128 (the
//         persistent h2 GEMM's fp32 epilogue)
//      4: write-only, raw_buffer_store_b64 (its f16-M epilogue)
//      5: write-only, global_store_dword (4 B/lane)
//      6: write-only, global_store_dwordx2 (8 B/lane)
// A read-only kernel writes one dword per block (its checksum) to dst.
__global__ void __launch_bounds__(256) pmc_calib_kernel(int kind, const u32x4* __restrict__ src,
                                                        u32x4* __restrict__ dst, long long n16) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[256 * 8];
  const long long stride = (long long)gridDim.x * 256;
  const long long i0 = (long long)blockIdx.x * 256 + threadIdx.x;
  unsigned acc = 0;
  if (kind == 0) {
    for (long long i = i0; i < n16; i += stride) {
      const u32x4 v = src[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  } else if (kind == 1) {
    // every wave DMAs 64 x 16 B per trip into its own LDS slice
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7FFFFFFF, 0x00020000);
    bf16_t* my = lds + (threadIdx.x >> 6) * 512;
    for (long long b = (long long)blockIdx.x * 256; b < n16; b += stride) {
      // wave-uniform chunk base; the byte offset of this lane's 16 B (< 2 GB)
      const long long wb = b + (threadIdx.x & ~63);
      if (wb < n16) {
        const uint32_t off = (uint32_t)((wb + (threadIdx.x & 63)) * 16);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)my, 16, off, 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const u32x4 v = *(const u32x4*)&lds[threadIdx.x * 8];
    acc = v.x ^ v.y ^ v.z ^ v.w;
  } else if (kind == 2) {
    for (long long i = i0; i < n16; i += stride) dst[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
  } else if (kind == 3 || kind == 4) {
    // 16 rows x 64 fp32 per wave staged in LDS (as the epilogue), then the
    // buffer stores of 16 B (kind 3) or of 8 B f16x4 (kind 4) per lane
    float* stg = (float*)lds + (threadIdx.x >> 6) * 256;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, 0x7FFFFFFF, 0x00020000);
    const long long per = kind == 3 ? 1 : 2;  // lanes per 16 B of output
    const long long nl = n16 * per;           // lane-stores in total
    for (long long i = i0; i < nl; i += stride) {
      stg[(threadIdx.x & 63) * 4 + 0] = (float)i;
      __builtin_amdgcn_wave_barrier();
      const f32x4 v = *(const f32x4*)&stg[(threadIdx.x & 63) * 4];
      if (kind == 3)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (uint32_t)(i * 16), 0,
                                               0);
      else
        __builtin_amdgcn_raw_buffer_store_b64(pack_f16x4(v), r, (uint32_t)(i * 8), 0, 0);
    }
  } else if (kind == 5) {
    unsigned* d = (unsigned*)dst;
    for (long long i = i0; i < n16 * 4; i += stride) d[i] = (unsigned)i;
  } else if (kind == 6) {
    u32x2* d = (u32x2*)dst;
    for (long long i = i0; i < n16 * 2; i += stride) d[i] = u32x2{(unsigned)i, 7u};
  }
  if (kind <= 1) {
    for (int o = 32; o > 0; o >>= 1) acc ^= (unsigned)__shfl_xor((int)acc, o);
    if ((threadIdx.x & 63) == 0 && acc == 0x9E3779B9u) ((unsigned*)dst)[blockIdx.x] = acc;
  }
}

extern "C" int nsm_pmc_calib(int kind, const void* src, void* dst, int64_t bytes, void* stream) {
  NSM_CHECK_ARG(kind >= 0 && kind <= 6 && bytes > 0 && bytes % 4096 == 0 && bytes < (1ll << 31),
                "pmc_calib: kind 0..6, bytes a multiple of 4096 below 2 GB");
  NSM_CHECK_ARG(dst && (kind >= 2 || src), "pmc_calib: null pointer");
  const long long n16 = bytes / 16;
  hipLaunchKernelGGL(pmc_calib_kernel, dim3(2048), dim3(256), 0, as_stream(stream), kind,
                     (const u32x4*)src, (u32x4*)dst, n16);
  NSM_LAUNCH_CHECK("pmc_calib");
  return 0;
}
