/*
 * nsm.h — C ABI of libnsm.so, the MI355X-native (gfx950 / CDNA4) hot path of
 * the Neural-Shadow-Mapping U-Net of SDU-Gary/PCSS-Unet.
 *
 * The reference exposes no FFI: its boundary is the Python nn.Module /
 * loss-callable surface. Each entry point below replaces the
 * ATen op(s) the reference dispatches at the cited line; the Python host
 * (pcss-unet_amd/nsm_amd) binds them with ctypes underneath a drop-in
 * `Unetmodel.Unet` / `customLoss.CustomLoss` / `pert_loss.PerturbationLoss`.
 *
 * Conventions (all entry points):
 *   - extern "C", POD arguments only: device pointers, int / int64 sizes,
 *     float hyper-parameters, and the HIP stream as `void*` (hipStream_t).
 *   - Activations are NHWC fp32, channel count padded to a multiple of 32
 *     ("cp"); padded channels are kept exactly zero by zero weights/affine.
 *   - Caller owns all memory (PyTorch caching allocator); the library never
 *     allocates or synchronises; every launch is asynchronous on `stream`
 *     and hipGraph-capturable.
 *   - Return 0 on success, else NSM_E_* ; message via nsm_get_last_error().
 */
#ifndef NSM_H_
#define NSM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NSM_OK 0
#define NSM_E_ARG 1 /* bad shape / pointer / alignment */
#define NSM_E_HIP 2 /* HIP launch error */
#define NSM_E_WS 3  /* workspace too small */

/* storage type of activation / activation-gradient buffers (void* args):
 * every elementwise entry point below that takes `int dtype` reads and writes
 * its NHWC tensors in that type and computes in fp32 */
#define NSM_F32 0
#define NSM_BF16 1
#define NSM_F16 2  /* IEEE half storage (the fp16-autocast mode) */

/* An operand-maximum slot (the `amax` arguments below): NSM_AMAX_WORDS uint32,
 * zeroed before its producer runs. It holds max|x| of one fp32 GEMM operand as
 * 64 partial maxima (fp32 bit patterns, compared as unsigned) on separate
 * 128-B lines; the f16x2 GEMMs reduce them to the operand's scale. */
#define NSM_AMAX_WORDS 2048
#define NSM_PACK_FWD 0   /* w[co][ci][k][k] -> [co_p][tap][ci_p]            */
#define NSM_PACK_DGRAD 1 /* w[co][ci][k][k] -> [ci_p][tap'][co_p], tap'=k*k-1-tap */

/* ---- library ----------------------------------------------------------- */
int nsm_version(void);
int nsm_get_last_error(char* buf, size_t n);

/* ---- parameter layout ------------------------------------------------------
 * Replaces the implicit weight layout of nn.Conv2d (Unetmodel.py:21,26) with
 * the MFMA operand layout; nsm_pad_vec pads bias / BN affine to cp. */
int nsm_pack_conv_weight(const float* w, int cout, int cin, int ksize, int cout_p, int cin_p,
                         int mode, float* out, void* stream);
int nsm_pad_vec(const float* v, int n, int n_p, float* out, void* stream);

/* All weight layouts of one training step in ONE launch (replaces the per-layer
 * nsm_pack_conv_weight / nsm_pack_conv_weight_bf16 / nsm_wino_weight / nsm_pad_vec
 * calls). kind 0: pack fp32, 1: pack bf16, a = {cout, cin, taps, cout_p, cin_p,
 * mode}; kind 2: Winograd U, a = {cout, cin, n_p, k_p, flip, tile}; kind 3: pad
 * vector, a = {n, n_p}; kind 4: Winograd U as an h2 tensor [alpha^2][n_p][2 k_p]
 * (nsm_to_h2's layout), a as kind 2, amax (required) = the slot that receives
 * max|w| of the filters, the scale source of U (beta = nsm_wino_beta(tile, 2));
 * a[6] = 0, or the first block (base / 512) + 1 of an earlier kind-4 job over
 * the same filters whose maximum this job shares (same slot); kind 5: pack as
 * an h2 tensor (a as kind 0; FWD [cout_p][2 taps cin_p], DGRAD [cin_p][2 taps
 * cout_p] float16), amax (required) = the slot that receives max|w| (beta 1),
 * a[6] as kind 4 (the FWD job of the same weight); kind 6: Winograd U as a
 * single-plane scaled f16 tensor [alpha^2][n_p][k_p] (the bf16 path's F(4x4)
 * forward, nsm_wino_gemm_f16), a and amax as kind 4; kind 7: pack IEEE half
 * (the fp16-autocast mode's NSM_F16 convolutions), a as kind 1. `base` = the job's first
 * item in the launch (jobs in ascending base order, consecutive);
 * nsm_prep_items() = the job's extent in the launch (its item count rounded up
 * to whole 512-item blocks: add it to get the next base; total_items = the
 * sum). jobs_dev: a device copy. max_pass: the table holds kind-4 / 5 / 6 jobs
 * (their max|w| pass runs first, one word per block into pmax [total_items /
 * 512], so those slots need no zeroing; their line 0 is stored, lines 1..63
 * must hold 0). zero0 / zero1 (nzero words each, may be 0): zeroed by the first
 * launch before anything is written — the step's weight slots (kinds 0 and 2
 * record max|written| by atomics; kinds 4-6 rely on lines 1..63 = 0) and the
 * forward's activation slots — so the step needs no fill launches. */
typedef struct {
  int kind;
  int a[7];
  long long base;
  const float* src;
  void* dst;
  uint32_t* amax; /* kinds 0, 2 (may be NULL): atomic max of |written| as fp32
                     bits (zeroed beforehand): the f16x2 GEMM operand scale;
                     kinds 4, 5, 6: max|w| (see above) */
} NsmPrepJob;
long long nsm_prep_items(const NsmPrepJob* job);
int nsm_prep_weights(const NsmPrepJob* jobs_dev, int njobs, long long total_items, int max_pass,
                     uint32_t* pmax, uint32_t* zero0, int64_t nzero0, uint32_t* zero1,
                     int64_t nzero1, void* stream);

/* ---- convolution as MFMA implicit GEMM (fp32 in, fp32 accumulate) ----------
 * nsm_conv_fwd: y[p][co] = bias[co] + sum_{tap,ci} pro(x[p+off(tap)][ci]) * W
 *   Replaces F.conv2d 3x3 pad 1 / 1x1 of DoubleConv (Unetmodel.py:21,26) and,
 *   with NSM_PACK_DGRAD weights and bias=NULL, its input-gradient (autograd
 *   ConvolutionBackward dgrad).  Optional prologue (pro_scale!=NULL):
 *   pro(v) = lrelu(v*scale[ci]+shift[ci], slope) * mask[b*cin_p+ci] on
 *   in-bounds pixels (3x3 halo stays 0) — the BN-apply + LeakyReLU +
 *   Dropout2d between the two convs (Unetmodel.py:22-24) fused into the
 *   operand load; with scale 1, shift 0, slope 0 it is the ReLU between the
 *   VGG19 convs (customLoss.py:20). mask may be NULL. */
int nsm_conv_fwd(const float* x, int ldx, int B, int H, int W, int cin_p, const float* wpk,
                 const float* bias, int cout_p, int ksize, float* y, int ldy, const float* pro_scale,
                 const float* pro_shift, const float* pro_mask, float slope, void* stream);

/* Same, plus fused BatchNorm batch statistics of y (bias included): if
 * stats != NULL it receives per-M-block partials [ceil(M/R)][2][cout_p]
 * {sum, M2 about the block mean}, R = nsm_conv_stat_rows(); feed them to
 * nsm_bn_finalize_train with rows_per_chunk = R (replaces the separate
 * statistics pass of nn.BatchNorm2d in train mode, Unetmodel.py:22,27). */
int nsm_conv_stat_rows(int B, int H, int W, int cout_p);
int nsm_conv_fwd_stats(const float* x, int ldx, int B, int H, int W, int cin_p, const float* wpk,
                       const float* bias, int cout_p, int ksize, float* y, int ldy,
                       const float* pro_scale, const float* pro_shift, const float* pro_mask,
                       float slope, float* stats, const uint32_t* amax_x, const uint32_t* amax_w,
                       void* stream);
/* amax_x / amax_w (device operand-maximum slots of x and wpk, both or neither;
 * ignored with a prologue): the GEMM runs the f16x2 split (NSM_F32_SPLIT=2). */

/* Winograd F(m x m, 3x3) 3x3 convolution (same padding 1) for deep layers,
 * tile m in {2, 4, 6}, alpha = m + 2, T = B*ceil(H/m)*ceil(W/m) tiles:
 * nsm_wino_weight transforms w[co][ci][3][3] into U[alpha^2][n_p][k_p]
 * (flip=0: forward, n=co, k=ci; flip=1: input-gradient, n=ci, k=co, filter
 * rotated 180 deg); nsm_conv3x3_wino then computes y = conv(x, W) + bias
 * through alpha^2 batched MFMA GEMMs, using nsm_wino_ws() floats of workspace.
 * Replaces the same F.conv2d 3x3 / ConvolutionBackward dgrad as nsm_conv_fwd
 * (Unetmodel.py:21) with 2.25x (m=2), 4x (m=4) or 5.06x (m=6) fewer multiplies. */
size_t nsm_wino_ws(int B, int H, int W, int cin_p, int cout_p, int tile);
int nsm_wino_weight(const float* w, int cout, int cin, int n_p, int k_p, int flip, int tile,
                    float* U, void* stream);
int nsm_conv3x3_wino(const float* x, int ldx, int B, int H, int W, int cin_p, const float* U,
                     const float* bias, int cout_p, int tile, int relu, float* y, int ldy,
                     float* ws, size_t ws_floats, void* stream);
/* the three stages of nsm_conv3x3_wino: V[alpha^2][T][cin_p] = B^T d B
 * (relu != 0: d = max(x, 0), the pending ReLU of a VGG feature map);
 * Mb[alpha^2][T][cout_p] = V . U^T (batched MFMA GEMMs); y = A^T Mb A + bias */
int nsm_wino_input(const float* x, int ldx, int B, int H, int W, int cin_p, int tile, int relu,
                   float* V, void* stream);
/* nsm_wino_input of the bilinear align_corners resize of x [B][hi][wi][ldx] to
 * H x W (Unetmodel.py:51-60,122-130: the decoder's x2 upsample feeding a
 * Winograd conv): the resized tensor is sampled inside the transform and never
 * written (relu must be 0 when hi, wi != H, W). amax (device, may be NULL):
 * atomic max of |V| as fp32 bits, the f16x2 GEMM's operand scale
 * (nsm_wino_gemm_s); zero it beforehand. */
int nsm_wino_input_resize(const float* x, int ldx, int B, int hi, int wi, int H, int W, int cin_p,
                          int tile, int relu, float* V, uint32_t* amax, void* stream);
int nsm_wino_gemm(const float* V, const float* U, int B, int H, int W, int cin_p, int cout_p,
                  int tile, float* Mb, void* stream);
/* nsm_wino_gemm with the operands' absolute maxima: amax_v / amax_u (device)
 * = bits of max|V|, max|U| (fp32 bit patterns compare as unsigned). With the
 * fp32 split on, the GEMM then runs the f16x2 split (power-of-two scaled
 * operands, two fp16 terms, three f16 MFMA products; nsm_conv_split16.inc)
 * instead of the bf16 three-way split; NULL maxima = nsm_wino_gemm. */
int nsm_wino_gemm_s(const float* V, const float* U, int B, int H, int W, int cin_p, int cout_p,
                    int tile, float* Mb, const uint32_t* amax_v, const uint32_t* amax_u,
                    void* stream);
/* max|x[i]| over n floats into the operand-maximum slot out (NSM_AMAX_WORDS,
 * zeroed first; NaN counts above +Inf): the maximum a GEMM operand needs when
 * its producer does not record it. */
int nsm_absmax(const float* x, int64_t n, uint32_t* out, void* stream);
/* p[0..n) = 0 (uint32 words): the activation-maximum slots of a forward whose
 * weight preparation does not run (frozen inference weights, GraphedUnet) */
int nsm_zero_u32(uint32_t* p, int64_t n, void* stream);
/* the same over n bf16 values (x 16-B aligned): the input maximum of a bf16
 * F(4x4) Winograd conv whose input producer records none (the decoder's lazy
 * resampling, NSM_LAZY_DECODER=1) */
int nsm_absmax_bf16(const void* x, int64_t n, uint32_t* out, void* stream);
/* PMC calibration (tools/pmc_calib.py): one launch moving exactly `bytes`
 * (a multiple of 4096, < 2 GB) in one access pattern of this library's
 * kernels, so rocprofv3's byte counters can be checked against a known count:
 * kind 0 read by global_load_dwordx4, 1 read by LDS-DMA buffer_load ... lds,
 * 2 write by global_store_dwordx4, 3 write by LDS-staged raw_buffer_store_b128
 * (the persistent h2 GEMM's fp32 epilogue), 4 write by raw_buffer_store_b64
 * (its f16-M epilogue), 5 write by 4-B stores, 6 write by 8-B stores. A
 * read-only kind writes at most one dword per block of 2048 to dst. */
int nsm_pmc_calib(int kind, const void* src, void* dst, int64_t bytes, void* stream);
/* ---- pre-split ("h2") Winograd operands (csrc/nsm_conv_h2.inc) -------------
 * An h2 tensor is an fp32 [rows][C] matrix X stored as fp16 [rows][2C]: with
 * s = 2^(15 - ceil(log2(beta * m))), m = the max of the operand-maximum slot
 * `amax` (of X itself, or of the tensor X is a transform of, beta the
 * transform's bound), the 8 channels of chunk j are h = f16(x s) at 16j..16j+7
 * and l = f16(x s - h) at 16j+8..16j+15. Same bytes as fp32; the GEMMs read
 * both terms by LDS-DMA and multiply h.h + h.l + l.h on the f16 matrix cores.
 * nsm_to_h2: X [rows][C] (C % 8 == 0) -> h2 (test / benchmark helper). */
int nsm_to_h2(const float* x, int64_t rows, int C, const uint32_t* amax, float beta, void* out,
              void* stream);
/* wino_beta(tile, which): the bound beta of a Winograd transform,
 * max|out| <= beta * max|in| (which 0: input B^T d B, 1: output gradient
 * A dY A^T, 2: filter G g G^T) — the factor between an h2 operand's scale
 * source and the operand */
float nsm_wino_beta(int tile, int which);
/* nsm_wino_input_resize writing V as an h2 tensor [alpha^2][T][2 cin_p]; scale
 * source amax_x = max|x| (recorded by x's producer), beta = wino_beta(tile, 0) */
int nsm_wino_input_h2(const float* x, int ldx, int B, int hi, int wi, int H, int W, int cin_p,
                      int tile, void* Vh, const uint32_t* amax_x, void* stream);
/* nsm_wino_dual_input writing Vd and dM as h2 tensors; scale source amax_dy =
 * max|dy| (its producer's), betas wino_beta(tile, 0) and (tile, 1) */
int nsm_wino_dual_input_h2(const float* dy, int lddy, int B, int H, int W, int c_p, int tile,
                           void* Vh, void* dMh, const uint32_t* amax_dy, void* stream);
/* nsm_wino_dual_input_h2 of a deferred BN backward (nsm_wino_dual_input_bn's
 * operands: g = dA1, y = Y1, the finalize coefficients): dY1 is formed per patch
 * element, never stored; bound: the dY1 bound nsm_bn_bwd_finalize derived from
 * max|k1 dz| — the scale source of Vh / dMh and of the GEMMs reading them.
 * Replaces the BN-backward apply + transform of the reference's autograd
 * backward through Unetmodel.py:21-24 (DoubleConv conv.0 -> BN -> LeakyReLU). */
/* The bf16 path's Winograd F(4x4) forward (Unetmodel.py:21, the DoubleConv's
 * 3x3 at >= 512 channels) on single-plane scaled f16 operands: V = s B^T x B
 * from the bf16 NHWC input x (amax_x: max|x| recorded by x's producer, beta =
 * nsm_wino_beta(4, 0)) as [36][T][cin_p] f16; the batched GEMM with U of prep
 * kind 6 (M fp32 [36][T][cout_p]); the output transform writing bf16 y [+ bias]
 * and, with partial, the BN partials of the rounded values (nslot as
 * nsm_wino_output_stats, nsm_wino_stat_slots). tile 4 only. */
int nsm_wino_input_f16(const void* x, int ldx, int B, int H, int W, int cin_p, int tile, void* V,
                       const uint32_t* amax_x, void* stream);
/* nsm_wino_input_f16 of the align_corners bilinear resize of x (bf16 [B][hi][wi]
 * [cin_p] NHWC, ld ldx) to H x W (the decoder's x2 upsample, Unetmodel.py:
 * 122-130), sampled per patch element and rounded to bf16 as the materialised
 * upsample would be; amax_x: max|x| (it bounds the upsample too). */
int nsm_wino_input_f16_resize(const void* x, int ldx, int B, int hi, int wi, int H, int W,
                              int cin_p, int tile, void* V, const uint32_t* amax_x, void* stream);
int nsm_wino_gemm_f16(const void* V, const void* U, int B, int H, int W, int cin_p, int cout_p,
                      int tile, float* Mb, const uint32_t* amax_v, float beta_v,
                      const uint32_t* amax_u, float beta_u, void* stream);
int nsm_wino_output_bf16(const float* Mb, int B, int H, int W, int cout_p, int tile,
                         const float* bias, void* y, int ldy, float* partial, int nslot,
                         void* stream);
/* The same GEMM / output transform with M held as f16 (half the bytes of the
 * GEMM's writes and the output transform's reads): nsm_wino_gemm_f16m writes
 * M16 [36][T][cout_p] f16, each 64 x 64 tile of each component scaled by the
 * power of two that puts ITS maximum at <= 2^15 (m16e [36][ceil(T/64)][cout_p/64]
 * int32 receives the exponents, cout_p % 64 == 0), so a tile's values stay
 * normal f16 down to 2^-29 of its own maximum; nsm_wino_output_bf16m reads the
 * exponents and the same scale slots / bounds to undo it. NSM_BF16_M16 selects
 * this pair in the Python path. */
/* Both F(4x4) transforms of the bf16 output gradient dY from one read: V
 * (the input gradient's operand, as nsm_wino_input_f16 of dY) and dM (as
 * nsm_wino_dout_f16), scale source amax_dy for both. NSM_BF16_DUAL selects it
 * in the Python path. */
int nsm_wino_dual_f16(const void* dy, int lddy, int B, int H, int W, int c_p, int tile, void* V,
                      void* dM, const uint32_t* amax_dy, void* stream);
/* nsm_wino_dual_f16 of a dY that is never stored: dY = k1 dz + k2 (y - mean) +
 * k3, dz = g lrelu'(y scale + shift) mask[b][c], formed per element and rounded
 * to bf16 as nsm_bn_bwd_apply writes it (g = dA1 of nsm_conv1x1_dgrad_bnbwd
 * mode 1, y = Y1, coef = the finalize's {k1, k2, k3}), the transforms scaled
 * from `bound` (nsm_bn_bwd_finalize's dY bound slot). The bf16 path's F(4x4)
 * layers (Unetmodel.py:21-24 backward); removes the nsm_bn_bwd_apply pass. */
int nsm_wino_dual_bn_f16(const void* g, int ldg, const void* y, int ldy, int B, int H, int W, int c_p,
                         int tile, const float* scale, const float* shift, float slope,
                         const float* mask, const float* mean, const float* coef, void* V, void* dM,
                         const uint32_t* bound, void* stream);
int nsm_wino_gemm_f16m(const void* V, const void* U, int B, int H, int W, int cin_p, int cout_p,
                       int tile, void* M16, int* m16e, const uint32_t* amax_v, float beta_v,
                       const uint32_t* amax_u, float beta_u, void* stream);
int nsm_wino_output_bf16m(const void* M16, const int* m16e, int B, int H, int W, int cin_p,
                          int cout_p, int tile, const uint32_t* amax_v, float beta_v,
                          const uint32_t* amax_u, float beta_u, const float* bias, void* y, int ldy,
                          float* partial, int nslot, void* stream);
/* eval: the same output transform writing lrelu(y*act_scale + act_shift,
 * slope) in bf16 (the DoubleConv's first BatchNorm from its running
 * statistics + LeakyReLU, Unetmodel.py:22-23, fused; the bf16 eval forward's
 * F(4x4) layers) */
int nsm_wino_output_bf16m_act(const void* M16, const int* m16e, int B, int H, int W, int cin_p,
                              int cout_p, int tile, const uint32_t* amax_v, float beta_v,
                              const uint32_t* amax_u, float beta_u, const float* bias, void* y,
                              int ldy, const float* act_scale, const float* act_shift, float slope,
                              void* stream);
/* Its weight gradient: dM = s (A dY A^T) of the bf16 output gradient dY as
 * [36][T][c_p] f16 (amax_dy: max|dY| from dY's producer, beta =
 * nsm_wino_beta(4, 1)); then dw [cout][cin][3][3] from dM and the forward's V
 * (batched split-K GEMMs on the f16 matrix cores, one product per k-step, and
 * the filter transform); ws >= nsm_wino_wgrad_f16_ws floats. tile 4. */
int nsm_wino_dout_f16(const void* dy, int lddy, int B, int H, int W, int c_p, int tile, void* dM,
                      const uint32_t* amax_dy, void* stream);
size_t nsm_wino_wgrad_f16_ws(int B, int H, int W, int cin_p, int cout_p, int tile);
int nsm_conv3x3_wgrad_wino_f16(const void* dM, const void* V, int B, int H, int W, int cin_p,
                               int cout_p, int cin, int cout, int tile, float* dw, float* ws,
                               size_t ws_floats, const uint32_t* amax_dy, const uint32_t* amax_x,
                               void* stream);
int nsm_wino_dual_input_bn_h2(const float* g, int ldg, const float* y, int ldy, int B, int H, int W,
                              int c_p, int tile, const float* scale, const float* shift,
                              float slope, const float* mask, const float* mean, const float* coef,
                              void* Vh, void* dMh, const uint32_t* bound, void* stream);
/* the weight gradient of a Winograd conv from h2 dM (nsm_wino_dual_input_h2) and
 * h2 V (nsm_wino_input_h2): batched split-K GEMMs on the f16 matrix cores, then
 * the filter transform; ws >= nsm_wino_wgrad_h2_ws floats */
size_t nsm_wino_wgrad_h2_ws(int B, int H, int W, int cin_p, int cout_p, int tile);
int nsm_conv3x3_wgrad_wino_h2(const void* dMh, const void* Vh, int B, int H, int W, int cin_p,
                              int cout_p, int cin, int cout, int tile, float* dw, float* ws,
                              size_t ws_floats, const uint32_t* amax_dy, const uint32_t* amax_x,
                              void* stream);
/* nsm_wino_gemm on h2 operands: V [alpha^2][T][2 cin_p], U [alpha^2][cout_p][2 cin_p]
 * with their scale sources (amax_v, beta_v), (amax_u, beta_u); Mb fp32 as
 * nsm_wino_gemm. */
int nsm_wino_gemm_h2(const void* V, const void* U, int B, int H, int W, int cin_p, int cout_p,
                     int tile, float* Mb, const uint32_t* amax_v, float beta_v,
                     const uint32_t* amax_u, float beta_u, void* stream);
/* ---- the DoubleConv's 1x1 convolution on h2 operands (csrc/nsm_conv_h2d.inc)
 * Replaces nn.Conv2d(in, out, 1) (Unetmodel.py:26), its input gradient with
 * the first BN's backward fused (as nsm_conv1x1_dgrad_bnbwd) and its weight
 * gradient, for the fp32 train step: xh / dy2h / dyh are h2 tensors (the
 * activated operand from nsm_bn_act_h2, the output-BN gradient from
 * nsm_to_h2), wh / w2dh the FWD / DGRAD h2 packs of prep kind 5, each with its
 * scale source slot (beta 1). nsm_conv1x1_h2: y [M][ldy] fp32 = x W^T + bias,
 * stats (may be NULL) = BN partials [ceil(M/R)][2][cout_p] with R =
 * nsm_conv1x1_h2_rows(M, cout_p, 2 cin_p, 0). nsm_conv1x1_dgrad_bnbwd_h2: modes
 * and outputs as nsm_conv1x1_dgrad_bnbwd, partial rows of R =
 * nsm_conv1x1_h2_rows(M, cip, 2 cop, 1) pixels, HW = pixels per image (mask row).
 * nsm_conv1x1_wgrad_h2: dw [cout][cin] (reference layout) with ws >=
 * nsm_conv1x1_wgrad_h2_ws floats. M = pixels. */
int nsm_conv1x1_h2_rows(int M, int N, int K, int bnbwd);
int nsm_conv1x1_h2(const void* xh, int M, int cin_p, const void* wh, const float* bias, int cout_p,
                   float* y, int ldy, float* stats, const uint32_t* amax_x,
                   const uint32_t* amax_w, void* stream);
int nsm_conv1x1_dgrad_bnbwd_h2(const void* dy2h, int M, int cop, const void* w2dh, int cip,
                               const float* y1, int ldy1, const float* scale, const float* shift,
                               const float* mean, const float* invstd, const float* mask, int HW,
                               float slope, int mode, float* partial, const float* coef,
                               float* out, int ldo, const uint32_t* amax_dy2,
                               const uint32_t* amax_w, uint32_t* amax_out, uint32_t* amax_k1dz,
                               void* stream);
size_t nsm_conv1x1_wgrad_h2_ws(int M, int cin_p, int cout_p);
/* (amax_k1dz, modes 0 / 1, may be NULL: the slot receiving max|scale * dz|,
 * nsm_bn_bwd_finalize's bound term for an h2 dY1 from nsm_bn_bwd_apply_h2) */
int nsm_conv1x1_wgrad_h2(const void* dyh, const void* xh, int M, int cin_p, int cout_p, int cin,
                         int cout, float* dw, float* ws, size_t ws_floats, const uint32_t* amax_dy,
                         const uint32_t* amax_x, void* stream);
/* The direct 3x3 convolution (conv2's, Cin < 64: Unetmodel.py:21) of the
 * fp32 train step on h2 operands: nsm_conv3x3_h2 y = conv3x3(x) + bias (pad 1)
 * from xh [B*H*W][2 cin_p] (nsm_input_prep_h2; for the input gradient the h2
 * dY1 with the DGRAD pack and bias NULL), wh the prep-kind-5 pack [cout_p][9]
 * [2 cin_p], stats = BN partials of nsm_conv3x3_h2_rows(M, cout_p) rows;
 * nsm_conv3x3_wgrad_h2 dw [cout][cin][3][3] from the h2 dY and X (cout_p 32). */
int nsm_conv3x3_h2_rows(int M, int N);
int nsm_conv3x3_h2(const void* xh, int B, int H, int W, int cin_p, const void* wh,
                   const float* bias, int cout_p, float* y, int ldy, float* stats,
                   const uint32_t* amax_x, const uint32_t* amax_w, void* stream);
size_t nsm_conv3x3_wgrad_h2_ws(int B, int H, int W, int cin_p, int cout_p);
int nsm_conv3x3_wgrad_h2(const void* dyh, const void* xh, int B, int H, int W, int cin_p,
                         int cout_p, int cin, int cout, float* dw, float* ws, size_t ws_floats,
                         const uint32_t* amax_dy, const uint32_t* amax_x, void* stream);
/* fp32 GEMM arithmetic of every fp32 convolution (the batched GEMMs of
 * nsm_wino_gemm / nsm_conv3x3_wino, the weight gradient of
 * nsm_conv3x3_wgrad_wino, the direct implicit GEMMs): 2 (default, env
 * NSM_F32_SPLIT) = the f16x2 split (power-of-two scaled operands as two fp16
 * terms, three v_mfma_f32_32x32x16_f16 products, fp32 accumulation) for the
 * GEMMs whose callers pass their operands' maxima, the bf16 split elsewhere;
 * 1 = each fp32 operand split exactly into three bf16 terms, the six products
 * above fp32 rounding on v_mfma_f32_32x32x16_bf16 with fp32 accumulation
 * (fp32 accuracy, 2.67x fewer MFMA cycles); 0 = v_mfma_f32_32x32x2_f32.
 * Returns the previous mode.
 * Replaces no reference interface (the reference runs cuDNN fp32 convs,
 * Unetmodel.py:16-27); host-wide setting, not per stream. */
int nsm_set_f32_split(int mode);
int nsm_wino_output(const float* Mb, int B, int H, int W, int cout_p, int tile, const float* bias,
                    float* y, int ldy, void* stream);
/* nsm_wino_output that also emits the BatchNorm batch statistics of y
 * (Unetmodel.py:21-22, the BN after a Winograd 3x3 conv) as counted partials
 * partial[nslot][3][cout_p] = {sum, M2, count}. nslot: a multiple of
 * nsm_wino_stat_step(cout_p, tile) = 256 / gcd(cout_p / channels per thread,
 * 256) (4 channels per thread for F(2x2) / F(4x4), 2 for F(6x6); 1 with
 * NSM_F6_OUT_CW=1); nsm_wino_stat_slots gives the tuned count (0 there: the
 * separate nsm_bn_stats pass is faster). */
int nsm_wino_output_stats(const float* Mb, int B, int H, int W, int cout_p, int tile,
                          const float* bias, float* y, int ldy, float* partial, int nslot,
                          void* stream);
int nsm_wino_stat_slots(int B, int H, int W, int cout_p, int tile);
int nsm_wino_stat_step(int cout_p, int tile);

/* Winograd weight gradient of the same 3x3 conv: dw[co][ci][3][3] (reference
 * layout, real dims) from dy [pixels][cout_p] and the forward's transformed
 * input V[alpha^2][T][cin_p] (nsm_wino_input output, same tile). */
size_t nsm_wino_wgrad_ws(int B, int H, int W, int cin_p, int cout_p, int tile);
int nsm_conv3x3_wgrad_wino(const float* dy, int lddy, const float* V, int B, int H, int W,
                           int cin_p, int cout_p, int cin, int cout, int tile, float* dw,
                           float* ws, size_t ws_floats, void* stream);
/* Both Winograd transforms of a 3x3 conv's output gradient dy [B*H*W][c_p]
 * from one read: V = the input transform for its input-gradient conv (as
 * nsm_wino_input), dM = the transform nsm_conv3x3_wgrad_wino applies (each
 * [(tile+2)^2][T][c_p]); then nsm_conv3x3_wgrad_wino_dm takes dM instead of dy.
 * amax_v / amax_dm (device, may be NULL): atomic max of |V| / |dM| (fp32 bits). */
int nsm_wino_dual_input(const float* dy, int lddy, int B, int H, int W, int c_p, int tile,
                        float* V, float* dM, uint32_t* amax_v, uint32_t* amax_dm, void* stream);
/* As nsm_wino_dual_input, with dy not materialised: each element is the
 * first BatchNorm's backward of g (grad wrt its LeakyReLU(+Dropout2d) output)
 * and y (its input), exactly what nsm_bn_bwd_apply(g, y, ..., coef) would
 * store (Unetmodel.py:21-24). */
int nsm_wino_dual_input_bn(const float* g, int ldg, const float* y, int ldy, int B, int H, int W,
                           int c_p, int tile, const float* scale, const float* shift, float slope,
                           const float* mask, const float* mean, const float* coef, float* V,
                           float* dM, uint32_t* amax_v, uint32_t* amax_dm, void* stream);
/* amax_dm / amax_v (device, both or neither): max|dM|, max|V| as recorded by
 * their producers -> the weight-gradient GEMM runs the f16x2 split. */
int nsm_conv3x3_wgrad_wino_dm(const float* dM, const float* V, int B, int H, int W, int cin_p,
                              int cout_p, int cin, int cout, int tile, float* dw, float* ws,
                              size_t ws_floats, const uint32_t* amax_dm, const uint32_t* amax_v,
                              void* stream);

/* nsm_conv_wgrad: dw[co][ci][kh][kw] (real cout x cin, reference layout) =
 *   sum_p dy[p][co] * pro(x[p+off(tap)][ci]); deterministic split-K over
 *   pixels through `ws` (nsm_conv_wgrad_ws() floats). Replaces the weight
 *   gradient of ConvolutionBackward for Unetmodel.py:21,26. If dbias != NULL
 *   it is left untouched (bias grads come from nsm_bn_bwd_finalize). */
size_t nsm_conv_wgrad_ws(int B, int H, int W, int cin_p, int cout_p, int ksize);
int nsm_conv_wgrad(const float* dy, int lddy, const float* x, int ldx, int B, int H, int W,
                   int cin_p, int cout_p, int ksize, const float* pro_scale, const float* pro_shift,
                   const float* pro_mask, float slope, float* ws, size_t ws_floats, int cin, int cout,
                   float* dw, const uint32_t* amax_dy, const uint32_t* amax_x, void* stream);

/* ---- BatchNorm2d(eps, momentum) train/eval (Unetmodel.py:22,27) ----------- */
int nsm_reduce_chunks(int M, int C); /* partial-buffer rows for the two below */
int nsm_reduce_rows(int M, int C);   /* rows per chunk of that plan */
/* per-channel chunk partials {sum, M2 about chunk mean}: partial[nchunk][2][C] */
int nsm_bn_stats(const void* y, int ld, int M, int C, float* partial, int nchunk, int dtype,
                 void* stream);
/* merge partials; batch mean/biased var normalise; unbiased var feeds running
 * stats, applied n_updates times (2 for conv5: checkpoint recompute,
 * Unetmodel.py:114-116); num_batches_tracked += n_updates.
 * Emits scale=gamma*invstd, shift=beta-mean*scale, mean, invstd.
 * rows_per_chunk == 0: counted partials [nchunk][3][C] = {sum, M2, count}
 * (nsm_wino_output_stats); nsm_bn_partials_merge keeps that layout. */
int nsm_bn_finalize_train(const float* partial, int nchunk, int rows_per_chunk, int M, int C,
                          int c_real,
                          const float* gamma, const float* beta, float* run_mean, float* run_var,
                          int64_t* num_batches, float momentum, float eps, int n_updates,
                          float* mean, float* invstd, float* scale, float* shift, uint32_t* bound,
                          float bound_mul, void* stream);
/* bound (may be NULL): operand-maximum slot receiving, as the atomic max of its
 * channels, bound_mul * (|scale| sqrt(var (M - 1)) + |beta|) >= max|lrelu(BN(y))|
 * * bound_mul over the batch (train-mode BN of M values; bound_mul = the
 * Dropout2d mask's maximum): the scale source of nsm_bn_act_h2 */
/* merge groups of `group` consecutive partial chunks ({sum, M2} rows of
 * rows_per_chunk rows) into ceil(nchunk/group) rows of rows_per_chunk*group
 * rows (Chan, fixed order): keeps nsm_bn_finalize_train short on huge grids */
int nsm_bn_partials_merge(const float* partial, int nchunk, int rows_per_chunk, int M, int C,
                          int group, float* out, void* stream);
int nsm_bn_finalize_eval(const float* run_mean, const float* run_var, const float* gamma,
                         const float* beta, int C, int c_real, float eps, float* mean,
                         float* invstd, float* scale, float* shift, void* stream);
/* out = lrelu(y*scale+shift, slope) (* mask[row / HW][c]) (+ res): BN apply +
 * LeakyReLU (Unetmodel.py:22-23,27-28), optionally Dropout2d (:24; mask NULL =
 * none), fused with the additive skip (Unetmodel.py:125,131,137) */
int nsm_bn_act(const void* y, int ldy, int M, int C, const float* scale, const float* shift,
               float slope, const float* mask, int HW, const void* res, int ldres, void* out,
               int ldo, int dtype, uint32_t* amax, void* stream);
/* nsm_bn_act (fp32, no skip) writing an h2 tensor out [M][2C] (float16; see
 * the pre-split operands above) with scale source `bound` (beta 1): the
 * activated 1x1 operand A1 of the fp32 train step (Unetmodel.py:22-24) */
int nsm_bn_act_h2(const float* y, int ldy, int M, int C, const float* scale, const float* shift,
                  float slope, const float* mask, int HW, void* out, const uint32_t* bound,
                  void* stream);
/* backward of  z = lrelu(mask * ... ) chains around a train-mode BN:
 *   dz = g * mask[b][c] * lrelu'(y*scale+shift); partial {sum dz, sum dz*xhat}. */
int nsm_bn_bwd_reduce(const void* g, int ldg, const void* y, int ldy, int M, int C, int HW,
                      const float* scale, const float* shift, float slope, const float* mask,
                      const float* mean, const float* invstd, float* partial, int nchunk,
                      int dtype, uint32_t* amax_k1dz, void* stream);
/* dgamma, dbeta (real channels), bias grad of the producing conv
 * (analytically 0 in train mode), coef[3][C] for nsm_bn_bwd_apply.
 * amax_k1dz (the reductions' optional slot: max|scale * dz| over the tensor)
 * and bound (may be NULL): the slot receiving max_c (max|k1 dz| + |k2|
 * sqrt(M - 1) / invstd + |k3|) >= max|dy| (Samuelson), the scale source of
 * nsm_bn_bwd_apply_h2. */
int nsm_bn_bwd_finalize(const float* partial, int nchunk, int M, int C, int c_real,
                        const float* gamma, const float* invstd, float* dgamma, float* dbeta,
                        float* dbias_prev, float* coef, const uint32_t* amax_k1dz,
                        uint32_t* bound, void* stream);
/* plain-sum merge: out[g][j] = sum of rows [g*group, (g+1)*group) of part[nrows][width]
 * (fixed order): the BN-backward partials of nsm_conv1x1_dgrad_bnbwd before
 * nsm_bn_bwd_finalize */
int nsm_sum_rows(const float* part, int nrows, int width, int group, float* out, void* stream);
/* dy = coef0*dz + coef1*(y-mean) + coef2 */
int nsm_bn_bwd_apply(const void* g, int ldg, const void* y, int ldy, int M, int C, int HW,
                     const float* scale, const float* shift, float slope, const float* mask,
                     const float* mean, const float* coef, void* dy, int lddy, int dtype,
                     uint32_t* amax, void* stream);
/* nsm_bn_bwd_apply (fp32) writing dy as an h2 tensor [M][2C] float16 with the
 * scale source bound (nsm_bn_bwd_finalize's): the 1x1 conv's output gradient
 * for its h2 weight / input gradients (nsm_conv1x1_wgrad_h2,
 * nsm_conv1x1_dgrad_bnbwd_h2) */
int nsm_bn_bwd_apply_h2(const float* g, int ldg, const float* y, int ldy, int M, int C, int HW,
                        const float* scale, const float* shift, float slope, const float* mask,
                        const float* mean, const float* coef, void* dy, const uint32_t* bound,
                        void* stream);
/* amax (bn_act, bn_bwd_apply; fp32 only, may be NULL): the operand-maximum
 * slot receiving max|out| / max|dy| for the f16x2 GEMM that consumes it. */

/* ---- resampling -------------------------------------------------------------
 * AvgPool2d(2) (Unetmodel.py:40,43,46): floor mode. bwd: dx = skip + dy/4. */
int nsm_avgpool2_fwd(const void* x, int B, int H, int W, int C, void* y, int dtype, void* stream);
int nsm_avgpool2_bwd_add(const void* dy, int B, int H, int W, int C, const void* skip, void* dx,
                         int dtype, void* stream);
/* bilinear, align_corners=True: nn.Upsample(x2) and _upsample_and_match
 * (Unetmodel.py:51-60,118-119). bwd is a deterministic gather. */
int nsm_resize_fwd(const void* x, int B, int Hi, int Wi, int C, void* y, int Ho, int Wo, int dtype,
                   void* stream);
int nsm_resize_bwd(const void* dy, int B, int Hi, int Wi, int C, void* dx, int Ho, int Wo,
                   int dtype, void* stream);

/* up x2 then resize to (th,tw) in one pass (Unetmodel.py:140-141: up9 then
 * _upsample_and_match back to the skip size); no 4x intermediate. */
/* The decoder's upsample of a block output that is never written: the source
 * taps are z = lrelu(y2*scale+shift) (+ res) (Unetmodel.py:27-28,125-137),
 * rounded as nsm_bn_act stores them; y2 = that block's second BN input, res
 * its skip [B*Hi*Wi][C] or NULL. nsm_up2_resize_fwd_act needs the row-blocked
 * composite (target width <= 2048, second step not upsizing). */
int nsm_resize_fwd_act(const void* y2, int B, int Hi, int Wi, int C, void* out, int Ho, int Wo,
                       const float* scale, const float* shift, float slope, const void* res,
                       int dtype, void* stream);
int nsm_up2_resize_fwd_act(const void* y2, int B, int h, int w, int C, void* out, int th, int tw,
                           const float* scale, const float* shift, float slope, const void* res,
                           int dtype, void* stream);
/* encoder block output z = lrelu(y*scale+shift) and AvgPool2d(2)(z) from one
 * read of y (Unetmodel.py:27-28,105,108,111) */
int nsm_bn_act_pool(const void* y, int B, int H, int W, int C, const float* scale,
                    const float* shift, float slope, void* z, void* pooled, int dtype,
                    uint32_t* amax, void* stream);
/* (nsm_bn_act_pool's amax: fp32, may be NULL — max|pooled|, the next Winograd
 * conv's h2 scale source) */
int nsm_up2_resize_fwd(const void* x, int B, int h, int w, int C, void* y, int th, int tw,
                       int dtype, void* stream);
int nsm_up2_resize_bwd(const void* dy, int B, int h, int w, int C, void* dx, int th, int tw,
                       int dtype, void* stream);
/* The same three gradient producers, also writing the BN-backward partials
 * {sum dz, sum dz*xhat} (nsm_bn_bwd_reduce's format, one row per kernel
 * block) of the block output they produce the gradient of: y2 = that block's
 * second BN input (Unetmodel.py:26-28), dz = g * lrelu'(y2*scale+shift), g
 * as written. partial[nchunk][2][C], nchunk = nsm_bnred_chunks(kind, ...)
 * (kind 0 avgpool2_bwd_add with H, W of dx; 1 resize_bwd with Hi, Wi; 2
 * up2_resize_bwd with h, w); 0 there = not available for this shape. */
int nsm_bnred_chunks(int kind, int B, int H, int W, int C);
int nsm_avgpool2_bwd_add_bnred(const void* dy, int B, int H, int W, int C, const void* skip,
                               void* dx, int dtype, const void* y2, const float* scale,
                               const float* shift, const float* mean, const float* invstd,
                               float slope, float* partial, uint32_t* amax_k1dz, void* stream);
int nsm_resize_bwd_bnred(const void* dy, int B, int Hi, int Wi, int C, void* dx, int Ho, int Wo,
                         int dtype, const void* y2, const float* scale, const float* shift,
                         const float* mean, const float* invstd, float slope, float* partial,
                         uint32_t* amax_k1dz, void* stream);
int nsm_up2_resize_bwd_bnred(const void* dy, int B, int h, int w, int C, void* dx, int th, int tw,
                             int dtype, const void* y2, const float* scale, const float* shift,
                             const float* mean, const float* invstd, float slope, float* partial,
                             uint32_t* amax_k1dz, void* stream);
/* amax_k1dz (may be NULL): slot receiving max|scale * dz| (nsm_bn_bwd_finalize's bound) */

/* ---- model boundary ---------------------------------------------------------
 * pixel_unshuffle(2) + NCHW->NHWC + channel pad (Unetmodel.py:65-67,101) */
int nsm_input_prep(const float* x, int B, int C, int H, int W, void* out, int cp, int dtype,
                   uint32_t* amax, void* stream);
/* (amax: fp32, may be NULL — max|out|, conv2's f16x2 operand scale) */
/* nsm_input_prep (fp32) writing X as an h2 tensor [B*H/2*W/2][2 cp]: its
 * scale source `amax` (zeroed by the caller) is first filled with max|x| over
 * the whole input by this call (X holds the same values) */
int nsm_input_prep_h2(const float* x, int B, int C, int H, int W, void* out, int cp, uint32_t* amax,
                      void* stream);
int nsm_input_grad(const void* dX, int B, int C, int H, int W, int cp, float* dx, int dtype,
                   void* stream);
/* conv10 1x1 16->4 + pixel_shuffle(2) + sigmoid (Unetmodel.py:63,143-148) */
int nsm_head_fwd(const void* z, int ldz, int B, int Rh, int Rw, const float* w10,
                 const float* b10, float* out, int dtype, void* stream);
int nsm_head_bwd_blocks(int B, int Rh, int Rw);
int nsm_head_bwd(const float* gout, const float* out, const void* z, int ldz, int B, int Rh,
                 int Rw, const float* w10, void* dz, float* partial, float* dw10, float* db10,
                 int dtype, void* stream);

/* ---- losses -----------------------------------------------------------------
 * nn.L1Loss (customLoss.py:96,134) scaled by alpha (customLoss.py:160);
 * bwd: grad = alpha * sign(o-t) / n * (*gscale) (+ grad if accumulate). */
int nsm_loss_blocks(int64_t n);
int nsm_l1_loss_fwd(const float* o, const float* t, int64_t n, float alpha, float* partial,
                    float* out, void* stream);
/* mean(exp(alpha*|a-b|) - 1): one frame pair of measure_temporal_instability
 * (pert_loss.py:170-199) */
int nsm_expdiff_mean(const float* a, const float* b, int64_t n, float alpha, float* partial,
                     float* out, void* stream);
int nsm_l1_loss_bwd(const float* o, const float* t, int64_t n, float alpha, const float* gscale,
                    float* grad, int accumulate, void* stream);
/* PerturbationLoss.perturb_input (pert_loss.py:26-59):
 * per-channel unbiased std over the batch of NCHW x -> std[C] */
int nsm_channel_std(const float* x, int B, int C, int H, int W, float* partial, float* std,
                    void* stream);
/* out = x + noise * std[c] * factor */
int nsm_perturb(const float* x, const float* noise, const float* std, int B, int C, int H,
                int W, float factor, float* out, void* stream);

/* ---- train-step tail (main.py:405,421: clip_grad_norm_ + AdamW) ----------- */
int nsm_sumsq(const float* g, int64_t n, float* partial, float* out, void* stream);
/* coef = inv_world * min(1, max_norm / (sqrt(sumsq)*inv_world + 1e-6)) */
int nsm_clip_coef(const float* sumsq, float inv_world, float max_norm, float* coef, void* stream);
int nsm_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                   float beta2, float eps, float weight_decay, int step, const float* gcoef,
                   void* stream);

/* ---- the reference's full step tail (main.py:287-423), no host sync ----------
 * The gradient is one flat fp32 buffer of the module's parameters in order;
 * seg_off[nseg+1] (device) delimits them. nsm_tail_plan (host) cuts the buffer
 * into blocks of nsm_tail_chunk() elements that never straddle a parameter:
 * blk_seg/blk_lo/blk_hi[nblk], seg_blk[nseg+1] (first block of each
 * parameter); call once with blk_seg == NULL to get nblk. Upload the arrays.
 * nsm_grad_tail, in place on g (the rank-sum of the DP all-reduce; inv_world
 * turns it into the mean first):
 *   NaN/Inf census; any parameter > 20 % invalid -> skip (main.py:295-317);
 *   else repair NaN -> mean + randn*std*0.1, Inf -> sign*max|valid|*10
 *   (:320-354; randn from `noise` if non-NULL, else a counter-based generator
 *   keyed by seed and the tail-call count step[1]); per-parameter clip to 1000*scale
 *   (:361-365); unscale by 1/scale (:368); per-parameter skip above 1e5,
 *   rescale to 1e3 above 1e3 (:383-397); clip_grad_norm_(max_norm) (:405);
 *   skip if a clipped norm > 10 (:408-418).
 *   Writes seg_coef[nseg][4] (pre-clip x unscale, 1e3 rescale, clip coef,
 *   zeroed), stat[4] (total norm, clip coef, max_norm, max clipped norm),
 *   flags[8] (skip, repaired, severe, nonfinite, huge, postclip, n_rescaled,
 *   n_zeroed), step[0] += !skip (AdamW steps taken) and step[1] += 1 (tail
 *   calls; `step` holds two ints). workspace: nsm_tail_ws_bytes().
 * nsm_adamw_tail: torch.optim.AdamW step (main.py:421, hyper-parameters
 *   main.py:955) with g scaled by seg_coef; a no-op when flags[0] is set; the
 *   bias corrections use the device step count. */
int64_t nsm_tail_chunk(void);
int nsm_tail_plan(const int64_t* seg_off, int nseg, int* blk_seg, int64_t* blk_lo,
                  int64_t* blk_hi, int* seg_blk, int cap);
size_t nsm_tail_ws_bytes(int nseg, int nblk);
int nsm_grad_tail(float* g, int nseg, const int64_t* seg_off, const int* seg_blk,
                  const int* blk_seg, const int64_t* blk_lo, const int64_t* blk_hi, int nblk,
                  float inv_world, float scale, float max_norm, const float* noise, uint64_t seed,
                  void* ws, size_t ws_bytes, float* seg_coef, float* stat, int* flags, int* step,
                  void* stream);
int nsm_adamw_tail(float* p, const float* g, float* m, float* v, const int* blk_seg,
                   const int64_t* blk_lo, const int64_t* blk_hi, int nblk, const float* seg_coef,
                   const int* flags, const int* step, double lr, double beta1, double beta2,
                   double eps, double weight_decay, void* stream);

/* ---- drop-in surface helpers ---------------------------------------------------
 * NCHW fp32 <-> NHWC [B*H*W][cp] (dtype NSM_F32 / NSM_BF16) for a standalone
 * DoubleConv call (Unetmodel.py:32-33); channels C..cp-1 are written as 0.
 * nsm_range_flag: flag[0] = 1 if any o[i] is outside [lo, hi] or NaN (the
 * `assert output.min() >= 0 and output.max() <= 1` of customLoss.py:131 /
 * pert_loss.py:131 as a sticky device flag; never writes 0). */
int nsm_nchw_to_nhwc(const float* x, int B, int C, int H, int W, void* y, int cp, int ldy,
                     int dtype, void* stream);
int nsm_nhwc_to_nchw(const void* z, int ldz, int B, int C, int H, int W, float* x, int dtype,
                     void* stream);
int nsm_range_flag(const float* o, int64_t n, float lo, float hi, int* flag, void* stream);
/* Dropout2d masks (Unetmodel.py:24,61) of all blocks of one forward in one
 * launch: job j writes out[off_j + b*cp_j + c] = (u < keep_j) / keep_j for
 * c < c_j and 0 for c_j <= c < cp_j, u ~ U[0,1) from a counter-based hash of
 * (seed, j, b, c). desc (device) = njobs x {off, c, cp, keep as float bits}. */
int nsm_dropout_masks(const int* desc, int njobs, int B, uint64_t seed, float* out, void* stream);
/* The same with the seed read from device memory (seed[0]): a HIP graph that
 * captures it draws new masks on every replay when the word is rewritten by a
 * captured producer (nsm_amd: torch's graph-safe generator). */
int nsm_dropout_masks_dev(const int* desc, int njobs, int B, const int64_t* seed, float* out,
                          void* stream);
/* Profiling marker: an empty kernel of (code + 1) workgroups of 64 lanes.
 * With NSM_STAGE_MARKS=1 the host brackets each encoder/decoder stage
 * (Unetmodel.py:104-148) with markers (code = stage id, 0 = stage end), so a
 * rocprofv3 PMC pass can attribute every dispatch to its stage
 * (tools/stage_pmc.py); never launched otherwise. */
int nsm_stage_mark(int code, void* stream);

/* ---- bf16 convolutions (BASELINE config 3) ---------------------------------
 * Same contracts as nsm_pack_conv_weight / nsm_conv_fwd_stats / nsm_conv_wgrad
 * with bf16 activations and packed weights (v_mfma_f32_32x32x16_bf16, fp32
 * accumulation). y = bf16(acc + bias); the fused BN partials are taken on the
 * rounded values (what BatchNorm reads under autocast); dw stays fp32. */
int nsm_pack_conv_weight_bf16(const float* w, int cout, int cin, int ksize, int cout_p, int cin_p,
                              int mode, void* out, void* stream);
int nsm_conv_fwd_bf16(const void* x, int ldx, int B, int H, int W, int cin_p, const void* wpk,
                      const float* bias, int cout_p, int ksize, void* y, int ldy,
                      const float* pro_scale, const float* pro_shift, const float* pro_mask,
                      float slope, float* stats, void* stream);
/* The 1x1 input gradient of a DoubleConv (dA1 = dY2 W2, Unetmodel.py:26) with
 * the backward of the first BN + LeakyReLU + Dropout2d (:22-24) in the GEMM
 * epilogue; y1 = that BN's input (Y1), scale/shift/mean/invstd its train-mode
 * vectors, mask [B][cip] or NULL, w2d the PACK_DGRAD layout of conv.4's weight.
 *   mode 0: partial[nchunk][2][cip] = {sum dz, sum dz*xhat} per chunk (the
 *           nsm_bn_bwd_reduce format; nchunk = nsm_conv1x1_bnbwd_chunks), dA1
 *           not written
 *   mode 1: mode 0 and dA1 written to out (then nsm_bn_bwd_apply)
 *   mode 2: out = dY1 = coef0*dz + coef1*(y1-mean) + coef2 (coef from
 *           nsm_bn_bwd_finalize); modes 0 + 2 run the GEMM twice so dA1 never
 *           reaches HBM.
 * amax_out (may be NULL): mode 2 (fp32) max|dY1| written; modes 0/1 (bf16)
 * max|scale * dz|, the k1 term of the dY1 bound nsm_bn_bwd_finalize derives
 * (the scale source of nsm_wino_dual_bn_f16).
 * Replaces ConvolutionBackward(conv.4) + BatchNorm/LeakyReLU/Dropout2d
 * backward of conv.1-3 (autograd of Unetmodel.py:21-26). dtype NSM_F32 | NSM_BF16 |
 * NSM_F16 (the 16-bit ones: dy2, w2d, y1, out in it). */
int nsm_conv1x1_dgrad_bnbwd(const void* dy2, int lddy2, int B, int H, int W, int cop,
                            const void* w2d, int cip, const void* y1, int ldy1,
                            const float* scale, const float* shift, const float* mean,
                            const float* invstd, const float* mask, float slope, int mode,
                            float* partial, const float* coef, void* out, int ldo, int dtype,
                            const uint32_t* amax_dy2, const uint32_t* amax_w,
                            uint32_t* amax_out, void* stream);
/* (amax_out: fp32 mode 2, may be NULL — max|dy| written, the h2 scale source
 * of its Winograd transforms) */
int nsm_conv1x1_bnbwd_chunks(int B, int H, int W, int cip, int cop, int dtype);
/* rows per BN-partial chunk of nsm_conv_fwd_bf16 (its M tile) */
/* Eval-mode DoubleConv half in one pass (Unetmodel.py:21-28 with BatchNorm on
 * its running statistics): y = lrelu(round(conv(x) + bias) * act_scale +
 * act_shift, slope) (+ res: the decoder's additive skip, :125-137), round =
 * the storage dtype's (the value the unfused conv -> bn_act pair stores in
 * between); act_scale / act_shift from nsm_bn_finalize_eval. dtype NSM_F32 |
 * NSM_BF16 | NSM_F16 (x, wpk, y, res in it). */
int nsm_conv_fwd_act(const void* x, int ldx, int B, int H, int W, int cin_p, const void* wpk,
                     const float* bias, int cout_p, int ksize, void* y, int ldy,
                     const float* act_scale, const float* act_shift, float slope, const void* res,
                     int ldres, int dtype, void* stream);
/* nsm_wino_output with the same eval BN + LeakyReLU (+ skip) on the way out */
int nsm_wino_output_act(const float* Mb, int B, int H, int W, int cout_p, int tile,
                        const float* bias, float* y, int ldy, const float* act_scale,
                        const float* act_shift, float slope, const float* res, int ldres,
                        void* stream);
int nsm_conv_stat_rows_bf16(int B, int H, int W, int cout_p);
size_t nsm_conv_wgrad_bf16_ws(int B, int H, int W, int cin_p, int cout_p, int ksize);
int nsm_conv_wgrad_bf16(const void* dy, int lddy, const void* x, int ldx, int B, int H, int W,
                        int cin_p, int cout_p, int ksize, const float* pro_scale,
                        const float* pro_shift, const float* pro_mask, float slope, float* ws,
                        size_t ws_floats, int cin, int cout, float* dw, void* stream);

/* ---- f16 convolutions (the reference's GPU precision, fp16 autocast:
 * main.py:257-259) ------------------------------------------------------------
 * The bf16 entries above on IEEE-half storage (v_mfma_f32_32x32x16_f16 /
 * 16x16x32_f16, fp32 accumulation; values rounded to nearest even, beyond
 * 65504 to +-Inf as in the reference's fp16 tensors): the same kernels,
 * compiled a second time with the f16 conversions (csrc/nsm_conv_s16.inc in
 * namespace nsm_h). BN-partial rows and the weight-gradient workspace:
 * nsm_conv_stat_rows_bf16 / nsm_conv_wgrad_bf16_ws (the tile plans are the
 * same). */
int nsm_pack_conv_weight_f16(const float* w, int cout, int cin, int ksize, int cout_p, int cin_p,
                             int mode, void* out, void* stream);
int nsm_conv_fwd_f16(const void* x, int ldx, int B, int H, int W, int cin_p, const void* wpk,
                     const float* bias, int cout_p, int ksize, void* y, int ldy,
                     const float* pro_scale, const float* pro_shift, const float* pro_mask,
                     float slope, float* stats, void* stream);
int nsm_conv_wgrad_f16(const void* dy, int lddy, const void* x, int ldx, int B, int H, int W,
                       int cin_p, int cout_p, int ksize, const float* pro_scale,
                       const float* pro_shift, const float* pro_mask, float slope, float* ws,
                       size_t ws_floats, int cin, int cout, float* dw, void* stream);

/* ---- VGG19 perceptual loss (customLoss.py:7-90, forward only) ------------
 * nsm_vgg_prep: out[2B*H*W][32] NHWC = (nan_to_num(clamp(v,0,1)) - mean)/denom
 * repeated into channels 0-2 (customLoss.py:44-62), images 0..B-1 from
 * `output`, B..2B-1 from `target` (both [B,1,H,W]); channels 3..31 zero.
 * nsm_maxpool2_fwd: nn.MaxPool2d(2,2) on NHWC [B*H*W][C] (VGG features 4,9,18,27). */
int nsm_vgg_prep(const float* output, const float* target, int B, int H, int W, float mean,
                 float denom, float* out, void* stream);
int nsm_maxpool2_fwd(const float* x, int B, int H, int W, int C, float* y, void* stream);

/* ---- frame loader (setdata.MmapLiverDataset's files) -----
 * nsm_npy_info: shape / dtype (0 f32, 1 f64) / data offset of an .npy file.
 * nsm_loader_create: mmap {split}_inputs.npy (f32 [N,C,H,W]) and
 *   {split}_labels.npy (f64|f32 [N,1,H,W]); this rank's contiguous shard
 *   [rank*N/world, (rank+1)*N/world) in order (DataLoader shuffle=False,
 *   main.py:850), batches of `batch` (last one short), cycling epochs; nthreads
 *   host threads stage upcoming batches into nslots pinned slots.
 * nsm_loader_next: async H2D of the next batch on `stream` into dev_x / dev_y
 *   (raw f32; labels converted on the host); returns the frame count or -1.
 * nsm_normalize_frames: x = (x - mean[c]) / (std[c] + eps) on the GPU
 *   (setdata.py:316). */
int nsm_npy_info(const char* path, int64_t* shape, int max_dims, int* ndim, int* dtype,
                 int64_t* data_offset);
void* nsm_loader_create(const char* inputs_path, const char* labels_path, int batch, int rank,
                        int world, int nslots, int nthreads);
int64_t nsm_loader_batches(void* loader);
int nsm_loader_frame_dims(void* loader, int* C, int* H, int* W);
int nsm_loader_next(void* loader, void* dev_x, void* dev_y, void* stream);
void nsm_loader_destroy(void* loader);
int nsm_normalize_frames(float* x, int B, int C, int64_t HW, const float* mean, const float* stdv,
                         float eps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NSM_H_ */
