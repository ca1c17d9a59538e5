"""Drop-in `Unet` / `DoubleConv` whose forward and backward run entirely on the
libnsm HIP kernels (MI355X / gfx950).

Surface parity with `/root/reference/Unetmodel.py`:
  * `DoubleConv(in_ch, out_ch, dropout_rate=0.2, dilation=1)` (:17-33) and
    `Unet(in_ch=4, out_ch=1, dropout_rate=0.2)` (:35-63) own the same
    sub-modules, so `state_dict()` keys/shapes/dtypes, `named_parameters()`
    order (66 tensors) and `named_modules()` match the reference exactly.
    The nn.Conv2d / nn.BatchNorm2d children are parameter holders only.
  * `forward(x[B,C,H,W]) -> [B,1,H-H%2,W-W%2]` in (0,1) (:90-149), including
    the odd-size bilinear guard, pixel_unshuffle, the conv5 checkpoint's
    double BN running-stat update (train + backward), the up9 blur
    (up x2 then resize back), additive skips, pixel_shuffle + sigmoid.
  * `rearrange_to_channels` / `reconstruct_from_channels` (:65-88).
  * `in_ch` generalises conv2 to 4*in_ch input channels (7-ch G-buffers).

Execution: one torch.autograd.Function per forward. Activations live in HBM
as NHWC fp32 `[pixels, channels padded to 32]`; every op is a libnsm kernel
launched on the current HIP stream (see DESIGN.md for the kernel list).
"""
import os
import warnings

import torch
import torch.distributed as dist
import torch.nn as nn

from . import ops, optim
from ._lib import call, ptr, require_gpu, stream
from . import prep
from .prep import H2_WINO, LazyBlockWeights, StepWeights

SLOPE = 0.2
# 3x3 convolutions with at least this many (padded) input channels use the
# Winograd F(m x m, 3x3) path for forward, input- and weight-gradient
# (MFMA-bound layers); NSM_WINOGRAD=0 disables it (direct implicit GEMM
# everywhere). The tile m of F(m x m, 3x3) per layer: wino_tile(); NSM_WINO_TILE=2/4/6
# forces one tile everywhere.
WINOGRAD_MIN_CHANNELS = (int(os.environ.get("NSM_WINO_MIN", "64"))
                         if os.environ.get("NSM_WINOGRAD", "1") != "0" else 1 << 30)
# NSM_ACT_POOL=0: the encoder block output and its AvgPool2d as two passes
# (bn_act, avgpool2) instead of one (ops.bn_act_pool)
ACT_POOL = os.environ.get("NSM_ACT_POOL", "1") != "0"
# NSM_LAZY_DECODER=1 (bf16): compute the decoder block outputs c5, merge6-8
# inside the next block's upsample (ops.Lazy) instead of materialising them.
# Off by default: B=64 bf16 A/B 1214 -> 1189 frames/s (the act-on-load upsample
# reads Y2 and the residual at every bilinear tap; conv9 stage +0.9 ms).
LAZY_DECODER = os.environ.get("NSM_LAZY_DECODER", "0") != "0"
# NSM_DUAL_WINO=0: the Winograd dgrad and wgrad transform the output gradient
# in two separate reads of it instead of one (nsm_wino_dual_input)
DUAL_TRANSFORM = os.environ.get("NSM_DUAL_WINO", "1") != "0"
# NSM_LAZY_DY1=1: the dual transform forms dY1 per element from dA1 and Y1
# (nsm_wino_dual_input_bn) instead of reading the dY1 nsm_bn_bwd_apply stored.
# Off: it saves the dY1 round trip but the F(6x6) kernel then issues 128
# loads per thread (two tensors over the overlapping 8x8 patches) and became
# issue-bound — conv7 apply 152 + dual 250 us -> fused 484 us, conv6 210 ->
# 260 us (only conv3 gained, 56 -> 48 us).
LAZY_DY1 = os.environ.get("NSM_LAZY_DY1", "0") != "0"
# NSM_LAZY_DY1_H2=0: on h2 Winograd operands, store dY1 (a second GEMM pass,
# or nsm_bn_bwd_apply) instead of forming it in the dual transform. There the
# F(6x6) BN-fused transform reads a block's pixel region once into LDS
# (wino_dual_bn_lds_kernel), which removes the issue bound above.
LAZY_DY1_H2 = os.environ.get("NSM_LAZY_DY1_H2", "1") != "0"
# NSM_WGRAD_F16=0: the bf16 path's F(4x4) layers take their weight gradient
# from the direct implicit GEMM instead of the Winograd domain (dM x V)
WGRAD_F16 = os.environ.get("NSM_WGRAD_F16", "1") != "0"
# NSM_BF16_DUAL=0: with WGRAD_F16, the bf16 output gradient's two F(4x4)
# transforms (the input gradient's V, the weight gradient's dM) by
# wino_input_f16 + wino_dout_f16 instead of from one read of dY1
# (ops.wino_dual_f16; B=64 step 1581 / 1586 -> 1596 / 1604 frames/s A/B)
BF16_DUAL = os.environ.get("NSM_BF16_DUAL", "1") != "0"
# NSM_LAZY_DY1_F16 (default 1): with BF16_DUAL, the bf16 F(4x4) layers' dY1
# formed per element inside the dual transform (ops.wino_dual_bn_f16, scale
# from the finalize's bound) instead of stored by nsm_bn_bwd_apply and read
# back. At 4 channels per thread that kernel ran at one wave per SIMD and lost
# (1572 / 1568 vs 1581 / 1580 frames/s); at 2 (BfLane<2>) it wins: B=64 step
# 1611.6 / 1628.0 / 1616.8 vs 1605.1 / 1609.2 / 1613.3 frames/s, A/B on one box
LAZY_DY1_F16 = os.environ.get("NSM_LAZY_DY1_F16", "1") != "0"
# NSM_EVAL_FUSED=0: eval forward with separate BN-apply passes instead of the
# BN + LeakyReLU (+ skip) in the conv epilogues (nsm_conv_fwd_act)
EVAL_FUSED = os.environ.get("NSM_EVAL_FUSED", "1") != "0"
# NSM_UP_WINO=0: materialise the decoder's x2-upsampled input of a Winograd
# conv (nsm_resize_fwd) instead of sampling it inside the input transform
UP_IN_WINO = os.environ.get("NSM_UP_WINO", "1") != "0"
# NSM_WINO_STATS=0: the BN statistics of the Winograd layers by a separate
# bn_stats pass instead of the output transform
WINO_BN_STATS = os.environ.get("NSM_WINO_STATS", "1") != "0"
_WINO_ENV = os.environ.get("NSM_WINO_TILE", "")
WINO_TILE = int(_WINO_ENV) if _WINO_ENV else 4   # the tile of the VGG stack


def wino_tile(cin_p, H, W):
    """F(m x m, 3x3) tile of a Winograd layer (cin_p channels at H x W).

    F(6x6) needs 64 GEMMs per 36 outputs, F(4x4) 36 per 16: F(6x6) when its
    MFMA work, tiling padding included, is below 0.9x F(4x4)'s (measured B=8
    7x512^2 fp32 step: conv6 5.67 -> 5.29 ms, conv7 6.02 -> 5.45, conv8 3.28 ->
    3.00, but conv5 at 32x32, where both tilings issue the same work, 0.86 ->
    0.93). Fwd, dgrad and wgrad of a layer share the tile (the wgrad reuses V).
    NSM_WINO_TILE=2/4/6 forces one tile."""
    if _WINO_ENV:
        return int(_WINO_ENV)
    f6 = 64 * -(-H // 6) * -(-W // 6)
    f4 = 36 * -(-H // 4) * -(-W // 4)
    return 6 if f6 < 0.9 * f4 else 4
# Materialise the activated 3x3 output A1 = lrelu(BN(Y1))*mask once (one
# streaming pass) so the 1x1 conv and its weight gradient run prologue-free on
# the LDS-DMA GEMMs, instead of re-applying BN+LReLU+mask in both operand
# loaders (bf16 +1.3 %, fp32 +1.2 % measured); NSM_BF16_ACT=0 / NSM_F32_ACT=0 keep
# the fused-prologue path.
BF16_MATERIALIZE_ACT = os.environ.get("NSM_BF16_ACT", "1") != "0"
F32_MATERIALIZE_ACT = os.environ.get("NSM_F32_ACT", "1") != "0"

# The backward of the first BN (+ LeakyReLU + Dropout2d) rides in the epilogue
# of the 1x1 input-gradient GEMM that produces its input gradient dA1
# (ops.conv1x1_dgrad_bn_bwd). NSM_BNB=0: separate reduce / apply passes
# everywhere; 1: the fused epilogue wherever it is used, storing dA1 + the
# partials (the reduce pass's dA1 read is gone); 2 (default): per layer, see
# bnb_mode.
BNB_MODE = int(os.environ.get("NSM_BNB", "2"))
# The output BN's backward reduction of blocks 2-8 rides in the kernel that
# produces their gradient (resize / pooling backward: ops.avgpool2_bwd_add,
# ops.resize_bwd, ops.up2_resize_bwd with bnred=); NSM_GRAD_BNRED=0 runs the
# separate nsm_bn_bwd_reduce pass instead
GRAD_BNRED = os.environ.get("NSM_GRAD_BNRED", "1") != "0"
# The weight-gradient launches of the Unet backward (GEMM, split reduce,
# Winograd weight-gradient output) run on a second stream: nothing on the
# input-gradient path reads them, so they fill its latency-bound launches and
# kernel tails. Under data parallelism each gradient bucket's all-reduce is
# issued from the side stream once it has caught up with the main one
# (_allreduce_bucket); NSM_WGRAD_STREAM=0 keeps one stream
# (also off under NSM_STAGE_MARKS: the per-stage counters attribute kernels by
# their order between the marker launches)
WGRAD_STREAM = (os.environ.get("NSM_WGRAD_STREAM", "1") != "0"
                and os.environ.get("NSM_STAGE_MARKS", "0") == "0")
# NSM_WGRAD_GRAPH_F32 (default 0): the side stream also inside a captured fp32
# step (GraphedTrainStep). Round 6, interleaved A/B on one box (3 rounds): fp32
# B=8 graph replay 753.2 / 755.0 / 756.3 frames/s without it vs 741.9 / 743.2 /
# 745.5 with it (the graph runs the weight-gradient branch concurrently and the
# co-scheduled kernels slow each other more than they gain), while the eager
# fp32 step gains from it (742.5-745.8 vs 728.3-733.1: it hides the host's
# launch gaps) and the bf16 B=64 step gains either way (graph 1627.9-1644.4 vs
# 1614.1-1629.4)
GRAPH_SIDE_F32 = int(os.environ.get("NSM_WGRAD_GRAPH_F32", "0"))
# NSM_WGRAD_PRIO: the side stream's priority (torch.cuda.Stream priority: lower
# numbers run first; 0 = the default streams')
WGRAD_PRIO = int(os.environ.get("NSM_WGRAD_PRIO", "0"))
_wg_stream = None      # the side stream while a Unet backward runs, else None
_wg_streams = {}       # one side stream per device
# The tensors the queued side-stream launches read, held (not freed) until the
# main stream has waited for those launches: [(event recorded on the side
# stream after them, tensors, bytes)], oldest first. Once the held bytes
# exceed NSM_WGRAD_HOLD_GB the oldest entries are released, each after the
# main stream waits for its event (a launch or two behind the side stream's
# tail, so the wait rarely stalls it).
#
# Not record_stream: a block recorded on another stream returns to the
# allocator only when the allocator, at a later malloc, finds that stream's
# event complete. An eager loop whose host runs ahead of the GPU then finds
# none complete and takes fresh device memory every step — the B=64 bf16
# eager step's reserved memory grew 5.9-9.7 GB per step, and once hipMalloc
# slowed (2.97 s inside one conv7 backward) the stage averaged 266-278 ms
# (tools/eager_probe.py --bench; DESIGN.md "The eager-step stall").
WGRAD_HOLD_BYTES = int(float(os.environ.get("NSM_WGRAD_HOLD_GB", "8")) * (1 << 30))
_wg_hold = []


def reserve_side_stream(device=None):
    """Create the weight-gradient side stream of `device` and bind it, and the
    current stream, to hardware queues now (one small launch on each). HIP binds
    a stream at its first launch to the least used of GPU_MAX_HW_QUEUES queues;
    RCCL's and ProcessGroupNCCL's streams, created by init_process_group, would
    otherwise take the free queues first and leave the side stream on the
    current stream's queue, serialised with it (the eager DP step at world size
    1: side and main kernels on one queue even at 8 queues, round-6 trace). Call
    it before torch.distributed.init_process_group."""
    dev = (torch.device(device) if device is not None
           else torch.device("cuda", torch.cuda.current_device()))
    s = _wg_streams.get(dev)
    if s is None:
        s = _wg_streams[dev] = torch.cuda.Stream(device=dev, priority=WGRAD_PRIO)
    buf = torch.empty(64, dtype=torch.int32, device=dev)
    call("nsm_zero_u32", ptr(buf), buf.numel(), stream())
    with torch.cuda.stream(s):
        call("nsm_zero_u32", ptr(buf), buf.numel(), stream())
    torch.cuda.synchronize(dev)
    return s


def _allreduce_bucket(flat, lo, hi, group):
    """Start the bucket's gradient all-reduce once both the current stream's
    work so far (biases, BN parameters) and the weight gradients queued on the
    side stream are done, WITHOUT making the current stream wait: the call is
    issued from the side stream after it has waited for the current one, so
    RCCL's stream waits on the side stream only and the encoder backward goes
    on (a join of the current stream here held it until the decoder's weight
    gradients were done). The eager DP step's remaining gap to the step without
    DP was the hardware-queue binding, not this (bench.py GPU_MAX_HW_QUEUES)."""
    side = _wg_stream
    if side is None:
        optim.allreduce_async(flat, lo, hi, group)
        return
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        optim.allreduce_async(flat, lo, hi, group)


def _wgrad(fn, *reads):
    """Run fn (weight-gradient launches) on the side stream after everything
    queued so far on the current stream. The tensors it reads stay referenced
    until the current stream has waited for it (_wg_hold), so their memory is
    never handed to a later launch on the current stream before fn's kernels
    have read it."""
    side = _wg_stream
    if side is None:
        fn()
        return
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        fn()
    ev = torch.cuda.Event()
    ev.record(side)
    ts = [t for t in reads if isinstance(t, torch.Tensor)]
    _wg_hold.append((ev, ts, sum(t.untyped_storage().nbytes() for t in ts)))
    held = sum(h[2] for h in _wg_hold)
    while held > WGRAD_HOLD_BYTES and len(_wg_hold) > 1:
        e, _, nb = _wg_hold.pop(0)
        cur.wait_event(e)
        held -= nb


def bnb_mode(cip, cop, dtype, h2=False):
    """0: conv_fwd + bn_bwd; 1: fused epilogue storing dA1, then bn_bwd_apply;
    2: fused epilogue twice (partials, then dY1; dA1 never stored) where the
    HBM bytes saved, (2*cip - cop) elements per pixel, outweigh the second
    pass's 2*cip*cop MFMA FLOPs (at ~5 TB/s and ~0.6 PF bf16 / ~0.12 PF fp32 for
    these K <= 512 GEMMs). bf16 keeps the separate passes where the GEMM is
    not an LDS-DMA tile with N >= 128 (conv2/conv3/conv9): one 92-160 KB block
    per CU leaves the epilogue's loads exposed there (measured: conv9 782 ->
    892 us, conv2 462 -> 533 us fused), while conv6/7/8 gain 77-170 us each."""
    if BNB_MODE == 0:
        return 0
    if dtype in ops.S16 and (cop % 64 or cip < 128):
        return 0 if BNB_MODE == 2 else 1
    if BNB_MODE == 1:
        return 1
    # fp32-product rate of the pass: bf16 ~0.6 PF; fp32 register-path f16x2
    # split ~0.12 PF; fp32 on h2 operands (nsm_conv_h2d.inc) ~1 PF of f16 MFMA
    # work = ~0.3 PF of fp32 products
    s, rate = (2, 6e14) if dtype in ops.S16 else (4, 3e14 if h2 else 1.2e14)
    return 2 if (2 * cip - cop) * s / 5e12 > 2 * cip * cop / rate else 1
ENCODER = (2, 3, 4, 5)
DECODER = (6, 7, 8, 9)
SKIP_OF = {6: 4, 7: 3, 8: 2}          # merge_k = conv_k(...) + c_skip  (Unetmodel.py:125,131,137)
POOL_SKIP = {4: 6, 3: 7, 2: 8}        # c_k feeds pool_k and decoder merge (6,7,8)


_WARNED = set()


def _warn_once(key, msg):
    if key not in _WARNED:
        _WARNED.add(key)
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def _storage_dtype(dtype):
    """Activation storage of a compute dtype: fp32, bf16, or ops.F16S (IEEE
    half bits in int16) for torch.float16."""
    return ops.F16S if dtype == torch.float16 else dtype


def _autocast_dtype():
    """The storage dtype a torch.autocast('cuda') region asks for: bf16 under
    bf16 autocast; f16 under fp16 autocast (the reference's own GPU mode,
    main.py:257-259: direct convolutions on f16 operands, f16 activations and
    activation gradients, fp32 accumulation / BN statistics / parameters /
    weight gradients); fp32 outside autocast."""
    if torch.is_autocast_enabled("cuda"):
        adt = torch.get_autocast_dtype("cuda")
        if adt in (torch.bfloat16, torch.float16):
            return _storage_dtype(adt)
    return torch.float32


def _nhwc(x, cp, dtype):
    """NCHW [B,C,H,W] -> NHWC 2-D [B*H*W, cp] in `dtype` (zero-padded channels)."""
    B, C, H, W = x.shape
    x = x.detach().to(torch.float32).contiguous()
    out = torch.empty(B * H * W, cp, dtype=dtype, device=x.device)
    call("nsm_nchw_to_nhwc", ptr(x), B, C, H, W, ptr(out), cp, cp, ops.dt(out), stream())
    return out


def _nchw(z, B, C, H, W):
    """NHWC 2-D [B*H*W, ld] -> fp32 NCHW [B,C,H,W] (first C channels)."""
    out = torch.empty(B, C, H, W, dtype=torch.float32, device=z.device)
    call("nsm_nhwc_to_nchw", ptr(z), z.stride(0), B, C, H, W, ptr(out), ops.dt(z), stream())
    return out


def _dropout_mask(p, B, ci, device):
    """ATen feature dropout (Unetmodel.py:24): bernoulli(1-p) / (1-p) per (n, c),
    padded to the NHWC channel count with zeros."""
    m = torch.empty(B, ci, device=device).bernoulli_(1 - p).div_(1 - p)
    cp = ops.pad32(ci)
    if cp != ci:
        m = torch.nn.functional.pad(m, (0, cp - ci))
    return m.contiguous()


class _DoubleConvFn(torch.autograd.Function):
    """A DoubleConv called on its own (Unetmodel.py:32-33) on the same fused
    kernels the Unet uses: NCHW in, NCHW out, BN running stats updated in
    train mode, the backward writes all 8 parameter gradients."""

    @staticmethod
    def forward(ctx, x, blk, *params):
        B, C, H, W = x.shape
        ci, co = blk.conv[0].in_channels, blk.conv[4].out_channels
        if C != ci:
            raise ValueError(f"DoubleConv expects {ci} channels, got {C}")
        training = blk.training
        dtype = _autocast_dtype()
        X = _nhwc(x, ops.pad32(ci), dtype)
        p = blk.conv[3].p
        mask = _dropout_mask(p, B, ci, x.device) if training and p > 0 else None
        s = _block_fwd(blk, X, B, H, W, training, mask, "doubleconv")
        z = ops.bn_act(s.Y2, s.bn2, SLOPE)
        ctx.blk, ctx.s, ctx.shape, ctx.training = blk, s, (B, C, H, W), training
        ctx.params = params
        out = _nchw(z, B, co, H, W)
        if dtype == torch.float32:
            return out
        return out.to(torch.float16 if dtype == ops.F16S else dtype)

    @staticmethod
    def backward(ctx, gout):
        if not ctx.training:
            raise RuntimeError("nsm_amd DoubleConv backward is implemented for train mode")
        blk, s = ctx.blk, ctx.s
        B, C, H, W = ctx.shape
        G = _nhwc(gout, s.cop, s.Y2.dtype)
        grads = {p: torch.empty_like(p) for p in ctx.params}
        dX = _block_bwd(blk, s, G, grads, True, "doubleconv")
        ctx.s = None
        dx = _nchw(dX, B, C, H, W) if ctx.needs_input_grad[0] else None
        return (dx, None) + tuple(grads[p] for p in ctx.params)


class DoubleConv(nn.Module):
    """The reference's DoubleConv (Unetmodel.py:17-33): same sub-modules and
    state_dict layout. Inside `Unet` the blocks are run by the fused Unet
    path; called on its own, forward runs `_DoubleConvFn` on the same kernels."""

    def __init__(self, in_ch, out_ch, dropout_rate=0.2, dilation=1):
        super().__init__()
        self.in_ch, self.out_ch, self.dropout_rate = in_ch, out_ch, dropout_rate
        self.conv = nn.Sequential(
            nn.Conv2d(in_ch, in_ch, 3, padding=1),
            nn.BatchNorm2d(in_ch, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True),
            nn.LeakyReLU(SLOPE, inplace=False),
            nn.Dropout2d(p=dropout_rate),
            nn.Conv2d(in_ch, out_ch, 1),
            nn.BatchNorm2d(out_ch, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True),
            nn.LeakyReLU(SLOPE, inplace=False),
        )

    def forward(self, x):
        require_gpu(x, "DoubleConv input")
        return _DoubleConvFn.apply(x, self, *tuple(self.parameters()))


class Unet(nn.Module):
    def __init__(self, in_ch=4, out_ch=1, dropout_rate=0.2):
        super().__init__()
        self.in_ch = in_ch
        self.conv2 = DoubleConv(4 * in_ch, 64, dropout_rate)
        self.pool2 = nn.AvgPool2d(2)
        self.conv3 = DoubleConv(64, 128, dropout_rate, dilation=2)
        self.pool3 = nn.AvgPool2d(2)
        self.conv4 = DoubleConv(128, 512, dropout_rate, dilation=4)
        self.pool4 = nn.AvgPool2d(2)
        self.conv5 = DoubleConv(512, 1024, dropout_rate)
        self.up6 = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv6 = DoubleConv(1024, 512, dropout_rate)
        self.up7 = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv7 = DoubleConv(512, 128, dropout_rate)
        self.up8 = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv8 = DoubleConv(128, 64, dropout_rate)
        self.up9 = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        self.conv9 = DoubleConv(64, 16, dropout_rate / 2)
        self.conv10 = nn.Conv2d(16, 4, 1)
        # parity hook: {k: [B, C_in(k)] scaled masks} consumed by the next forward
        self._inject_masks = None
        # when True, conv5's BNs get the reference's checkpoint-recompute update in backward
        self.emulate_checkpoint_bn = True
        # data parallel: (group,) when the backward launches its own grad all-reduces
        self._grad_allreduce = None
        # data parallel: (group, src) when forward broadcasts rank 0's BN buffers
        self._bn_broadcast = None
        self._bn_flat_cache = None
        # activation storage / MFMA dtype: None = fp32, or bf16 / f16 inside a
        # torch.autocast(dtype=torch.bfloat16 / float16) region; set_compute_dtype() pins it
        self.compute_dtype = None

    def set_compute_dtype(self, dtype):
        """torch.float32 (exact fp32 MFMA, Winograd for the deep convs),
        torch.bfloat16 (BASELINE config 3: bf16 activations and MFMA products,
        fp32 accumulation / BN statistics / parameters / gradients) or
        torch.float16 (the reference's fp16-autocast mode, main.py:257-259:
        direct convolutions on f16 operands, f16 activations and activation
        gradients, the same fp32 accumulation and state)."""
        if dtype not in (None, torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f"unsupported compute dtype {dtype}")
        self.compute_dtype = dtype
        return self

    def activation_dtype(self):
        """Storage dtype of the activations: fp32, bf16 or ops.F16S."""
        if self.compute_dtype is not None:
            return _storage_dtype(self.compute_dtype)
        return _autocast_dtype()

    def overlap_grad_allreduce(self, group=None, enable=True):
        """Data-parallel overlap: the backward starts the RCCL
        all-reduce of the decoder+head gradient bucket (conv6..conv10, 80 % of
        the 60 MiB, contiguous at the end of the flat buffer) as soon as the
        decoder backward is queued, so it runs on RCCL's stream under the
        encoder backward; the encoder bucket follows at the end.
        nsm_amd.allreduce_grads() then only waits for them."""
        self._grad_allreduce = (group,) if enable else None
        return self

    def data_parallel(self, group=None, overlap=True, broadcast_buffers=True):
        """Plain DP semantics (DDP's defaults): the gradient
        all-reduce overlapped with the backward, and rank 0's BatchNorm running
        statistics broadcast to every rank at the start of each train-mode
        forward (DDP broadcast_buffers=True), so all ranks — and rank 0's
        checkpoint — carry the same buffers."""
        self.overlap_grad_allreduce(group, overlap)
        if broadcast_buffers:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            self._bn_broadcast = (group, src)
        else:
            self._bn_broadcast = None
        return self

    def _bn_flat(self):
        """All BN running_mean/running_var as views of ONE fp32 buffer and all
        num_batches_tracked as views of ONE int64 buffer (re-homed when a
        `.to()` or assignment replaced them), so the DP broadcast is two calls."""
        bns = [m for m in self.modules() if isinstance(m, nn.BatchNorm2d) and m.track_running_stats]
        cache = self._bn_flat_cache
        if cache is not None:
            f, i = cache
            fp, ip = f.untyped_storage().data_ptr(), i.untyped_storage().data_ptr()
            if all(b.running_mean.untyped_storage().data_ptr() == fp
                   and b.running_var.untyped_storage().data_ptr() == fp
                   and b.num_batches_tracked.untyped_storage().data_ptr() == ip for b in bns):
                return cache
        with torch.no_grad():
            f = torch.cat([t.reshape(-1) for b in bns for t in (b.running_mean, b.running_var)])
            i = torch.stack([b.num_batches_tracked.reshape(()) for b in bns])
            off = 0
            for k, b in enumerate(bns):
                n = b.running_mean.numel()
                b.running_mean = f[off:off + n]
                b.running_var = f[off + n:off + 2 * n]
                b.num_batches_tracked = i[k]
                off += 2 * n
        self._bn_flat_cache = (f, i)
        return self._bn_flat_cache

    def broadcast_buffers(self, src=0, group=None):
        """Overwrite every rank's BN buffers with rank `src`'s (two collectives)."""
        f, i = self._bn_flat()
        dist.broadcast(f, src, group=group)
        dist.broadcast(i, src, group=group)

    # reference helpers (Unetmodel.py:65-88)
    def rearrange_to_channels(self, x):
        return torch.nn.functional.pixel_unshuffle(x, 2)

    def reconstruct_from_channels(self, x):
        return torch.nn.functional.pixel_shuffle(x, 2)

    def block(self, k):
        return getattr(self, f"conv{k}")

    def forward(self, x):
        require_gpu(x, "Unet input")
        params = tuple(self.parameters())
        for p in params[:1]:
            require_gpu(p, "Unet parameters")
        if "hooks" not in _WARNED and any(m._backward_hooks or m._backward_pre_hooks
                                          for m in self.modules() if m is not self):
            # main.py:207-222 registers a logging hook on every leaf module
            _warn_once("hooks", "nsm_amd.Unet: backward hooks on sub-modules are not invoked by "
                       "the fused Unet path (the reference's main.py:207-222 hooks only log "
                       "NaN/Inf/norms); FlatAdamW(sanitize=True).last_flags() reports the "
                       "step tail's NaN/Inf/norm decisions instead")
        if self._bn_broadcast is not None and self.training:
            group, src = self._bn_broadcast
            with ops.stage("dp.bn_broadcast"):   # timed by bench.py at N > 1
                self.broadcast_buffers(src, group)
        return _UnetFn.apply(x, self, *params)


# ---------------------------------------------------------------------------
# forward / backward orchestration
# ---------------------------------------------------------------------------
def _masks_for(mod, B, device, training):
    """[B, C_in_padded] Dropout2d masks of the blocks with p > 0: injected ones
    (parity), else all drawn in ONE nsm_dropout_masks launch seeded from torch's
    default CPU generator (so torch.manual_seed makes them reproducible).
    Returns (masks, their maxima) — a mask's maximum bounds the activated 1x1
    operand (bn_train(bound=...)): 1/(1-p) for drawn masks."""
    masks, mmax = {}, {}
    inj = mod._inject_masks
    mod._inject_masks = None
    jobs = []
    for k in ENCODER + DECODER:
        blk = mod.block(k)
        p = blk.conv[3].p
        if not training or p == 0:
            continue
        ci = blk.conv[0].in_channels
        cp = ops.pad32(ci)
        if inj is not None and k in inj:
            mmax[k] = float(inj[k].abs().max())   # parity hook (tests): host value
            m = inj[k].to(device=device, dtype=torch.float32).reshape(B, ci)
            if cp != ci:
                m = torch.nn.functional.pad(m, (0, cp - ci))
            masks[k] = m.contiguous()
        else:
            jobs.append((k, ci, cp, 1.0 - p))
    if jobs:
        import struct
        desc, off = [], 0
        for k, ci, cp, keep in jobs:
            fb = struct.unpack("<i", struct.pack("<f", keep))[0]
            desc += [off, ci, cp, fb]
            off += B * cp
        flat = torch.empty(off, dtype=torch.float32, device=device)
        # the descriptor depends only on (B, blocks): uploaded once, then cached
        # (a per-forward H2D copy from pageable memory would synchronise the host)
        key = (B, str(device), tuple(desc))
        cache = mod.__dict__.setdefault("_mask_desc", {})
        dev_desc = cache.get(key)
        if dev_desc is None:
            dev_desc = cache[key] = torch.tensor(desc, dtype=torch.int32).to(device)
        if torch.cuda.is_current_stream_capturing():
            # a captured step (GraphedTrainStep): the seed drawn on the device by
            # torch's graph-safe generator, so every replay draws new masks
            seed_t = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=device)
            call("nsm_dropout_masks_dev", ptr(dev_desc), len(jobs), B, ptr(seed_t), ptr(flat),
                 stream())
        else:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            call("nsm_dropout_masks", ptr(dev_desc), len(jobs), B, seed, ptr(flat), stream())
        off = 0
        for k, ci, cp, keep in jobs:
            masks[k] = flat[off:off + B * cp].view(B, cp)
            mmax[k] = 1.0 / keep
            off += B * cp
    return masks, mmax


class _BlockSaved:
    __slots__ = ("X", "Y1", "Y2", "bn1", "bn2", "mask", "B", "H", "W", "cip", "cop", "V", "A1",
                 "pw", "Z", "am", "Vf16")


# a block's operand-maximum slots (the f16x2 GEMMs' operand scales, filled by
# the operands' producers): Winograd V, Vd, dM; the 1x1 conv's A1 and dY2; the
# scale sources of the pre-split (h2) Winograd operands: the block input X
# (written by the previous block's output pass) and dY1
# (h2 1x1 operands: AM_A1 holds the bound of A1 from its BN finalize, AM_K1DZ
# max|k1 dz| of the output BN's backward, AM_DY2B the bound of dY2 derived from it)
AM_V, AM_VD, AM_DM, AM_A1, AM_DY2, AM_X, AM_DY1, AM_K1DZ, AM_DY2B = range(9)
# (the direct 3x3 on h2 operands: AM_K1DZ1 max|k1 dz| of the first BN's
# backward, AM_DY1B the bound of the h2 dY1 derived from it)
AM_K1DZ1, AM_DY1B = 9, 10
AM_PER_BLOCK = 11


def _slot(am, i):
    """Slot i of a block's operand-maximum slots, or None."""
    return ops.amax_slot(am, i)


def _block_slots(amax, k):
    """Block k's operand-maximum slots of the step's buffer, or None."""
    w = ops.AMAX_WORDS * AM_PER_BLOCK
    return None if amax is None else amax[k * w:(k + 1) * w]


def _x_slot(amax, k):
    """Block k's input-maximum slot (AM_X), filled by the pass that writes
    block k's input (or the tensor it is resampled from), or None."""
    return _slot(_block_slots(amax, k), AM_X)


def _is_h2(U):
    return U is not None and U.dtype == ops.H2


def fuses_resize(blk, dtype, training=True):
    """True when the block's 3x3 conv runs on Winograd and can sample the
    decoder's x2 upsample inside its input transform (UP_IN_WINO): the fp32
    layers from WINOGRAD_MIN_CHANNELS, the bf16 path's F(4x4) f16 layers
    (prep.bf16_wino; nsm_wino_input_f16_resize)."""
    cip = ops.pad32(blk.conv[0].in_channels)
    if not UP_IN_WINO:
        return False
    if dtype == torch.float32:
        return cip >= WINOGRAD_MIN_CHANNELS
    # (bf16 training: the weight gradient must come from the kept V, as the
    # block input itself is never materialised)
    return PREP_BATCH and prep.bf16_wino(cip, dtype, training) and (WGRAD_F16 or not training)


def _block_eval_fused(blk, xin, B, H, W, pw, name, src_hw, res, am=None):
    """Eval: both convs with BN (running statistics) + LeakyReLU (+ the skip
    add) in their epilogues — nothing but A1 and the block output is stored."""
    c0, bn1m, c4, bn2m = blk.conv[0], blk.conv[1], blk.conv[4], blk.conv[5]
    ci, co = c0.in_channels, c4.out_channels
    cip, cop = ops.pad32(ci), ops.pad32(co)
    dtype = xin.dtype
    bn1 = _bn_eval(bn1m, cip, ci, bn1m.eps, xin.device, pw.vec("g1"), pw.vec("be1"))
    b1 = pw.vec("b1")
    if cip >= WINOGRAD_MIN_CHANNELS and dtype == torch.float32:
        tile = wino_tile(cip, H, W)
        A1 = ops.conv3x3_wino(xin, B, H, W, pw.U1(tile, False), b1, cip, tile=tile,
                              tag=name + ".conv.0.fwd", src_hw=src_hw, act=(bn1, None),
                              amax_v=_slot(am, AM_V), amax_u=pw.amax_U1(False))
    elif _has_f16_u(pw) and am is not None:
        # bf16 eval: Winograd F(4x4) on f16 operands, BN + LeakyReLU in the
        # output transform; the V scale from max|x| (the fused epilogues that
        # wrote x record none; with src_hw, x is the source of the decoder's
        # upsample the input transform samples, and bounds it)
        ops.absmax(xin, _slot(am, AM_X))
        A1 = ops.conv3x3_wino_f16(xin, B, H, W, pw.Uf16(), b1, cip,
                                  amax=(_slot(am, AM_X), pw.amax_Uf16()), stats=False,
                                  tag=name + ".conv.0.fwd", act=bn1, src_hw=src_hw)[0]
    else:
        assert src_hw is None
        A1 = ops.conv_fwd_act(xin, B, H, W, pw.w1(ops.PACK_FWD), b1, cip, 3, bn1, slope=SLOPE,
                              tag=name + ".conv.0.fwd")
    bn2 = _bn_eval(bn2m, cop, co, bn2m.eps, xin.device, pw.vec("g2"), pw.vec("be2"))
    Z = ops.conv_fwd_act(A1, B, H, W, pw.w2(ops.PACK_FWD), pw.vec("b2"), cop, 1, bn2, res=res,
                         slope=SLOPE, tag=name + ".conv.4.fwd")
    s = _BlockSaved()
    s.X = s.Y1 = s.Y2 = s.mask = s.V = s.A1 = s.Vf16 = None
    s.bn1, s.bn2, s.pw, s.Z = bn1, bn2, pw, Z
    s.B, s.H, s.W, s.cip, s.cop = B, H, W, cip, cop
    s.am = am
    return s


def _block_fwd(blk, X, B, H, W, training, mask, name="", pw=None, src=None, fuse_out=False,
               res=None, am=None, mask_max=1.0):
    """pw: the block's weight layouts (prep.StepWeights.block, all written by the
    step's single preparation launch), or None to build them here per call.
    src=(x_low, hi, wi): X is the bilinear resize of x_low to H x W, sampled
    inside the Winograd input transform (X is None then; fuses_resize).
    fuse_out (eval, EVAL_FUSED): the block output lrelu(bn2(Y2)) (+ res) is
    produced by the convs' epilogues, returned as s.Z (Y1/Y2 not stored).
    am: the block's zeroed operand-maximum slots (AM_*: the f16x2 GEMMs'
    operand scales), or None (bf16 split). mask_max: the maximum of `mask` (the
    bound of the h2 activated operand, bn_train(bound=...))."""
    c0, bn1m, c4, bn2m = blk.conv[0], blk.conv[1], blk.conv[4], blk.conv[5]
    ci, co = c0.in_channels, c4.out_channels
    cip, cop = ops.pad32(ci), ops.pad32(co)
    xin = X if src is None else src[0]
    src_hw = None if src is None else (src[1], src[2])
    assert xin.shape[1] == (2 * cip if xin.dtype == ops.H2 else cip), (xin.shape, cip)
    assert src is None or fuses_resize(blk, xin.dtype, training)
    dtype = xin.dtype
    if pw is None:
        pw = LazyBlockWeights(blk, dtype)
    if fuse_out and not training and EVAL_FUSED:
        return _block_eval_fused(blk, xin, B, H, W, pw, name, src_hw, res, am)
    b1 = pw.vec("b1")
    V = Vf16 = None
    if cip >= WINOGRAD_MIN_CHANNELS and dtype == torch.float32:
        tile = wino_tile(cip, H, W)
        U1 = pw.U1(tile, False)
        # h2 U: V is written pre-split, scaled from max|X| (AM_X)
        am_v = _slot(am, AM_X if _is_h2(U1) else AM_V)
        part1 = None
        if training and WINO_BN_STATS:
            # the output transform also writes the BN batch-statistics partials
            Y1, V, part1 = ops.conv3x3_wino(xin, B, H, W, U1, b1, cip, tile=tile,
                                            tag=name + ".conv.0.fwd", keep_v=True, stats=True,
                                            src_hw=src_hw, amax_v=am_v,
                                            amax_u=pw.amax_U1(False))
        else:
            Y1, V = ops.conv3x3_wino(xin, B, H, W, U1, b1, cip, tile=tile,
                                     tag=name + ".conv.0.fwd", keep_v=True, src_hw=src_hw,
                                     amax_v=am_v, amax_u=pw.amax_U1(False))
        if training and part1 is None:
            part1 = ops.bn_partials(Y1)
    elif _has_f16_u(pw):
        # bf16: Winograd F(4x4) forward on single-plane scaled f16 operands
        # (src: the decoder's x2 upsample sampled by the input transform)
        keep = WGRAD_F16 and training
        r = ops.conv3x3_wino_f16(xin, B, H, W, pw.Uf16(), b1, cip,
                                 amax=(_slot(am, AM_X), pw.amax_Uf16()), stats=training,
                                 tag=name + ".conv.0.fwd", keep_v=keep, src_hw=src_hw)
        Y1, part1 = r[0], r[1]
        Vf16 = r[2] if keep else None
        if training and part1 is None:
            part1 = ops.bn_partials(Y1)
    else:
        w1 = pw.w1(ops.PACK_FWD)
        if w1.dtype == ops.H2:   # h2 operands (X from input_prep_h2; csrc/nsm_conv_h2d.inc)
            assert X.dtype == ops.H2
            Y1, part1 = ops.conv3x3_h2(X, B, H, W, w1, b1, cip, stats=training,
                                       amax=(_slot(am, AM_X), pw.amax_w1(ops.PACK_FWD)),
                                       tag=name + ".conv.0.fwd")
        else:
            Y1, part1 = ops.conv_fwd_bn(X, B, H, W, w1, b1, cip, 3, tag=name + ".conv.0.fwd",
                                        stats=training,
                                        amax=(_slot(am, AM_X), pw.amax_w1(ops.PACK_FWD)))
    eps1, eps2 = bn1m.eps, bn2m.eps
    w2 = pw.w2(ops.PACK_FWD)
    b2 = pw.vec("b2")
    # h2 1x1 operands (fp32 training, csrc/nsm_conv_h2d.inc): A1 written by
    # bn_act_h2, scaled from the bound the BN finalize records in AM_A1
    h2x = training and w2.dtype == ops.H2
    if training:
        bn1 = ops.bn_train(Y1, bn1m, ci, bn1m.momentum, eps1, part=part1, gamma=pw.vec("g1"),
                           beta=pw.vec("be1"),
                           bound=(_slot(am, AM_A1), mask_max if mask is not None else 1.0)
                           if h2x else None)
    else:
        bn1 = _bn_eval(bn1m, cip, ci, eps1, xin.device, pw.vec("g1"), pw.vec("be1"))
    A1 = None
    if h2x:
        A1 = ops.bn_act_h2(Y1, bn1, SLOPE, mask=mask, HW=H * W, bound=_slot(am, AM_A1))
        Y2, part2 = ops.conv1x1_h2(A1, w2, b2, cop, stats=True,
                                   amax=(_slot(am, AM_A1), pw.amax_w2(ops.PACK_FWD)),
                                   tag=name + ".conv.4.fwd")
    elif BF16_MATERIALIZE_ACT if dtype in ops.S16 else F32_MATERIALIZE_ACT:
        # the same fp32 arithmetic and bf16 rounding as the fused operand prologue
        A1 = ops.bn_act(Y1, bn1, SLOPE, mask=mask, HW=H * W, amax=_slot(am, AM_A1))
        Y2, part2 = ops.conv_fwd_bn(A1, B, H, W, w2, b2, cop, 1, tag=name + ".conv.4.fwd",
                                    stats=training,
                                    amax=(_slot(am, AM_A1), pw.amax_w2(ops.PACK_FWD)))
    else:
        Y2, part2 = ops.conv_fwd_bn(Y1, B, H, W, w2, b2, cop, 1, pro=(bn1.scale, bn1.shift, mask),
                                    tag=name + ".conv.4.fwd", stats=training)
    if training:
        bn2 = ops.bn_train(Y2, bn2m, co, bn2m.momentum, eps2, part=part2, gamma=pw.vec("g2"),
                           beta=pw.vec("be2"))
    else:
        bn2 = _bn_eval(bn2m, cop, co, eps2, xin.device, pw.vec("g2"), pw.vec("be2"))
    s = _BlockSaved()
    s.X, s.Y1, s.Y2, s.bn1, s.bn2, s.mask = X, Y1, Y2, bn1, bn2, mask
    s.pw = pw
    s.B, s.H, s.W, s.cip, s.cop = B, H, W, cip, cop
    s.V = V if training else None  # Winograd-domain input, reused by the weight gradient
    s.Vf16 = Vf16 if training else None  # (the bf16 path's F(4x4) V, likewise)
    s.A1 = A1 if training else None  # activated 1x1 operand, reused by its weight gradient
    s.Z = None
    s.am = am
    return s


def _block_bwd(blk, s, G, grads, need_dx, name="", gpart=None):
    """G: grad wrt the block output z = lrelu(bn2(Y2)) [M, cop]; gpart: the
    BN-backward partials of G that its producer already wrote (ops.bn_bwd)."""
    c0, bn1m, c4, bn2m = blk.conv[0], blk.conv[1], blk.conv[4], blk.conv[5]
    ci, co = c0.in_channels, c4.out_channels
    B, H, W = s.B, s.H, s.W
    HW = H * W
    g = grads
    dtype = G.dtype
    w2d = s.pw.w2(ops.PACK_DGRAD)
    h2 = s.V is not None and s.V.dtype == ops.H2
    am_dy1 = _slot(s.am, AM_DY1)
    if s.A1 is not None and s.A1.dtype == ops.H2:
        # h2 1x1 operands (csrc/nsm_conv_h2d.inc): the BN backward writes dY2
        # pre-split, scaled from the bound its finalize derives (AM_DY2B); the
        # weight and input gradients read it by LDS-DMA
        am_dy2 = _slot(s.am, AM_DY2B)
        dY2h = ops.bn_bwd(G, s.Y2, s.bn2, HW, None, co, g[bn2m.weight], g[bn2m.bias], g[c4.bias],
                          part=gpart, h2=(_slot(s.am, AM_K1DZ), am_dy2))
        A1 = s.A1
        _wgrad(lambda: ops.conv1x1_wgrad_h2(dY2h, A1, ci, co, g[c4.weight],
                                            amax=(am_dy2, _slot(s.am, AM_A1)),
                                            tag=name + ".conv.4.wgrad"), dY2h, A1)
        s.A1 = A1 = None
        # h2 Winograd 3x3: one GEMM pass storing dA1 + the BN-backward partials;
        # the dual transform forms dY1 per element (wino_dual_input_bn_h2), so
        # dY1 is never stored and the GEMM never recomputed, under the bound
        # the finalize derives from max|k1 dz| (AM_DY1B)
        lazy = h2 and need_dx and LAZY_DY1_H2
        # a direct 3x3 on h2 operands (conv2) takes dY1 as h2 too, written by
        # the BN backward with the bound its finalize derives (AM_DY1B); the
        # recompute form (mode 2) writes fp32 dY1, so it is not used there
        h2_3x3 = s.X is not None and s.X.dtype == ops.H2
        recompute = not lazy and not h2_3x3 and bnb_mode(s.cip, s.cop, dtype, h2=True) == 2
        if h2_3x3 or lazy:
            am_dy1 = _slot(s.am, AM_DY1B)
        dY1 = ops.conv1x1_dgrad_bn_bwd_h2(dY2h, HW, w2d, s.Y1, s.bn1, s.mask, ci, g[bn1m.weight],
                                          g[bn1m.bias], g[c0.bias], recompute,
                                          tag=name + ".conv.4.dgrad",
                                          amax=(am_dy2, s.pw.amax_w2(ops.PACK_DGRAD)),
                                          amax_out=None if h2_3x3 or lazy else am_dy1,
                                          h2_out=(_slot(s.am, AM_K1DZ1), am_dy1)
                                          if h2_3x3 or lazy else None, defer=lazy)
        return _block_bwd_3x3(blk, s, dY1, grads, need_dx, name, h2, am_dy1)
    dY2 = ops.bn_bwd(G, s.Y2, s.bn2, HW, None, co, g[bn2m.weight], g[bn2m.bias], g[c4.bias],
                     part=gpart, amax=_slot(s.am, AM_DY2))
    am_w2d = (_slot(s.am, AM_DY2), s.pw.amax_w2(ops.PACK_DGRAD))
    if s.A1 is not None:
        A1 = s.A1
        _wgrad(lambda: ops.conv_wgrad(dY2, A1, B, H, W, 1, ci, co, g[c4.weight],
                                      tag=name + ".conv.4.wgrad",
                                      amax=(_slot(s.am, AM_DY2), _slot(s.am, AM_A1))), dY2, A1)
        s.A1 = A1 = None
    else:
        pro = (s.bn1.scale, s.bn1.shift, s.mask)
        _wgrad(lambda: ops.conv_wgrad(dY2, s.Y1, B, H, W, 1, ci, co, g[c4.weight], pro=pro,
                                      tag=name + ".conv.4.wgrad"), dY2, s.Y1, *pro)
    mode = bnb_mode(s.cip, s.cop, dtype)
    if mode == 2 and _wino_f16(s):
        mode = 1   # dY1 through nsm_bn_bwd_apply, which records max|dY1| (the dgrad's V scale)
    # pre-split (h2) Winograd operands: dY1's producer records max|dY1|, the
    # scale source of both its transforms (Vd, dM)
    # dY1 is consumed only by its two Winograd transforms: leave the BN apply
    # to the dual transform kernel, dY1 is never stored
    lazy = s.V is not None and need_dx and DUAL_TRANSFORM and LAZY_DY1 and not h2
    # bf16 F(4x4): dY1 formed inside the dual transform, scaled from the bound
    # the finalize derives (AM_DY1B, from max|k1 dz| of the GEMM epilogue)
    lazy16 = mode == 1 and _wino_f16(s) and need_dx and BF16_DUAL and LAZY_DY1_F16
    if mode:
        if lazy16:
            am_dy1 = _slot(s.am, AM_DY1B)
        dY1 = ops.conv1x1_dgrad_bn_bwd(dY2, B, H, W, w2d, s.Y1, s.bn1, s.mask, ci, g[bn1m.weight],
                                       g[bn1m.bias], g[c0.bias], mode == 2,
                                       tag=name + ".conv.4.dgrad", defer=lazy or lazy16,
                                       amax=am_w2d, amax_out=None if lazy16 else am_dy1,
                                       bound=(_slot(s.am, AM_K1DZ1), am_dy1) if lazy16 else None)
    else:
        dA1 = ops.conv_fwd(dY2, B, H, W, w2d, None, s.cip, 1, tag=name + ".conv.4.dgrad",
                           amax=am_w2d)
        dY1 = ops.bn_bwd(dA1, s.Y1, s.bn1, HW, s.mask, ci, g[bn1m.weight], g[bn1m.bias],
                         g[c0.bias], defer=lazy, amax=am_dy1)
    return _block_bwd_3x3(blk, s, dY1, grads, need_dx, name, h2, am_dy1)


def _block_bwd_3x3(blk, s, dY1, grads, need_dx, name, h2, am_dy1):
    """The 3x3 conv's weight and input gradients of a DoubleConv from dY1 (the
    gradient wrt its output Y1; a DeferredBnBwd where the dual transform forms
    it). h2: the forward kept an h2 V (pre-split Winograd operands)."""
    c0 = blk.conv[0]
    ci = c0.in_channels
    B, H, W = s.B, s.H, s.W
    g = grads
    dtype = s.Y1.dtype
    Vd = None
    if h2:
        tile = wino_tile(s.cip, H, W)
        if isinstance(dY1, ops.DeferredBnBwd):
            Vd, dM = ops.wino_dual_input_bn_h2(dY1, s.Y1, s.bn1, s.mask, B, H, W, tile, am_dy1)
        else:
            Vd, dM = ops.wino_dual_input_h2(dY1, B, H, W, tile, am_dy1)
        V = s.V
        _wgrad(lambda: ops.conv3x3_wgrad_wino(dY1, V, B, H, W, s.cip, ci, ci, g[c0.weight],
                                              tile=tile, tag=name + ".conv.0.wgrad", dM=dM,
                                              amax=(am_dy1, _slot(s.am, AM_X))), dM, V)
        s.V = V = None
        if not need_dx:
            return None
        return ops.conv3x3_wino(dY1, B, H, W, s.pw.U1(tile, True), None, s.cip, tile=tile,
                                tag=name + ".conv.0.dgrad", v_in=Vd, amax_v=am_dy1,
                                amax_u=s.pw.amax_U1(True))
    if s.V is not None:
        tile = wino_tile(s.cip, H, W)
        dM = None
        if need_dx and DUAL_TRANSFORM:
            # dY1's two Winograd transforms (dgrad input, wgrad) from one read
            am2 = (_slot(s.am, AM_VD), _slot(s.am, AM_DM))
            if isinstance(dY1, ops.DeferredBnBwd):
                Vd, dM = ops.wino_dual_input_bn(dY1, s.Y1, s.bn1, s.mask, B, H, W, tile=tile,
                                                amax=am2)
            else:
                Vd, dM = ops.wino_dual_input(dY1, B, H, W, tile=tile, amax=am2)
        V = s.V
        _wgrad(lambda: ops.conv3x3_wgrad_wino(dY1, V, B, H, W, s.cip, ci, ci, g[c0.weight],
                                              tile=tile, tag=name + ".conv.0.wgrad", dM=dM,
                                              amax=(_slot(s.am, AM_DM), _slot(s.am, AM_V))),
               dM, V, dY1 if dM is None else None)
        s.V = V = None
    elif s.X is not None and s.X.dtype == ops.H2:   # direct 3x3 on h2 operands (dY1 from the BN backward)
        assert dY1.dtype == ops.H2
        _wgrad(lambda: ops.conv3x3_wgrad_h2(dY1, s.X, B, H, W, ci, ci, g[c0.weight],
                                            tag=name + ".conv.0.wgrad",
                                            amax=(am_dy1, _slot(s.am, AM_X))), dY1, s.X)
        if not need_dx:
            return None
        return ops.conv3x3_h2(dY1, B, H, W, s.pw.w1(ops.PACK_DGRAD), None, s.cip, stats=False,
                              amax=(am_dy1, s.pw.amax_w1(ops.PACK_DGRAD)),
                              tag=name + ".conv.0.dgrad")[0]
    elif s.Vf16 is not None:   # bf16 F(4x4): dY's transform, then the Winograd-domain GEMMs
        if isinstance(dY1, ops.DeferredBnBwd):   # dY1 formed per element, never stored
            Vd, dM = ops.wino_dual_bn_f16(dY1, s.Y1, s.bn1, s.mask, B, H, W, am_dy1)
        elif need_dx and BF16_DUAL:   # with the input gradient's V, from one read of dY1
            Vd, dM = ops.wino_dual_f16(dY1, B, H, W, am_dy1)
        else:
            dM = ops.wino_dout_f16(dY1, B, H, W, am_dy1)
        Vf = s.Vf16
        _wgrad(lambda: ops.conv3x3_wgrad_wino_f16(dM, Vf, B, H, W, s.cip, s.cip, ci, ci,
                                                  g[c0.weight], amax=(am_dy1, _slot(s.am, AM_X)),
                                                  tag=name + ".conv.0.wgrad"), dM, Vf)
        s.Vf16 = Vf = None
    else:
        _wgrad(lambda: ops.conv_wgrad(dY1, s.X, B, H, W, 3, ci, ci, g[c0.weight],
                                      tag=name + ".conv.0.wgrad",
                                      amax=(am_dy1, _slot(s.am, AM_X))), dY1, s.X)
    if not need_dx:
        return None
    if s.cip >= WINOGRAD_MIN_CHANNELS and dtype == torch.float32:
        tile = wino_tile(s.cip, H, W)
        U1d = s.pw.U1(tile, True)
        return ops.conv3x3_wino(dY1, B, H, W, U1d, None, s.cip, tile=tile,
                                tag=name + ".conv.0.dgrad", v_in=Vd, amax_v=_slot(s.am, AM_VD),
                                amax_u=s.pw.amax_U1(True))
    if _wino_f16(s):   # bf16: Winograd F(4x4) on f16 operands, as the forward
        return ops.conv3x3_wino_f16(dY1, B, H, W, s.pw.Uf16(True), None, s.cip,
                                    amax=(am_dy1, s.pw.amax_Uf16()), stats=False,
                                    tag=name + ".conv.0.dgrad", v_in=Vd)[0]
    w1d = s.pw.w1(ops.PACK_DGRAD)
    return ops.conv_fwd(dY1, B, H, W, w1d, None, s.cip, 3, tag=name + ".conv.0.dgrad",
                        amax=(am_dy1, s.pw.amax_w1(ops.PACK_DGRAD)))


def _has_f16_u(pw):
    """The block's weight layouts hold the bf16 path's F(4x4) filters."""
    return getattr(pw, "Uf16", None) is not None and pw.Uf16() is not None


def _wino_f16(s):
    """True when block s's 3x3 runs the bf16 path's F(4x4) f16 Winograd
    (forward and input gradient; its filters were prepared)."""
    pw = s.pw
    return (s.Y1 is not None and s.Y1.dtype == torch.bfloat16
            and getattr(pw, "Uf16", None) is not None and pw.Uf16(True) is not None)


def _bnred_of(s):
    """bnred= of a gradient producer reducing block s's output-BN backward:
    (Y2, bn2) and, where the block's 1x1 runs on h2 operands, its max|k1 dz|
    slot (the dY2 bound, bn_bwd(h2=...))."""
    if s.A1 is not None and s.A1.dtype == ops.H2:
        return s.Y2, s.bn2, _slot(s.am, AM_K1DZ)
    return s.Y2, s.bn2


def block_shapes(Rh, Rw):
    """(h, w) each DoubleConv runs at, for the half-resolution input Rh x Rw
    (Unetmodel.py:104-142: floor halving by AvgPool2d, decoder at the skip size)."""
    enc, h, w = {}, Rh, Rw
    for k in ENCODER:
        enc[k] = (h, w)
        h, w = h // 2, w // 2
    return {**enc, 6: enc[4], 7: enc[3], 8: enc[2], 9: (Rh, Rw)}


PREP_BATCH = os.environ.get("NSM_PREP_BATCH", "1") != "0"


class FrozenWeights:
    """Inference with frozen weights (nsm_amd.infer.GraphedUnet): inside
    `with FrozenWeights(model):` the first eval forward prepares the weight
    layouts (the prep launches) and the eval BatchNorm vectors (one
    nsm_bn_finalize_eval per BN) as usual and keeps them; later forwards skip
    those launches (a graph captured then holds only the per-frame work: the
    reference's infer.py loads its weights once, infer.py:40-60). The kept
    buffers stay valid while the weights and BN statistics do: refresh()
    rewrites them in place (same addresses, so a captured graph stays valid)
    after any change."""

    def __init__(self, mod):
        self.mod = mod
        self.sws = {}      # key -> StepWeights (persistent output buffers)
        self.bn = {}       # (id(bn module), C) -> (bn module, C, c_real, eps, BNState)
        self.ready = False

    def __enter__(self):
        global _FROZEN
        if _FROZEN is not None:
            raise RuntimeError("FrozenWeights contexts do not nest")
        _FROZEN = self
        return self

    def __exit__(self, *exc):
        global _FROZEN
        _FROZEN = None
        return False

    def bn_eval(self, bn_mod, C, c_real, eps, device, gamma, beta):
        key = (id(bn_mod), C)
        ent = self.bn.get(key)
        if ent is None:
            st = ops.bn_eval(bn_mod, C, c_real, eps, device, gamma=gamma, beta=beta)
            self.bn[key] = (bn_mod, C, c_real, eps, st)
            return st
        return ent[4]

    def refresh(self):
        """Rewrite the kept weight layouts and BN vectors from the module's
        current parameters and running statistics (same buffers)."""
        for sw in self.sws.values():
            if not sw.valid(self.mod):
                raise RuntimeError("FrozenWeights.refresh: the parameters were re-allocated "
                                   "(e.g. FlatAdamW re-homed them); build a new one")
            sw.run()
        for bn_mod, C, c_real, eps, st in self.bn.values():
            ops.bn_eval_into(st, bn_mod, C, c_real, eps)


_FROZEN = None


def _bn_eval(bn_mod, C, c_real, eps, device, gamma, beta):
    if _FROZEN is not None:
        return _FROZEN.bn_eval(bn_mod, C, c_real, eps, device, gamma, beta)
    return ops.bn_eval(bn_mod, C, c_real, eps, device, gamma=gamma, beta=beta)


def _step_weights(mod, dtype, Rh, Rw, training, act_slots=None):
    """The step's weight layouts, written by ONE prep launch (cached per
    signature; rebuilt when the parameters moved, e.g. FlatAdamW re-homing).
    act_slots: the forward's activation-maximum slots, zeroed by that launch.
    NSM_PREP_BATCH=0: None (every block packs its own, one launch per layout)."""
    if not PREP_BATCH:
        return None
    # pre-split (h2) Winograd operands in fp32 training with the f16x2 arithmetic
    h2 = bool(training) and dtype == torch.float32 and H2_WINO and ops.get_f32_split() == 2
    key = (dtype, Rh, Rw, bool(training), WINOGRAD_MIN_CHANNELS, h2)
    cache = mod.__dict__.setdefault("_step_weights", {})
    sw = cache.get(key)
    if sw is None or not sw.valid(mod):
        sw = cache[key] = StepWeights(mod, dtype, block_shapes(Rh, Rw), training,
                                      WINOGRAD_MIN_CHANNELS, wino_tile, h2=h2)
    fz = _FROZEN if not training else None
    if fz is not None and fz.ready and fz.sws.get(key) is sw:
        # frozen inference weights: the layouts are kept; only the forward's
        # activation-maximum slots need zeroing
        if act_slots is not None:
            call("nsm_zero_u32", ptr(act_slots), act_slots.numel(), stream())
        return sw
    if fz is not None:
        fz.sws[key] = sw
    sw.run(act_slots)
    return sw


class _UnetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        training = mod.training
        B, C, H, W = x.shape
        dev = x.device
        x32 = x.detach().to(torch.float32)
        orig_hw = (H, W)
        if H % 2 or W % 2:  # Unetmodel.py:94-97
            He, We = H - H % 2, W - W % 2
            x32 = ops.resize(x32.contiguous().view(B * C * H * W, 1), B * C, H, W, He, We).view(B, C, He, We)
            H, W = He, We
        x32 = x32.contiguous()
        Rh, Rw = H // 2, W // 2
        cin_p = ops.pad32(4 * C)
        assert mod.conv2.conv[0].in_channels == 4 * C, (
            f"Unet expects {mod.conv2.conv[0].in_channels // 4} input channels, got {C}")
        cdt = mod.activation_dtype()
        masks, mask_max = _masks_for(mod, B, dev, training)
        # per-step maxima of the f16x2 GEMM operands of every block (their
        # producers fill them), zeroed by the weight preparation's first launch
        amax = torch.empty(AM_PER_BLOCK * 10 * ops.AMAX_WORDS, dtype=torch.int32, device=dev)
        sw = _step_weights(mod, cdt, Rh, Rw, training, act_slots=amax)
        if sw is None:
            amax = None
        w1_2 = sw.block(2).w1(ops.PACK_FWD) if sw and ops.pad32(
            mod.conv2.conv[0].in_channels) < WINOGRAD_MIN_CHANNELS else None
        if w1_2 is not None and w1_2.dtype == ops.H2:
            # conv2's direct 3x3 on h2 operands: X pre-split, scaled from max|x|
            X = ops.input_prep_h2(x32, cin_p, _x_slot(amax, 2))
        else:
            X = ops.input_prep(x32, cin_p, cdt, amax=_x_slot(amax, 2))

        saved, c, shapes = {}, {}, {}
        inp, h, w = X, Rh, Rw
        for k in ENCODER:
            with ops.stage(f"conv{k}.fwd"):
                s = _block_fwd(mod.block(k), inp, B, h, w, training, masks.get(k), f"conv{k}",
                               pw=sw.block(k) if sw else None, fuse_out=True,
                               am=_block_slots(amax, k), mask_max=mask_max.get(k, 1.0))
                saved[k], shapes[k] = s, (h, w)
                if s.Z is not None:
                    c[k] = s.Z
                    if k < 5:
                        inp = ops.avgpool2(c[k], B, h, w)
                elif k < 5 and ACT_POOL:   # z and its pooling from one read of Y2
                    c[k], inp = ops.bn_act_pool(s.Y2, s.bn2, B, h, w, SLOPE,
                                                amax=_x_slot(amax, k + 1))
                elif k == 5 and LAZY_DECODER and cdt == torch.bfloat16:
                    c[k] = ops.Lazy(s.Y2, s.bn2, None)   # sampled by conv6's upsample
                else:
                    # max|c_k| bounds the next block's input (its pooling or
                    # bilinear upsample), the scale source of an h2 V
                    c[k] = ops.bn_act(s.Y2, s.bn2, SLOPE, amax=_x_slot(amax, k + 1))
                    if k < 5:
                        inp = ops.avgpool2(c[k], B, h, w)
                if k < 5:
                    h, w = h // 2, w // 2
        skip_shape = {6: shapes[4], 7: shapes[3], 8: shapes[2], 9: (Rh, Rw)}
        cur, (h, w) = c[5], shapes[5]
        ups = {}
        for k in DECODER:
            with ops.stage(f"conv{k}.fwd"):
                h2, w2 = 2 * h, 2 * w
                th, tw = skip_shape[k]
                src = None
                lazy = isinstance(cur, ops.Lazy)
                if (th, tw) != (h2, w2):   # up x2 then _upsample_and_match, fused
                    up = ops.up2_resize_act(cur, B, h, w, th, tw, SLOPE) if lazy else None
                    if up is None:
                        cur = cur.materialise(SLOPE) if lazy else cur
                        up = ops.up2_resize(cur, B, h, w, th, tw)
                elif fuses_resize(mod.block(k), cdt, training):  # sampled by the input transform
                    if lazy:
                        cur = cur.materialise(SLOPE)
                        if amax is not None:   # (bn_act of a Lazy records no maximum)
                            ops.absmax(cur, _x_slot(amax, k))
                    up, src = None, (cur, h, w)
                elif lazy:                 # the previous block output computed on load
                    up = ops.resize_act(cur, B, h, w, h2, w2, SLOPE)
                else:                      # match is the identity (bitwise, as in ATen)
                    up = ops.resize(cur, B, h, w, h2, w2)
                if lazy and up is not None and amax is not None:
                    # the lazy resampling kernels record no maximum: block k's
                    # input-maximum slot (the bf16 F(4x4) V scale) from up itself
                    ops.absmax(up, _x_slot(amax, k))
                ups[k] = (h, w, h2, w2, th, tw)
                res = c[SKIP_OF[k]] if k in SKIP_OF else None
                s = _block_fwd(mod.block(k), up, B, th, tw, training, masks.get(k), f"conv{k}",
                               pw=sw.block(k) if sw else None, src=src, fuse_out=True, res=res,
                               am=_block_slots(amax, k), mask_max=mask_max.get(k, 1.0))
                saved[k] = s
                if s.Z is not None:
                    cur = s.Z
                elif k != 9 and LAZY_DECODER and cdt == torch.bfloat16:
                    cur = ops.Lazy(s.Y2, s.bn2, res)     # only the next upsample reads it
                else:
                    cur = ops.bn_act(s.Y2, s.bn2, SLOPE, res=res,
                                     amax=_x_slot(amax, k + 1) if k < 9 else None)
                h, w = th, tw
        z9 = cur
        with ops.stage("head.fwd"):
            out = ops.head_fwd(z9, B, Rh, Rw, mod.conv10.weight.detach(), mod.conv10.bias.detach())

        if _FROZEN is not None and not training:
            _FROZEN.ready = True   # layouts and BN vectors kept from this forward on
        if training:
            # the running statistics changed in place (HIP kernels): bump their
            # version counters so version-keyed caches (GraphedUnet) see it
            for bm in mod.modules():
                if isinstance(bm, nn.BatchNorm2d):
                    for b in (bm.running_mean, bm.running_var, bm.num_batches_tracked):
                        torch.autograd.graph.increment_version(b)
        ctx.mod = mod
        ctx.saved_blocks = saved
        ctx.ups = ups
        ctx.meta = (B, C, H, W, orig_hw, Rh, Rw, training)
        ctx.z9 = z9
        ctx.save_for_backward(out)
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, gout):
        mod = ctx.mod
        (out,) = ctx.saved_tensors
        B, C, H, W, orig_hw, Rh, Rw, training = ctx.meta
        if not training:
            raise RuntimeError("nsm_amd Unet backward is implemented for train mode (as the "
                               "reference trains); eval-mode BN backward is not on the hot path")
        params = ctx.params
        dev = out.device
        total = sum(p.numel() for p in params)
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        grads, off = {}, 0
        views, offset_of = [], {}
        for p in params:
            v = flat[off:off + p.numel()].view_as(p)
            grads[p] = v
            views.append(v)
            offset_of[id(p)] = off
            off += p.numel()
        dp = mod._grad_allreduce
        split = offset_of.get(id(mod.conv6.conv[0].weight)) if dp is not None else None
        global _wg_stream
        side = None
        if WGRAD_STREAM and not (GRAPH_SIDE_F32 == 0 and torch.cuda.is_current_stream_capturing()
                                 and ctx.saved_blocks[2].Y1.dtype == torch.float32):
            side = _wg_streams.get(dev)
            if side is None:
                side = _wg_streams[dev] = torch.cuda.Stream(device=dev, priority=WGRAD_PRIO)
        _wg_stream = side
        try:
            return _UnetFn._backward(ctx, gout, mod, out, params, flat, grads, views, dp, split)
        finally:
            _wg_stream = None
            if side is not None:   # the gradients are complete when backward returns
                torch.cuda.current_stream().wait_stream(side)
            _wg_hold.clear()

    @staticmethod
    def _backward(ctx, gout, mod, out, params, flat, grads, views, dp, split):
        B, C, H, W, orig_hw, Rh, Rw, training = ctx.meta
        total = flat.numel()

        gout = gout.contiguous().to(torch.float32)
        with ops.stage("head.bwd"):
            G = ops.head_bwd(gout, out, ctx.z9, B, Rh, Rw, mod.conv10.weight.detach(),
                             grads[mod.conv10.weight], grads[mod.conv10.bias])
        sb = ctx.saved_blocks
        skip_grad = {}
        gpart = None
        for k in (9, 8, 7, 6):
            s = sb[k]
            with ops.stage(f"conv{k}.bwd"):
                dX = _block_bwd(mod.block(k), s, G, grads, True, f"conv{k}", gpart=gpart)
                h, w, h2, w2, th, tw = ctx.ups[k]
                # the x2 resize backward also reduces block k-1's output-BN
                # backward (not the up9 composite: its gather kernel measured
                # slower with the reduction than the separate pass, bf16 B=64
                # conv9 stage 4.43 -> 4.70 ms)
                if (th, tw) != (h2, w2):
                    dprev, gpart = ops.up2_resize_bwd(dX, B, h, w, th, tw), None
                elif GRAD_BNRED:
                    dprev, gpart = ops.resize_bwd(dX, B, h, w, h2, w2, bnred=_bnred_of(sb[k - 1]))
                else:
                    dprev, gpart = ops.resize_bwd(dX, B, h, w, h2, w2), None
            # the previous merge / c5 receives dprev; merge_{k-1} = conv + c_skip
            if k - 1 in SKIP_OF:
                skip_grad[SKIP_OF[k - 1]] = dprev
            G = dprev
        if split is not None:   # conv6..conv10 grads are final: overlap their all-reduce
            _allreduce_bucket(flat, split, total, dp[0])
        # encoder: G is now d c5
        need_x = ctx.needs_input_grad[0]
        for k in (5, 4, 3, 2):
            s = sb[k]
            st = ops.stage(f"conv{k}.bwd")
            st.__enter__()
            dX = _block_bwd(mod.block(k), s, G, grads, need_dx=(k > 2 or need_x), name=f"conv{k}",
                            gpart=gpart)
            if k == 5 and training and mod.emulate_checkpoint_bn:
                # checkpoint recompute of conv5 (Unetmodel.py:114-116): 2nd BN update
                blk = mod.block(5)
                M = s.B * s.H * s.W
                ops.bn_running_update(s.bn1, M, s.cip, blk.conv[1], blk.conv[0].in_channels,
                                      blk.conv[1].momentum, blk.conv[1].eps)
                ops.bn_running_update(s.bn2, M, s.cop, blk.conv[5], blk.conv[4].out_channels,
                                      blk.conv[5].momentum, blk.conv[5].eps)
            if k > 2:
                ph, pw = sb[k - 1].H, sb[k - 1].W
                if GRAD_BNRED:
                    G, gpart = ops.avgpool2_bwd_add(dX, B, ph, pw, skip_grad.get(k - 1),
                                                    bnred=_bnred_of(sb[k - 1]))
                else:
                    G = ops.avgpool2_bwd_add(dX, B, ph, pw, skip_grad.get(k - 1))
            else:
                G = dX
            st.__exit__(None, None, None)
        if split is not None:
            _allreduce_bucket(flat, 0, split, dp[0])
        dx = None
        if need_x:
            dx = ops.input_grad(G, B, C, H, W)
            if (H, W) != tuple(orig_hw):
                H0, W0 = orig_hw
                dx = ops.resize_bwd(dx.view(B * C * H * W, 1), B * C, H0, W0, H, W).view(B, C, H0, W0)
        ctx.saved_blocks = None
        ctx.z9 = None
        return (dx, None) + tuple(views)
