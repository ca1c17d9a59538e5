"""Tensor-level wrappers over the libnsm C ABI (one function per entry point).

Activations are NHWC fp32 2-D views `[pixels, channels_padded]`; every
wrapper allocates its outputs with the PyTorch caching allocator and launches
on the current HIP stream. No host synchronisation anywhere.
"""
import os

import torch

from ._lib import call, ptr, stream

F32 = torch.float32
BF16 = torch.bfloat16
# storage of NSM_F16 activations (the fp16-autocast mode): IEEE half bits held
# in int16 tensors, so that they are never taken for the h2 operands
# (torch.float16, H2 below) the fp32 path's producers write
F16S = torch.int16
PACK_FWD, PACK_DGRAD = 0, 1
NSM_F32, NSM_BF16, NSM_F16 = 0, 1, 2
S16 = (BF16, F16S)   # the 16-bit storage dtypes (csrc/nsm_conv_s16.inc, compiled for both)


def dt(t):
    """C-ABI dtype code of an activation tensor (include/nsm.h NSM_F32 /
    NSM_BF16 / NSM_F16)."""
    if t.dtype == BF16:
        return NSM_BF16
    if t.dtype == F16S:
        return NSM_F16
    if t.dtype != F32:
        raise TypeError(f"activations must be float32, bfloat16 or f16 storage (int16), "
                        f"got {t.dtype}")
    return NSM_F32


def like(M, C, ref):
    return torch.empty(M, C, dtype=ref.dtype, device=ref.device)


def pad32(c):
    return (c + 31) // 32 * 32


def empty(*shape, device):
    return torch.empty(*shape, dtype=F32, device=device)


def set_f32_split(mode):
    """Arithmetic of the fp32 GEMMs: 2 (default) = the f16x2 split of
    power-of-two scaled operands (csrc/nsm_conv_split16.inc) where the operand
    maxima are passed (the Winograd GEMMs of the model path), the bf16 split
    elsewhere; 1 = the exact three-way bf16 split everywhere
    (csrc/nsm_conv_split.inc); 0 = the fp32 MFMA. Returns the previous mode."""
    from ._lib import lib
    return int(lib.nsm_set_f32_split(int(mode)))


def get_f32_split():
    """The current fp32 GEMM arithmetic mode (set_f32_split / NSM_F32_SPLIT)."""
    from ._lib import lib
    m = int(lib.nsm_set_f32_split(-1))
    lib.nsm_set_f32_split(m)
    return m


# ---- parameters ------------------------------------------------------------
def pack_conv_weight(w, cout_p, cin_p, mode, dtype=F32):
    """MFMA operand layout of a conv weight, in the activations' dtype."""
    cout, cin, k, _ = w.shape
    taps = k * k
    out = torch.empty(cout_p * taps * cin_p, dtype=dtype, device=w.device)
    fn = {BF16: "nsm_pack_conv_weight_bf16", F16S: "nsm_pack_conv_weight_f16"}.get(
        dtype, "nsm_pack_conv_weight")
    call(fn, ptr(w), cout, cin, k, cout_p, cin_p, mode, ptr(out), stream())
    return out


AMAX_WORDS = 2048   # include/nsm.h NSM_AMAX_WORDS: one operand-maximum slot


def amax_slots(n, device):
    """n zeroed operand-maximum slots (include/nsm.h NSM_AMAX_WORDS each)."""
    return torch.zeros(n * AMAX_WORDS, dtype=torch.int32, device=device)


def amax_slot(buf, i):
    """Slot i of an amax_slots buffer (None -> None). A slot past the buffer's
    end raises: its pointer would aim the kernels' atomics outside it."""
    if buf is None:
        return None
    s = buf[i * AMAX_WORDS:(i + 1) * AMAX_WORDS]
    if s.numel() != AMAX_WORDS:
        raise IndexError(f"amax slot {i} outside a buffer of {buf.numel() // AMAX_WORDS} slots")
    return s


def absmax(x, out=None):
    """Operand-maximum slot holding max|x| (nsm_absmax): the f16x2 GEMM
    operand scale of a tensor whose producer did not record it."""
    if x.dtype not in (F32, BF16):
        raise TypeError(f"absmax: fp32 or bf16 tensor expected, got {x.dtype}")
    if out is None:
        out = amax_slots(1, x.device)
    call("nsm_absmax_bf16" if x.dtype == BF16 else "nsm_absmax", ptr(x), x.numel(), ptr(out),
         stream())
    return out


def pad_vec(v, n_p):
    if v.numel() == n_p:
        return v
    out = empty(n_p, device=v.device)
    call("nsm_pad_vec", ptr(v), v.numel(), n_p, ptr(out), stream())
    return out


# ---- convolution -----------------------------------------------------------
# Kernel probes: {tag: [(start_event, end_event), ...]} — bench.py registers a
# tag to time one specific launch with HIP events on the launch stream.
PROBES = {}


def _probe(tag):
    lst = PROBES.get(tag) if tag is not None else None
    if lst is None:
        return None
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    lst.append((a, b))
    return b


class Partials:
    """Per-channel BN partials {sum, M2} over row chunks of rpc rows:
    [nchunk][2][C]; rpc == 0: counted partials [nchunk][3][C] {sum, M2, count}."""
    __slots__ = ("buf", "nchunk", "rpc", "_merged")

    def __init__(self, buf, nchunk, rpc):
        self.buf, self.nchunk, self.rpc = buf, nchunk, rpc
        self._merged = None


# Stage markers for per-stage PMC attribution (tools/stage_pmc.py): with
# NSM_STAGE_MARKS=1 every stage is bracketed by nsm_stage_mark launches whose
# grid encodes the stage (code = STAGE_CODES[tag] + 1 blocks; 0 = stage end).
STAGE_NAMES = ["conv2", "conv3", "conv4", "conv5", "conv6", "conv7", "conv8", "conv9", "head"]
STAGE_CODES = {f"{n}.{d}": 1 + 2 * i + j for i, n in enumerate(STAGE_NAMES)
               for j, d in enumerate(("fwd", "bwd"))}
STAGE_CODES.update({"dp.bn_broadcast": 40, "dp.allreduce_wait": 41})
MARK_STAGES = os.environ.get("NSM_STAGE_MARKS", "0") == "1"


def _mark(code):
    call("nsm_stage_mark", code, stream())


class stage:
    """Context manager: if `tag` is registered in PROBES, bracket everything
    launched inside with HIP events on the current stream (bench.py uses it
    for the per-stage roofline table); with NSM_STAGE_MARKS=1 also with
    marker launches (per-stage rocprofv3 counters)."""
    __slots__ = ("tag", "end")

    def __init__(self, tag):
        self.tag = tag
        self.end = None

    def __enter__(self):
        if MARK_STAGES and self.tag in STAGE_CODES:
            _mark(STAGE_CODES[self.tag])
        self.end = _probe(self.tag)
        return self

    def __exit__(self, *exc):
        if self.end is not None:
            self.end.record()
        if MARK_STAGES and self.tag in STAGE_CODES:
            _mark(0)
        return False


def conv_fwd(x, B, H, W, wpk, bias, cout_p, ksize, pro=None, out=None, tag=None, slope=0.2,
             amax=(None, None)):
    """x: [B*H*W, cin_p]; returns y [B*H*W, cout_p]. pro=(scale, shift, mask|None):
    the operand loader applies lrelu(x*scale+shift, slope)*mask. amax =
    (max|x|, max|wpk|) operand-maximum slots: with both (fp32, no prologue)
    the GEMM runs the f16x2 split."""
    return conv_fwd_bn(x, B, H, W, wpk, bias, cout_p, ksize, pro, out, tag, stats=False,
                       slope=slope, amax=amax)[0]


def _pair(amax):
    """Both slots' pointers, or (None, None) unless both are given."""
    if amax[0] is None or amax[1] is None:
        return None, None
    return ptr(amax[0]), ptr(amax[1])


def conv_fwd_bn(x, B, H, W, wpk, bias, cout_p, ksize, pro=None, out=None, tag=None, stats=True,
                slope=0.2, amax=(None, None)):
    """conv_fwd returning (y, Partials|None): with stats=True the GEMM epilogue
    also emits the BN batch-statistics partials of y."""
    from ._lib import lib
    M, cin_p = x.shape
    y = out if out is not None else like(M, cout_p, x)
    if wpk.dtype != x.dtype or y.dtype != x.dtype:
        raise TypeError("conv_fwd: activations, packed weights and output must share a dtype")
    sc = sh = mk = None
    if pro is not None:
        sc, sh, mk = pro
    part = None
    if stats:
        rows_fn = lib.nsm_conv_stat_rows_bf16 if x.dtype in S16 else lib.nsm_conv_stat_rows
        rpc = rows_fn(B, H, W, cout_p)
        nchunk = -(-M // rpc)
        part = Partials(empty(nchunk * 2 * cout_p, device=x.device), nchunk, rpc)
    ev = _probe(tag)
    args = (ptr(x), x.stride(0), B, H, W, cin_p, ptr(wpk), ptr(bias), cout_p, ksize, ptr(y),
            y.stride(0), ptr(sc), ptr(sh), ptr(mk), slope,
            ptr(part.buf) if part is not None else None)
    if x.dtype == BF16:
        call("nsm_conv_fwd_bf16", *args, stream())
    elif x.dtype == F16S:
        call("nsm_conv_fwd_f16", *args, stream())
    else:
        call("nsm_conv_fwd_stats", *args, *_pair(amax), stream())
    if ev is not None:
        ev.record()
    return y, part


def conv_fwd_act(x, B, H, W, wpk, bias, cout_p, ksize, st, res=None, slope=0.2, tag=None):
    """Eval: lrelu(BN(conv(x) + bias)) (+ res) in one pass, BN from the
    running statistics (st = bn_eval's BNState): the conv output itself is
    never stored (nsm_conv_fwd_act)."""
    M = x.shape[0]
    y = like(M, cout_p, x)
    if wpk.dtype != x.dtype or (res is not None and res.dtype != x.dtype):
        raise TypeError("conv_fwd_act: activations, weights and skip must share a dtype")
    ev = _probe(tag)
    call("nsm_conv_fwd_act", ptr(x), x.stride(0), B, H, W, x.shape[1], ptr(wpk), ptr(bias),
         cout_p, ksize, ptr(y), y.stride(0), ptr(st.scale), ptr(st.shift), slope, ptr(res),
         res.stride(0) if res is not None else 0, dt(x), stream())
    if ev is not None:
        ev.record()
    return y


def wino_tiles(B, H, W, tile):
    return B * ((H + tile - 1) // tile) * ((W + tile - 1) // tile)


def wino_weight(w, n_p, k_p, flip, tile=4):
    """Winograd-domain filters U[(tile+2)^2][n_p][k_p] of a 3x3 conv weight
    (flip=False: forward; flip=True: input-gradient of that conv)."""
    cout, cin = w.shape[0], w.shape[1]
    U = empty((tile + 2) ** 2 * n_p * k_p, device=w.device)
    call("nsm_wino_weight", ptr(w), cout, cin, n_p, k_p, int(flip), tile, ptr(U), stream())
    return U


def conv3x3_wino(x, B, H, W, U, bias, cout_p, tile=4, tag=None, keep_v=False, relu=False,
                 stats=False, nslot=None, src_hw=None, act=None, v_in=None, amax_v=None,
                 amax_u=None):
    """3x3 (pad 1) convolution of x [B*H*W, cin_p] via Winograd F(tile x tile, 3x3).
    keep_v=True also returns the transformed input V [(tile+2)^2][T][cin_p],
    reused by the Winograd weight gradient. stats=True returns (y, V|None,
    Partials|None): the BN batch-statistics partials of y written by the output
    transform (counted layout, rpc 0), None where nsm_wino_stat_slots says the
    separate pass is faster (nslot: override the slot count, tests).
    src_hw=(hi, wi): x is [B*hi*wi, cin_p], convolved after a bilinear
    align_corners resize to H x W that the input transform samples on the fly.
    act=(BNState, res|None): eval BN + LeakyReLU (+ skip) applied by the output
    transform (nsm_wino_output_act). v_in: x's input transform already made
    (wino_dual_input); x is then not read.
    amax_v / amax_u: operand-maximum slots (amax_slot) of max|V| / max|U| (V's is zeroed by the
    caller and filled by the input transform, or by wino_dual_input for v_in;
    U's by the weight preparation): with both, the GEMM runs the f16x2 split
    (csrc/nsm_conv_split16.inc), else the bf16 split."""
    from ._lib import lib
    cin_p = x.shape[1]
    M = B * H * W
    hi, wi = src_hw if src_hw is not None else (H, W)
    assert x.shape[0] == B * hi * wi, (x.shape, B, hi, wi)
    nb, T = (tile + 2) ** 2, wino_tiles(B, H, W, tile)
    Mb = empty(nb * T * cout_p, device=x.device)
    y = empty(M, cout_p, device=x.device)
    st = stream()
    h2 = U.dtype == H2   # pre-split operands (csrc/nsm_conv_h2.inc)
    ev_all = _probe(tag)  # the whole convolution: input transform + GEMM + output transform
    if v_in is not None:
        V = v_in
    elif h2:
        # amax_v: max|x| (x's producer), the scale source of the h2 V
        V = torch.empty(nb * T * 2 * cin_p, dtype=H2, device=x.device)
        call("nsm_wino_input_h2", ptr(x), x.stride(0), B, hi, wi, H, W, cin_p, tile, ptr(V),
             ptr(amax_v), st)
    else:
        V = empty(nb * T * cin_p, device=x.device)    # kept alive for the wgrad
        call("nsm_wino_input_resize", ptr(x), x.stride(0), B, hi, wi, H, W, cin_p, tile,
             int(relu), ptr(V), ptr(amax_v), st)
    ev = _probe(tag + ".gemm" if tag else None)   # the batched MFMA GEMM alone
    if h2:
        assert V.dtype == H2 and amax_v is not None and amax_u is not None
        call("nsm_wino_gemm_h2", ptr(V), ptr(U), B, H, W, cin_p, cout_p, tile, ptr(Mb),
             ptr(amax_v), wino_beta(tile, 0), ptr(amax_u), wino_beta(tile, 2), st)
    else:
        both = amax_v is not None and amax_u is not None
        call("nsm_wino_gemm_s", ptr(V), ptr(U), B, H, W, cin_p, cout_p, tile, ptr(Mb),
             ptr(amax_v) if both else None, ptr(amax_u) if both else None, st)
    if ev is not None:
        ev.record()
    part = None
    if act is not None:
        assert not stats
        ast, res = act
        call("nsm_wino_output_act", ptr(Mb), B, H, W, cout_p, tile, ptr(bias), ptr(y),
             y.stride(0), ptr(ast.scale), ptr(ast.shift), 0.2, ptr(res),
             res.stride(0) if res is not None else 0, st)
        if ev_all is not None:
            ev_all.record()
        return (y, V) if keep_v else y
    if not stats:
        nslot = 0
    elif nslot is None:
        nslot = int(lib.nsm_wino_stat_slots(B, H, W, cout_p, tile))
    if nslot > 0:
        part = Partials(empty(nslot * 3 * cout_p, device=x.device), nslot, 0)
        call("nsm_wino_output_stats", ptr(Mb), B, H, W, cout_p, tile, ptr(bias), ptr(y),
             y.stride(0), ptr(part.buf), nslot, st)
    else:
        call("nsm_wino_output", ptr(Mb), B, H, W, cout_p, tile, ptr(bias), ptr(y), y.stride(0),
             st)
    if ev_all is not None:
        ev_all.record()
    if stats:
        return y, (V if keep_v else None), part
    return (y, V) if keep_v else y


def wino_dout_f16(dy, B, H, W, amax_dy):
    """dM [36][T][C] f16 = s A dY A^T of the bf16 output gradient
    (nsm_wino_dout_f16): the F(4x4) weight gradient's transform of dY."""
    c_p = dy.shape[1]
    dM = torch.empty(36 * wino_tiles(B, H, W, 4) * c_p, dtype=H2, device=dy.device)
    call("nsm_wino_dout_f16", ptr(dy), dy.stride(0), B, H, W, c_p, 4, ptr(dM), ptr(amax_dy), stream())
    return dM


def wino_dual_f16(dy, B, H, W, amax_dy):
    """(V, dM) of the bf16 output gradient from one read (nsm_wino_dual_f16):
    V as conv3x3_wino_f16's input transform of dy (the input gradient's
    operand, its v_in), dM as wino_dout_f16(dy)."""
    c_p = dy.shape[1]
    n = 36 * wino_tiles(B, H, W, 4) * c_p
    V = torch.empty(n, dtype=H2, device=dy.device)
    dM = torch.empty(n, dtype=H2, device=dy.device)
    call("nsm_wino_dual_f16", ptr(dy), dy.stride(0), B, H, W, c_p, 4, ptr(V), ptr(dM), ptr(amax_dy),
         stream())
    return V, dM


def conv3x3_wgrad_wino_f16(dM, V, B, H, W, cin_p, cout_p, cin, cout, dw, amax, tag=None):
    """dw [cout, cin, 3, 3] of the bf16 path's F(4x4) 3x3 from dM (wino_dout_f16)
    and the forward's V (conv3x3_wino_f16(keep_v=True)); amax = (max|dY| slot,
    max|x| slot), their scale sources."""
    from ._lib import lib
    n = int(lib.nsm_wino_wgrad_f16_ws(B, H, W, cin_p, cout_p, 4))
    ws = empty(n, device=dM.device)
    ev = _probe(tag)
    call("nsm_conv3x3_wgrad_wino_f16", ptr(dM), ptr(V), B, H, W, cin_p, cout_p, cin, cout, 4,
         ptr(dw), ptr(ws), n, ptr(amax[0]), ptr(amax[1]), stream())
    if ev is not None:
        ev.record()


# NSM_BF16_M16=0: the bf16 path's Winograd M in fp32 instead of f16
BF16_M16 = os.environ.get("NSM_BF16_M16", "1") != "0"


def conv3x3_wino_f16(x, B, H, W, U, bias, cout_p, amax, stats=True, tag=None, keep_v=False,
                     m16=None, v_in=None, act=None, src_hw=None):
    """The bf16 path's 3x3 (pad 1) forward by Winograd F(4x4,3x3) on single-plane
    scaled f16 operands (nsm_wino_input_f16 / _gemm_f16 / _output_bf16): x
    [B*H*W, cin_p] bf16, U the prep-kind-6 filters [36][cout_p][cin_p] f16,
    amax = (max|x| slot filled by x's producer, max|w| slot of the prep);
    m16 (default NSM_BF16_M16): M between the GEMM and the output transform
    as f16 (nsm_wino_gemm_f16m / _output_bf16m) instead of fp32; v_in: V
    already formed from x (wino_dual_f16), the input transform skipped.
    act: eval BNState — the output transform writes lrelu(BN(y)) instead of y
    (nsm_wino_output_bf16m_act; f16 M, no statistics). src_hw=(hi, wi): x is
    [B*hi*wi, cin_p], convolved after the align_corners resize to H x W that
    the input transform samples (nsm_wino_input_f16_resize; amax[0] = max|x|).
    Returns (y bf16 [B*H*W, cout_p], Partials of the rounded y | None) and,
    with keep_v, V (the weight gradient's operand)."""
    from ._lib import lib
    assert x.dtype == BF16 and U.dtype == H2
    cin_p = x.shape[1]
    T = wino_tiles(B, H, W, 4)
    st = stream()
    ev = _probe(tag)
    if v_in is not None:
        V = v_in
    elif src_hw is not None:
        hi, wi = src_hw
        assert x.shape[0] == B * hi * wi, (x.shape, B, hi, wi)
        V = torch.empty(36 * T * cin_p, dtype=H2, device=x.device)
        call("nsm_wino_input_f16_resize", ptr(x), x.stride(0), B, hi, wi, H, W, cin_p, 4, ptr(V),
             ptr(amax[0]), st)
    else:
        assert x.shape[0] == B * H * W, (x.shape, B, H, W)
        V = torch.empty(36 * T * cin_p, dtype=H2, device=x.device)
        call("nsm_wino_input_f16", ptr(x), x.stride(0), B, H, W, cin_p, 4, ptr(V), ptr(amax[0]), st)
    m16 = (BF16_M16 if m16 is None else m16) or act is not None
    bv, bu = wino_beta(4, 0), wino_beta(4, 2)
    Mb = torch.empty(36 * T * cout_p, dtype=H2 if m16 else torch.float32, device=x.device)
    # f16 M: one scale exponent per 64 x 64 tile of each component
    m16e = (torch.empty(36 * (-(-T // 64)) * (cout_p // 64), dtype=torch.int32, device=x.device)
            if m16 else None)
    evg = _probe(tag + ".gemm" if tag else None)   # the batched MFMA GEMM alone
    if m16:
        call("nsm_wino_gemm_f16m", ptr(V), ptr(U), B, H, W, cin_p, cout_p, 4, ptr(Mb), ptr(m16e),
             ptr(amax[0]), bv, ptr(amax[1]), bu, st)
    else:
        call("nsm_wino_gemm_f16", ptr(V), ptr(U), B, H, W, cin_p, cout_p, 4, ptr(Mb), ptr(amax[0]),
             bv, ptr(amax[1]), bu, st)
    if evg is not None:
        evg.record()
    if not keep_v:
        V = None
    y = torch.empty(B * H * W, cout_p, dtype=BF16, device=x.device)
    if act is not None:
        assert not stats
        call("nsm_wino_output_bf16m_act", ptr(Mb), ptr(m16e), B, H, W, cin_p, cout_p, 4,
             ptr(amax[0]), bv, ptr(amax[1]), bu, ptr(bias), ptr(y), y.stride(0), ptr(act.scale),
             ptr(act.shift), 0.2, st)
        if ev is not None:
            ev.record()
        return (y, None, V) if keep_v else (y, None)
    nslot = int(lib.nsm_wino_stat_slots(B, H, W, cout_p, 4)) if stats else 0
    part = None
    if nslot > 0:
        part = Partials(empty(nslot * 3 * cout_p, device=x.device), nslot, 0)
    pb = ptr(part.buf) if part is not None else None
    if m16:
        call("nsm_wino_output_bf16m", ptr(Mb), ptr(m16e), B, H, W, cin_p, cout_p, 4, ptr(amax[0]),
             bv, ptr(amax[1]), bu, ptr(bias), ptr(y), y.stride(0), pb, nslot, st)
    else:
        call("nsm_wino_output_bf16", ptr(Mb), B, H, W, cout_p, 4, ptr(bias), ptr(y), y.stride(0),
             pb, nslot, st)
    if ev is not None:
        ev.record()
    return (y, part, V) if keep_v else (y, part)


H2 = torch.float16   # storage dtype of the pre-split (h2) Winograd operands
_BETA = {}


def wino_beta(tile, which):
    """nsm_wino_beta: the bound of a Winograd transform (0 input, 1 output
    gradient, 2 filter) between an h2 operand and its scale source."""
    key = (tile, which)
    if key not in _BETA:
        from ._lib import lib
        _BETA[key] = float(lib.nsm_wino_beta(tile, which))
    return _BETA[key]


def wino_dual_input_h2(dy, B, H, W, tile, amax_dy):
    """wino_dual_input writing (Vd, dM) as h2 tensors; amax_dy: max|dy| slot
    (filled by dy's producer), their scale source."""
    c_p = dy.shape[1]
    n = (tile + 2) ** 2 * wino_tiles(B, H, W, tile) * 2 * c_p
    Vd = torch.empty(n, dtype=H2, device=dy.device)
    dM = torch.empty(n, dtype=H2, device=dy.device)
    call("nsm_wino_dual_input_h2", ptr(dy), dy.stride(0), B, H, W, c_p, tile, ptr(Vd), ptr(dM),
         ptr(amax_dy), stream())
    return Vd, dM


def wino_dual_input(dy, B, H, W, tile=4, amax=(None, None)):
    """(Vd, dM) of the output gradient dy [B*H*W, C_p] from one read of it:
    Vd feeds conv3x3_wino(v_in=Vd) (the input gradient), dM feeds
    conv3x3_wgrad_wino(dM=dM) (the weight gradient). amax: zeroed operand-maximum
    slots (or None) receiving max|Vd|, max|dM| (the f16x2 GEMMs' operand scales)."""
    c_p = dy.shape[1]
    n = (tile + 2) ** 2 * wino_tiles(B, H, W, tile) * c_p
    Vd = empty(n, device=dy.device)
    dM = empty(n, device=dy.device)
    call("nsm_wino_dual_input", ptr(dy), dy.stride(0), B, H, W, c_p, tile, ptr(Vd), ptr(dM),
         ptr(amax[0]), ptr(amax[1]), stream())
    return Vd, dM


class DeferredBnBwd:
    """dY of a train-mode BN backward whose last pass (nsm_bn_bwd_apply) was
    not run: g (grad wrt lrelu(BN(y))*mask) and the finalize coefficients.
    Consumed by wino_dual_input_bn, which forms dY per element on the fly."""
    __slots__ = ("g", "coef", "shape", "device", "dtype")

    def __init__(self, g, coef):
        self.g, self.coef = g, coef
        self.shape, self.device, self.dtype = g.shape, g.device, g.dtype


def wino_dual_input_bn(d, y, st, mask, B, H, W, tile=4, slope=0.2, amax=(None, None)):
    """wino_dual_input of the BN backward d = DeferredBnBwd(g, coef) of BN
    input y (state st, Dropout2d mask [B][C] or None): dY is never stored."""
    c_p = y.shape[1]
    n = (tile + 2) ** 2 * wino_tiles(B, H, W, tile) * c_p
    Vd = empty(n, device=y.device)
    dM = empty(n, device=y.device)
    call("nsm_wino_dual_input_bn", ptr(d.g), d.g.stride(0), ptr(y), y.stride(0), B, H, W, c_p,
         tile, ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(d.coef),
         ptr(Vd), ptr(dM), ptr(amax[0]), ptr(amax[1]), stream())
    return Vd, dM


def wino_dual_input_bn_h2(d, y, st, mask, B, H, W, tile, bound, slope=0.2):
    """wino_dual_input_h2 of d = DeferredBnBwd(g, coef) (BN input y, state st,
    mask [B][C] or None): dY is formed per element, never stored; bound: the dY
    bound slot bn_bwd_finalize filled (the scale source of Vd, dM and their
    GEMMs)."""
    c_p = y.shape[1]
    n = (tile + 2) ** 2 * wino_tiles(B, H, W, tile) * 2 * c_p
    Vd = torch.empty(n, dtype=H2, device=y.device)
    dM = torch.empty(n, dtype=H2, device=y.device)
    call("nsm_wino_dual_input_bn_h2", ptr(d.g), d.g.stride(0), ptr(y), y.stride(0), B, H, W, c_p,
         tile, ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(d.coef), ptr(Vd),
         ptr(dM), ptr(bound), stream())
    return Vd, dM


def wino_dual_bn_f16(d, y, st, mask, B, H, W, bound, slope=0.2):
    """wino_dual_f16 of d = DeferredBnBwd(dA1, coef) (bf16 BN input y, state
    st, mask [B][C] or None): dY1 is formed per element (rounded to bf16 as
    nsm_bn_bwd_apply stores it), never stored (nsm_wino_dual_bn_f16); bound:
    the dY1 bound slot the finalize filled (the scale source of V and dM and
    of the GEMMs reading them)."""
    c_p = y.shape[1]
    n = 36 * wino_tiles(B, H, W, 4) * c_p
    V = torch.empty(n, dtype=H2, device=y.device)
    dM = torch.empty(n, dtype=H2, device=y.device)
    call("nsm_wino_dual_bn_f16", ptr(d.g), d.g.stride(0), ptr(y), y.stride(0), B, H, W, c_p, 4,
         ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(d.coef), ptr(V), ptr(dM),
         ptr(bound), stream())
    return V, dM


def conv3x3_wgrad_wino(dy, V, B, H, W, cin_p, cin, cout, dw, tile=4, tag=None, dM=None,
                       amax=(None, None)):
    """dw [cout, cin, 3, 3] of a 3x3 conv whose forward kept V (conv3x3_wino, same tile).
    dM: dy's transform from wino_dual_input (dy is then not read). amax = (max|dM|,
    max|V|) slots: with both (and dM given) the GEMM runs the f16x2 split."""
    from ._lib import lib
    cout_p = dy.shape[1]
    ev = _probe(tag)
    if dM is not None and dM.dtype == H2:
        # h2 dM / V (wino_dual_input_h2, conv3x3_wino's h2 V): amax = (max|dy|, max|x|),
        # their scale sources
        assert V.dtype == H2 and amax[0] is not None and amax[1] is not None
        n = int(lib.nsm_wino_wgrad_h2_ws(B, H, W, cin_p, cout_p, tile))
        ws = empty(n, device=dy.device)
        call("nsm_conv3x3_wgrad_wino_h2", ptr(dM), ptr(V), B, H, W, cin_p, cout_p, cin, cout,
             tile, ptr(dw), ptr(ws), n, ptr(amax[0]), ptr(amax[1]), stream())
        if ev is not None:
            ev.record()
        return
    n = int(lib.nsm_wino_wgrad_ws(B, H, W, cin_p, cout_p, tile))
    ws = empty(n, device=dy.device)
    if dM is None:
        call("nsm_conv3x3_wgrad_wino", ptr(dy), dy.stride(0), ptr(V), B, H, W, cin_p, cout_p, cin,
             cout, tile, ptr(dw), ptr(ws), n, stream())
    else:
        both = amax[0] is not None and amax[1] is not None
        call("nsm_conv3x3_wgrad_wino_dm", ptr(dM), ptr(V), B, H, W, cin_p, cout_p, cin, cout,
             tile, ptr(dw), ptr(ws), n, ptr(amax[0]) if both else None,
             ptr(amax[1]) if both else None, stream())
    if ev is not None:
        ev.record()


def conv_wgrad(dy, x, B, H, W, ksize, cin, cout, dw, pro=None, tag=None, amax=(None, None)):
    """dw (reference layout [cout, cin, k, k], contiguous) <- sum_p dy (x) x.
    amax = (max|dy|, max|x|) slots: the fp32 GEMM runs the f16x2 split."""
    from ._lib import lib
    cout_p, cin_p = dy.shape[1], x.shape[1]
    bf = dy.dtype in S16
    if x.dtype != dy.dtype:
        raise TypeError("conv_wgrad: dy and x must share a dtype")
    n = int((lib.nsm_conv_wgrad_bf16_ws if bf else lib.nsm_conv_wgrad_ws)(B, H, W, cin_p, cout_p,
                                                                           ksize))
    ws = empty(max(n, 1), device=dy.device)
    sc = sh = mk = None
    if pro is not None:
        sc, sh, mk = pro
    ev = _probe(tag)
    args = (ptr(dy), dy.stride(0), ptr(x), x.stride(0), B, H, W, cin_p, cout_p, ksize, ptr(sc),
            ptr(sh), ptr(mk), 0.2, ptr(ws), n, cin, cout, ptr(dw))
    if bf:
        call("nsm_conv_wgrad_bf16" if dy.dtype == BF16 else "nsm_conv_wgrad_f16", *args, stream())
    else:
        call("nsm_conv_wgrad", *args, *_pair(amax), stream())
    if ev is not None:
        ev.record()


def call_ws(B, H, W, cin_p, cout_p, ksize):
    from ._lib import lib
    return lib.nsm_conv_wgrad_ws(B, H, W, cin_p, cout_p, ksize)


# ---- batch norm ------------------------------------------------------------
def reduce_chunks(M, C):
    from ._lib import lib
    return lib.nsm_reduce_chunks(M, C)


class BNState:
    """Per-BN tensors the backward needs (all [C_padded])."""
    __slots__ = ("scale", "shift", "mean", "invstd", "part", "nchunk", "gamma", "beta")

    def __init__(self, C, device):
        self.scale = empty(C, device=device)
        self.shift = empty(C, device=device)
        self.mean = empty(C, device=device)
        self.invstd = empty(C, device=device)
        self.part = None
        self.nchunk = 0
        self.gamma = None
        self.beta = None


def bn_partials(y):
    """Standalone batch-statistics pass over y [M, C] (when not fused)."""
    from ._lib import lib
    M, C = y.shape
    nchunk, rpc = reduce_chunks(M, C), lib.nsm_reduce_rows(M, C)
    part = Partials(empty(nchunk * 2 * C, device=y.device), nchunk, rpc)
    call("nsm_bn_stats", ptr(y), y.stride(0), M, C, ptr(part.buf), nchunk, dt(y), stream())
    return part


MERGE_ABOVE = int(os.environ.get("NSM_MERGE_ABOVE", "1024"))  # partial chunks beyond which a parallel first-level merge runs


def merged(part, M, C):
    """Partials with at most MERGE_ABOVE chunks (cached on the Partials)."""
    if part.nchunk <= MERGE_ABOVE:
        return part
    if part._merged is None:
        G = -(-part.nchunk // MERGE_ABOVE)
        n2 = -(-part.nchunk // G)
        buf = empty(n2 * (2 if part.rpc else 3) * C, device=part.buf.device)
        call("nsm_bn_partials_merge", ptr(part.buf), part.nchunk, part.rpc, M, C, G, ptr(buf),
             stream())
        part._merged = Partials(buf, n2, part.rpc * G)
    return part._merged


def _finalize(part, M, C, bn_mod, c_real, momentum, eps, n_updates, st, gamma, beta=None,
              bound=None):
    part = merged(part, M, C)
    if beta is None:
        beta = pad_vec(bn_mod.bias.detach(), C)
    track = bn_mod.track_running_stats
    slot, mul = bound if bound is not None else (None, 1.0)
    call("nsm_bn_finalize_train", ptr(part.buf), part.nchunk, part.rpc, M, C, c_real, ptr(gamma),
         ptr(beta), ptr(bn_mod.running_mean if track else None),
         ptr(bn_mod.running_var if track else None),
         ptr(bn_mod.num_batches_tracked if track else None), momentum, eps, n_updates,
         ptr(st.mean), ptr(st.invstd), ptr(st.scale), ptr(st.shift), ptr(slot), float(mul),
         stream())


def bn_train(y, bn_mod, c_real, momentum, eps, n_updates=1, part=None, gamma=None, beta=None,
             bound=None):
    """Train-mode BN: batch statistics of y [M, C] (given as fused GEMM
    partials, or computed here) + running-stat update in place on the module's
    buffers -> BNState with scale/shift for the fused apply. gamma / beta: the
    affine parameters padded to C (pad_vec'd here when not given).
    bound=(slot, mask_max): the zeroed operand-maximum slot receiving a bound
    of max|lrelu(BN(y))| * mask_max (nsm_bn_finalize_train), the scale source
    of bn_act_h2."""
    M, C = y.shape
    if part is None:
        part = bn_partials(y)
    st = BNState(C, y.device)
    st.part, st.nchunk = part, part.nchunk
    st.gamma = gamma if gamma is not None else pad_vec(bn_mod.weight.detach(), C)
    st.beta = beta if beta is not None else pad_vec(bn_mod.bias.detach(), C)
    _finalize(part, M, C, bn_mod, c_real, momentum, eps, n_updates, st, st.gamma, st.beta,
              bound=bound)
    return st


def bn_running_update(st, M, C, bn_mod, c_real, momentum, eps, n_updates=1):
    """Re-apply the running-stat update from saved partials (the conv5
    checkpoint recompute in the reference's backward)."""
    scratch = BNState(C, st.part.buf.device)
    _finalize(st.part, M, C, bn_mod, c_real, momentum, eps, n_updates, scratch, st.gamma, st.beta)


def bn_eval(bn_mod, C, c_real, eps, device, gamma=None, beta=None):
    st = BNState(C, device)
    st.gamma = gamma if gamma is not None else pad_vec(bn_mod.weight.detach(), C)
    beta = beta if beta is not None else pad_vec(bn_mod.bias.detach(), C)
    st.beta = beta
    bn_eval_into(st, bn_mod, C, c_real, eps)
    return st


def bn_eval_into(st, bn_mod, C, c_real, eps):
    """(Re)compute an eval BNState's vectors in place from the running
    statistics and st.gamma / st.beta (nsm_bn_finalize_eval)."""
    call("nsm_bn_finalize_eval", ptr(bn_mod.running_mean), ptr(bn_mod.running_var), ptr(st.gamma),
         ptr(st.beta), C, c_real, eps, ptr(st.mean), ptr(st.invstd), ptr(st.scale), ptr(st.shift),
         stream())


def bn_act(y, st, slope=0.2, res=None, out=None, mask=None, HW=0, amax=None):
    """lrelu(y*scale+shift) (* mask[b, c] with b = row // HW) (+ res).
    amax: operand-maximum slot receiving max|out| (of the fp32 values before a
    bf16 store's rounding)."""
    M, C = y.shape
    o = out if out is not None else like(M, C, y)
    assert res is None or res.dtype == y.dtype
    assert mask is None or HW > 0
    call("nsm_bn_act", ptr(y), y.stride(0), M, C, ptr(st.scale), ptr(st.shift), slope, ptr(mask),
         HW, ptr(res), res.stride(0) if res is not None else 0, ptr(o), o.stride(0), dt(y),
         ptr(amax), stream())
    return o


def bn_act_h2(y, st, slope=0.2, mask=None, HW=0, bound=None):
    """bn_act (fp32, no skip) written as an h2 tensor [M, 2C] float16
    (nsm_bn_act_h2); bound: the slot bn_train(bound=...) filled, its scale
    source."""
    M, C = y.shape
    assert y.dtype == F32 and bound is not None and (mask is None or HW > 0)
    o = torch.empty(M, 2 * C, dtype=H2, device=y.device)
    call("nsm_bn_act_h2", ptr(y), y.stride(0), M, C, ptr(st.scale), ptr(st.shift), slope,
         ptr(mask), HW, ptr(o), ptr(bound), stream())
    return o


def to_h2(x, amax, beta=1.0):
    """fp32 [rows, C] -> h2 tensor [rows, 2C] float16 (nsm_to_h2), scale source
    (amax slot, beta)."""
    rows, C = x.shape
    assert x.is_contiguous() and x.dtype == F32
    o = torch.empty(rows, 2 * C, dtype=H2, device=x.device)
    call("nsm_to_h2", ptr(x), rows, C, ptr(amax), float(beta), ptr(o), stream())
    return o


def conv1x1_h2(xh, wh, bias, cout_p, stats=True, amax=(None, None), tag=None):
    """1x1 conv on h2 operands (nsm_conv1x1_h2): xh [M, 2 cin_p] (bn_act_h2),
    wh the FWD h2 pack; amax = (scale source of xh, of wh). Returns (y fp32
    [M, cout_p], Partials|None)."""
    from ._lib import lib
    M, cin2 = xh.shape
    assert xh.dtype == H2 and wh.dtype == H2 and amax[0] is not None and amax[1] is not None
    y = empty(M, cout_p, device=xh.device)
    part = None
    if stats:
        rpc = int(lib.nsm_conv1x1_h2_rows(M, cout_p, cin2, 0))
        nchunk = -(-M // rpc)
        part = Partials(empty(nchunk * 2 * cout_p, device=xh.device), nchunk, rpc)
    ev = _probe(tag)
    call("nsm_conv1x1_h2", ptr(xh), M, cin2 // 2, ptr(wh), ptr(bias), cout_p, ptr(y), y.stride(0),
         ptr(part.buf) if part is not None else None, ptr(amax[0]), ptr(amax[1]), stream())
    if ev is not None:
        ev.record()
    return y, part


def conv1x1_wgrad_h2(dyh, xh, cin, cout, dw, amax=(None, None), tag=None):
    """dw [cout, cin, 1, 1] <- sum_p dy (x) x over h2 pixel rows
    (nsm_conv1x1_wgrad_h2); amax = (scale source of dyh, of xh)."""
    from ._lib import lib
    M, cout2 = dyh.shape
    cin_p, cout_p = xh.shape[1] // 2, cout2 // 2
    assert xh.shape[0] == M and dyh.dtype == H2 and xh.dtype == H2
    n = int(lib.nsm_conv1x1_wgrad_h2_ws(M, cin_p, cout_p))
    ws = empty(max(n, 1), device=dyh.device)
    ev = _probe(tag)
    call("nsm_conv1x1_wgrad_h2", ptr(dyh), ptr(xh), M, cin_p, cout_p, cin, cout, ptr(dw), ptr(ws),
         n, ptr(amax[0]), ptr(amax[1]), stream())
    if ev is not None:
        ev.record()


def bn_bwd(g, y, st, HW, mask, c_real, dgamma, dbeta, dbias_prev, slope=0.2, part=None,
           defer=False, amax=None, h2=None):
    """Backward through lrelu(.)*mask after a train-mode BN: returns dy
    (grad wrt the BN input) and writes dgamma/dbeta/dbias_prev (real chans).
    part=(partial, nchunk): the {sum dz, sum dz*xhat} partials already written
    by g's producer (GradPart), so the reduce pass is skipped. defer=True:
    DeferredBnBwd(g, coef) instead of dy (its consumer forms dy itself).
    amax: operand-maximum slot receiving max|dy| (fp32).
    h2=(k1dz slot, bound slot), both zeroed (fp32): dy is returned as an h2
    tensor [M, 2C] (nsm_bn_bwd_apply_h2) scaled from the bound the finalize
    derives from max|k1 dz| (recorded by the reduce pass, or by g's producer
    when part is given: pass it the same k1dz slot)."""
    M, C = y.shape
    assert g.dtype == y.dtype
    k1dz, bound = h2 if h2 is not None else (None, None)
    if part is None:
        nchunk = reduce_chunks(M, C)
        partial = empty(nchunk * 2 * C, device=y.device)
        call("nsm_bn_bwd_reduce", ptr(g), g.stride(0), ptr(y), y.stride(0), M, C, HW,
             ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(st.invstd),
             ptr(partial), nchunk, dt(y), ptr(k1dz), stream())
    else:
        partial, nchunk = part
        if nchunk > SUM_ROWS_ABOVE:
            G = -(-nchunk // SUM_ROWS_ABOVE)
            n2 = -(-nchunk // G)
            buf = empty(n2 * 2 * C, device=y.device)
            call("nsm_sum_rows", ptr(partial), nchunk, 2 * C, G, ptr(buf), stream())
            partial, nchunk = buf, n2
    coef = empty(3 * C, device=y.device)
    call("nsm_bn_bwd_finalize", ptr(partial), nchunk, M, C, c_real, ptr(st.gamma), ptr(st.invstd),
         ptr(dgamma), ptr(dbeta), ptr(dbias_prev), ptr(coef), ptr(k1dz), ptr(bound), stream())
    if defer:
        return DeferredBnBwd(g, coef)
    if h2 is not None:
        assert y.dtype == F32
        dyh = torch.empty(M, 2 * C, dtype=H2, device=y.device)
        call("nsm_bn_bwd_apply_h2", ptr(g), g.stride(0), ptr(y), y.stride(0), M, C, HW,
             ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(coef), ptr(dyh),
             ptr(bound), stream())
        return dyh
    dy = like(M, C, y)
    call("nsm_bn_bwd_apply", ptr(g), g.stride(0), ptr(y), y.stride(0), M, C, HW, ptr(st.scale),
         ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(coef), ptr(dy), dy.stride(0), dt(y),
         ptr(amax), stream())
    return dy


SUM_ROWS_ABOVE = int(os.environ.get("NSM_SUM_ROWS_ABOVE", "512"))  # BN-backward partial rows beyond which nsm_sum_rows merges them first


def conv1x1_dgrad_bn_bwd(dY2, B, H, W, w2d, y, st, mask, c_real, dgamma, dbeta, dbias_prev,
                         recompute, slope=0.2, tag=None, defer=False, amax=(None, None),
                         amax_out=None, bound=None):
    """dY1 of a DoubleConv's first BN from dY2 (grad wrt the 1x1 conv output):
    the 1x1 input gradient dA1 = dY2 W2 with the BN + LeakyReLU + Dropout2d
    backward in its epilogue (nsm_conv1x1_dgrad_bnbwd) — the same values as
    bn_bwd(conv_fwd(dY2, w2d, ...), y, ...) without the separate reduce pass.
    recompute=True: a partials-only GEMM pass, then the GEMM again writing dY1
    (dA1 never stored); False: one pass storing dA1 + partials, then
    nsm_bn_bwd_apply. defer=True (with recompute=False): DeferredBnBwd(dA1,
    coef) instead of dy, the apply pass left to the consumer. amax = (max|dY2|,
    max|w2d|) slots: the fp32 GEMM passes run the f16x2 split. amax_out: slot
    receiving max|dY1| (fp32; the h2 scale source of its Winograd transforms).
    bound=(k1dz slot, bound slot), both zeroed (bf16, defer): the GEMM records
    max|scale*dz| and the finalize derives the dY1 bound from it, the scale
    source of wino_dual_bn_f16."""
    from ._lib import lib
    M, cop = dY2.shape
    C = y.shape[1]
    if dY2.dtype != y.dtype or w2d.dtype != y.dtype:
        raise TypeError("conv1x1_dgrad_bn_bwd: dY2, packed weight and Y1 must share a dtype")
    dtc = dt(y)
    nchunk = int(lib.nsm_conv1x1_bnbwd_chunks(B, H, W, C, cop, dtc))
    partial = empty(nchunk * 2 * C, device=y.device)
    dA1 = None if recompute else like(M, C, y)
    args = (ptr(dY2), dY2.stride(0), B, H, W, cop, ptr(w2d), C, ptr(y), y.stride(0),
            ptr(st.scale), ptr(st.shift), ptr(st.mean), ptr(st.invstd), ptr(mask), slope)
    ev = _probe(tag)
    am = _pair(amax) if dtc == NSM_F32 else (None, None)
    k1dz, bslot = bound if bound is not None else (None, None)
    assert bound is None or (dtc != NSM_F32 and not recompute)
    call("nsm_conv1x1_dgrad_bnbwd", *args, 0 if recompute else 1, ptr(partial), None, ptr(dA1),
         dA1.stride(0) if dA1 is not None else 0, dtc, *am, ptr(k1dz), stream())
    if nchunk > SUM_ROWS_ABOVE:
        G = -(-nchunk // SUM_ROWS_ABOVE)
        n2 = -(-nchunk // G)
        buf = empty(n2 * 2 * C, device=y.device)
        call("nsm_sum_rows", ptr(partial), nchunk, 2 * C, G, ptr(buf), stream())
        partial, nchunk = buf, n2
    coef = empty(3 * C, device=y.device)
    call("nsm_bn_bwd_finalize", ptr(partial), nchunk, M, C, c_real, ptr(st.gamma), ptr(st.invstd),
         ptr(dgamma), ptr(dbeta), ptr(dbias_prev), ptr(coef), ptr(k1dz), ptr(bslot), stream())
    if defer and not recompute:
        if ev is not None:
            ev.record()
        return DeferredBnBwd(dA1, coef)
    dy = like(M, C, y)
    if recompute:
        call("nsm_conv1x1_dgrad_bnbwd", *args, 2, None, ptr(coef), ptr(dy), dy.stride(0), dtc,
             *am, ptr(amax_out) if dtc == NSM_F32 else None, stream())
    else:
        call("nsm_bn_bwd_apply", ptr(dA1), dA1.stride(0), ptr(y), y.stride(0), M, C, H * W,
             ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(coef), ptr(dy),
             dy.stride(0), dtc, ptr(amax_out), stream())
    if ev is not None:
        ev.record()
    return dy


def conv1x1_dgrad_bn_bwd_h2(dY2h, HW, w2dh, y, st, mask, c_real, dgamma, dbeta, dbias_prev,
                            recompute, slope=0.2, tag=None, amax=(None, None), amax_out=None,
                            h2_out=None, defer=False):
    """conv1x1_dgrad_bn_bwd on h2 operands (nsm_conv1x1_dgrad_bnbwd_h2): dY2h
    [M, 2 cop] (bn_bwd(h2=...)), w2dh the DGRAD h2 pack; amax = (scale source
    of dY2h, of w2dh). HW: pixels per image (the Dropout2d mask row).
    h2_out=(k1dz slot, bound slot), zeroed (recompute=False only): dY1 is
    returned as an h2 tensor (nsm_bn_bwd_apply_h2) for the direct 3x3's h2
    gradients, or with defer=True as DeferredBnBwd(dA1, coef) whose consumer
    (wino_dual_input_bn_h2) forms dY1 under the bound slot's scale."""
    assert h2_out is None or not recompute
    assert not defer or h2_out is not None
    k1dz, bound = h2_out if h2_out is not None else (None, None)
    from ._lib import lib
    M, cop2 = dY2h.shape
    C = y.shape[1]
    assert dY2h.dtype == H2 and w2dh.dtype == H2 and y.dtype == F32
    nchunk = -(-M // int(lib.nsm_conv1x1_h2_rows(M, C, cop2, 1)))
    partial = empty(nchunk * 2 * C, device=y.device)
    dA1 = None if recompute else like(M, C, y)
    args = (ptr(dY2h), M, cop2 // 2, ptr(w2dh), C, ptr(y), y.stride(0), ptr(st.scale),
            ptr(st.shift), ptr(st.mean), ptr(st.invstd), ptr(mask), HW, slope)
    ev = _probe(tag)
    call("nsm_conv1x1_dgrad_bnbwd_h2", *args, 0 if recompute else 1, ptr(partial), None, ptr(dA1),
         dA1.stride(0) if dA1 is not None else 0, ptr(amax[0]), ptr(amax[1]), None, ptr(k1dz),
         stream())
    if nchunk > SUM_ROWS_ABOVE:
        G = -(-nchunk // SUM_ROWS_ABOVE)
        n2 = -(-nchunk // G)
        buf = empty(n2 * 2 * C, device=y.device)
        call("nsm_sum_rows", ptr(partial), nchunk, 2 * C, G, ptr(buf), stream())
        partial, nchunk = buf, n2
    coef = empty(3 * C, device=y.device)
    call("nsm_bn_bwd_finalize", ptr(partial), nchunk, M, C, c_real, ptr(st.gamma), ptr(st.invstd),
         ptr(dgamma), ptr(dbeta), ptr(dbias_prev), ptr(coef), ptr(k1dz), ptr(bound), stream())
    if defer:
        if ev is not None:
            ev.record()
        return DeferredBnBwd(dA1, coef)
    if h2_out is not None:
        dyh = torch.empty(M, 2 * C, dtype=H2, device=y.device)
        call("nsm_bn_bwd_apply_h2", ptr(dA1), dA1.stride(0), ptr(y), y.stride(0), M, C, HW,
             ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(coef), ptr(dyh),
             ptr(bound), stream())
        if ev is not None:
            ev.record()
        return dyh
    dy = like(M, C, y)
    if recompute:
        call("nsm_conv1x1_dgrad_bnbwd_h2", *args, 2, None, ptr(coef), ptr(dy), dy.stride(0),
             ptr(amax[0]), ptr(amax[1]), ptr(amax_out), None, stream())
    else:
        call("nsm_bn_bwd_apply", ptr(dA1), dA1.stride(0), ptr(y), y.stride(0), M, C, HW,
             ptr(st.scale), ptr(st.shift), slope, ptr(mask), ptr(st.mean), ptr(coef), ptr(dy),
             dy.stride(0), NSM_F32, ptr(amax_out), stream())
    if ev is not None:
        ev.record()
    return dy


# ---- resampling --------------------------------------------------------------
def avgpool2(x, B, H, W):
    C = x.shape[1]
    y = like(B * (H // 2) * (W // 2), C, x)
    call("nsm_avgpool2_fwd", ptr(x), B, H, W, C, ptr(y), dt(x), stream())
    return y


def _bnred(kind, B, H, W, C, bnred, device, slope=0.2):
    """(extra C-ABI args, (partial, nchunk)) for a gradient producer that also
    reduces the BN backward of bnred = (y2, BNState[, k1dz slot]); (None, None)
    when the fused form does not apply to this shape. The k1dz slot receives
    max|scale * dz| (bn_bwd(h2=...))."""
    from ._lib import lib
    if bnred is None:
        return None, None
    n = int(lib.nsm_bnred_chunks(kind, B, H, W, C))
    if n <= 0:
        return None, None
    y2, st = bnred[:2]
    k1dz = bnred[2] if len(bnred) > 2 else None
    partial = empty(n * 2 * C, device=device)
    return ((ptr(y2), ptr(st.scale), ptr(st.shift), ptr(st.mean), ptr(st.invstd), slope,
             ptr(partial), ptr(k1dz)), (partial, n))


def avgpool2_bwd_add(dy, B, H, W, skip, bnred=None):
    """AvgPool2d backward + skip-gradient add. bnred=(y2, BNState): returns
    (dx, part) with the BN-backward partials of dx for that BN (part None
    when the fused form does not apply)."""
    C = dy.shape[1]
    dx = like(B * H * W, C, dy)
    assert skip is None or skip.dtype == dy.dtype
    extra, part = _bnred(0, B, H, W, C, bnred, dy.device)
    if extra is None:
        call("nsm_avgpool2_bwd_add", ptr(dy), B, H, W, C, ptr(skip), ptr(dx), dt(dy), stream())
    else:
        call("nsm_avgpool2_bwd_add_bnred", ptr(dy), B, H, W, C, ptr(skip), ptr(dx), dt(dy),
             *extra, stream())
    return dx if bnred is None else (dx, part)


def resize(x, B, Hi, Wi, Ho, Wo):
    C = x.shape[-1]
    y = like(B * Ho * Wo, C, x)
    call("nsm_resize_fwd", ptr(x), B, Hi, Wi, C, ptr(y), Ho, Wo, dt(x), stream())
    return y


def resize_bwd(dy, B, Hi, Wi, Ho, Wo, bnred=None):
    """bnred: as avgpool2_bwd_add (returns (dx, part))."""
    C = dy.shape[-1]
    dx = like(B * Hi * Wi, C, dy)
    extra, part = _bnred(1, B, Hi, Wi, C, bnred, dy.device)
    if extra is None:
        call("nsm_resize_bwd", ptr(dy), B, Hi, Wi, C, ptr(dx), Ho, Wo, dt(dy), stream())
    else:
        call("nsm_resize_bwd_bnred", ptr(dy), B, Hi, Wi, C, ptr(dx), Ho, Wo, dt(dy), *extra,
             stream())
    return dx if bnred is None else (dx, part)


class Lazy:
    """A decoder block output z = lrelu(bn2(Y2)) (+ res) that is not
    materialised: the next upsample computes it on load (resize_act)."""
    __slots__ = ("y2", "st", "res")

    def __init__(self, y2, st, res):
        self.y2, self.st, self.res = y2, st, res

    def materialise(self, slope=0.2):
        return bn_act(self.y2, self.st, slope, res=self.res)


def resize_act(z, B, Hi, Wi, Ho, Wo, slope=0.2):
    """resize of a Lazy block output (nsm_resize_fwd_act)."""
    C = z.y2.shape[-1]
    y = like(B * Ho * Wo, C, z.y2)
    call("nsm_resize_fwd_act", ptr(z.y2), B, Hi, Wi, C, ptr(y), Ho, Wo, ptr(z.st.scale),
         ptr(z.st.shift), slope, ptr(z.res), dt(z.y2), stream())
    return y


def up2_resize_act(z, B, h, w, th, tw, slope=0.2):
    """up x2 + resize of a Lazy block output (nsm_up2_resize_fwd_act), or None
    when the row-blocked kernel does not take this geometry."""
    if not (tw <= 2048 and th * 2 >= 2 * h - 1 and tw * 2 >= 2 * w - 1):
        return None
    C = z.y2.shape[-1]
    y = like(B * th * tw, C, z.y2)
    call("nsm_up2_resize_fwd_act", ptr(z.y2), B, h, w, C, ptr(y), th, tw, ptr(z.st.scale),
         ptr(z.st.shift), slope, ptr(z.res), dt(z.y2), stream())
    return y


def bn_act_pool(y, st, B, H, W, slope=0.2, amax=None):
    """(z, avgpool2(z)) with z = lrelu(y*scale+shift), one read of y.
    amax: operand-maximum slot receiving max|pooled| (fp32)."""
    C = y.shape[-1]
    z = like(B * H * W, C, y)
    pooled = like(B * (H // 2) * (W // 2), C, y)
    call("nsm_bn_act_pool", ptr(y), B, H, W, C, ptr(st.scale), ptr(st.shift), slope, ptr(z),
         ptr(pooled), dt(y), ptr(amax), stream())
    return z, pooled


def up2_resize(x, B, h, w, th, tw):
    """bilinear x2 (align_corners) then resize to (th, tw), one pass."""
    C = x.shape[-1]
    y = like(B * th * tw, C, x)
    call("nsm_up2_resize_fwd", ptr(x), B, h, w, C, ptr(y), th, tw, dt(x), stream())
    return y


def up2_resize_bwd(dy, B, h, w, th, tw, bnred=None):
    """bnred: as avgpool2_bwd_add (returns (dx, part))."""
    C = dy.shape[-1]
    dx = like(B * h * w, C, dy)
    extra, part = _bnred(2, B, h, w, C, bnred, dy.device)
    if extra is None:
        call("nsm_up2_resize_bwd", ptr(dy), B, h, w, C, ptr(dx), th, tw, dt(dy), stream())
    else:
        call("nsm_up2_resize_bwd_bnred", ptr(dy), B, h, w, C, ptr(dx), th, tw, dt(dy), *extra,
             stream())
    return dx if bnred is None else (dx, part)


# ---- boundary ----------------------------------------------------------------
def input_prep(x, cp, dtype=F32, amax=None):
    """fp32 NCHW model input -> NHWC [B*H/2*W/2, cp] activations in `dtype`.
    amax: operand-maximum slot receiving max|out| (fp32)."""
    B, C, H, W = x.shape
    out = torch.empty(B * (H // 2) * (W // 2), cp, dtype=dtype, device=x.device)
    call("nsm_input_prep", ptr(x), B, C, H, W, ptr(out), cp, dt(out),
         ptr(amax) if dtype == F32 else None, stream())
    return out


def input_prep_h2(x, cp, amax):
    """input_prep written as an h2 tensor [B*H/2*W/2, 2 cp] (nsm_input_prep_h2);
    amax: a zeroed slot the call fills with max|x|, its scale source."""
    B, C, H, W = x.shape
    out = torch.empty(B * (H // 2) * (W // 2), 2 * cp, dtype=H2, device=x.device)
    call("nsm_input_prep_h2", ptr(x), B, C, H, W, ptr(out), cp, ptr(amax), stream())
    return out


def conv3x3_h2(xh, B, H, W, wh, bias, cout_p, stats=True, amax=(None, None), tag=None):
    """Direct 3x3 conv (pad 1) on h2 operands (nsm_conv3x3_h2): xh [B*H*W,
    2 cin_p], wh a kind-5 3x3 pack (FWD; DGRAD with bias None for the input
    gradient); amax = (scale source of xh, of wh). Returns (y fp32, Partials|None)."""
    from ._lib import lib
    M, cin2 = xh.shape
    assert xh.dtype == H2 and wh.dtype == H2 and M == B * H * W
    y = empty(M, cout_p, device=xh.device)
    part = None
    if stats:
        rpc = int(lib.nsm_conv3x3_h2_rows(M, cout_p))
        part = Partials(empty(-(-M // rpc) * 2 * cout_p, device=xh.device), -(-M // rpc), rpc)
    ev = _probe(tag)
    call("nsm_conv3x3_h2", ptr(xh), B, H, W, cin2 // 2, ptr(wh), ptr(bias), cout_p, ptr(y),
         y.stride(0), ptr(part.buf) if part is not None else None, ptr(amax[0]), ptr(amax[1]),
         stream())
    if ev is not None:
        ev.record()
    return y, part


def conv3x3_wgrad_h2(dyh, xh, B, H, W, cin, cout, dw, amax=(None, None), tag=None):
    """dw [cout, cin, 3, 3] of a direct 3x3 conv from its h2 output gradient and
    h2 input (nsm_conv3x3_wgrad_h2); amax = (scale source of dyh, of xh)."""
    from ._lib import lib
    cin_p, cout_p = xh.shape[1] // 2, dyh.shape[1] // 2
    n = int(lib.nsm_conv3x3_wgrad_h2_ws(B, H, W, cin_p, cout_p))
    ws = empty(max(n, 1), device=dyh.device)
    ev = _probe(tag)
    call("nsm_conv3x3_wgrad_h2", ptr(dyh), ptr(xh), B, H, W, cin_p, cout_p, cin, cout, ptr(dw),
         ptr(ws), n, ptr(amax[0]), ptr(amax[1]), stream())
    if ev is not None:
        ev.record()


def input_grad(dX, B, C, H, W):
    dx = empty(B, C, H, W, device=dX.device)
    call("nsm_input_grad", ptr(dX), B, C, H, W, dX.shape[1], ptr(dx), dt(dX), stream())
    return dx


def head_fwd(z, B, Rh, Rw, w10, b10):
    out = empty(B, 1, 2 * Rh, 2 * Rw, device=z.device)
    call("nsm_head_fwd", ptr(z), z.stride(0), B, Rh, Rw, ptr(w10), ptr(b10), ptr(out), dt(z),
         stream())
    return out


def head_bwd(gout, out, z, B, Rh, Rw, w10, dw10, db10):
    from ._lib import lib
    nblk = lib.nsm_head_bwd_blocks(B, Rh, Rw)
    partial = empty(nblk * 68, device=z.device)
    dz = torch.empty(*z.shape, dtype=z.dtype, device=z.device)
    call("nsm_head_bwd", ptr(gout), ptr(out), ptr(z), z.stride(0), B, Rh, Rw, ptr(w10), ptr(dz),
         ptr(partial), ptr(dw10), ptr(db10), dt(z), stream())
    return dz


# ---- VGG19 perceptual loss ----------------------------------------------------
def vgg_prep(output, target, mean, denom):
    """[2B*H*W, 32] NHWC input of the VGG stack (output images, then target)."""
    B, _, H, W = output.shape
    out = empty(2 * B * H * W, 32, device=output.device)
    call("nsm_vgg_prep", ptr(output), ptr(target), B, H, W, float(mean), float(denom), ptr(out),
         stream())
    return out


def maxpool2(x, B, H, W):
    C = x.shape[1]
    y = empty(B * (H // 2) * (W // 2), C, device=x.device)
    call("nsm_maxpool2_fwd", ptr(x), B, H, W, C, ptr(y), stream())
    return y


def l1_mean(a, b, alpha=1.0):
    """alpha * mean|a - b| over all elements, as a 0-dim device tensor."""
    from ._lib import lib
    n = a.numel()
    assert b.numel() == n and a.is_contiguous() and b.is_contiguous()
    partial = empty(int(lib.nsm_loss_blocks(n)), device=a.device)
    out = torch.empty((), dtype=F32, device=a.device)
    call("nsm_l1_loss_fwd", ptr(a), ptr(b), n, float(alpha), ptr(partial), ptr(out), stream())
    return out
