"""Weight layouts of one step, prepared in ONE launch (include/nsm.h
`nsm_prep_weights`).

Every convolution of the U-Net (Unetmodel.py:21,26) reads its weight in an
MFMA operand layout: packed [co][tap][ci] for the direct forward, flipped
[ci][tap'][co] for the input gradient, Winograd-domain U = G g G^T (forward and
rotated for the input gradient), bias / BN affine vectors padded to the NHWC
channel count. The weights change every optimizer step, so these layouts are
rebuilt every step: `StepWeights` writes all of them with one kernel launch
into persistent buffers (the job table holds raw pointers, uploaded once per
parameter storage), instead of ~40 small launches. `LazyBlockWeights` is the
per-call path (a standalone DoubleConv).
"""
import ctypes
import os

import torch

from . import ops
from ._lib import call, lib, ptr, stream


class NsmPrepJob(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("a", ctypes.c_int * 7), ("base", ctypes.c_longlong),
                ("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("amax", ctypes.c_void_p)]


KIND_PACK_F32, KIND_PACK_BF16, KIND_WINO, KIND_PAD, KIND_WINO_H2, KIND_PACK_H2 = 0, 1, 2, 3, 4, 5
KIND_WINO_F16 = 6
KIND_PACK_F16 = 7   # IEEE half pack (the fp16-autocast mode's direct convolutions)
# NSM_H2=0: the fp32 training step keeps fp32 Winograd operands (the GEMMs
# split them in-kernel, nsm_conv_split16.inc) instead of the pre-split h2
# tensors their producers write (nsm_conv_h2.inc)
H2_WINO = os.environ.get("NSM_H2", "1") != "0"
# NSM_H2_1X1=0: the DoubleConv 1x1 convolutions of the fp32 training step keep
# fp32 operands (register-path f16x2 split) instead of h2 operands written by
# their producers (csrc/nsm_conv_h2d.inc); on with the h2 Winograd operands
H2_1X1 = os.environ.get("NSM_H2_1X1", "1") != "0"
# NSM_BF16_WINO=0: the bf16 training step's 3x3 forward at >= NSM_BF16_WINO_MIN
# input channels stays on the direct implicit GEMM instead of Winograd F(4x4)
# on single-plane scaled f16 operands (ops.conv3x3_wino_f16). Measured (B=64
# step, A/B on one box): off 1240-1245, conv6 only (>= 1024) 1267-1270,
# conv5-conv7 (>= 512) 1276-1279 frames/s; conv6's forward 3.87 -> 2.5 ms
# (input transform 0.38 + GEMM 1.53 + output transform 0.61: the fp32 M,
# 2.25 x 4 B per output element, bounds the last two)
BF16_WINO = os.environ.get("NSM_BF16_WINO", "1") != "0"
BF16_WINO_MIN = int(os.environ.get("NSM_BF16_WINO_MIN", "512"))
# NSM_BF16_WINO_EVAL=0: the bf16 eval forward (configs[4]'s 1080p bf16 line)
# keeps its 3x3 convs on the direct implicit GEMM instead of the same F(4x4)
# f16 Winograd (BN + LeakyReLU in the output transform)
BF16_WINO_EVAL = os.environ.get("NSM_BF16_WINO_EVAL", "1") != "0"


def bf16_wino(cip, dtype, training):
    """True when a DoubleConv's 3x3 forward runs ops.conv3x3_wino_f16."""
    return (BF16_WINO and (training or BF16_WINO_EVAL) and dtype == torch.bfloat16
            and cip >= BF16_WINO_MIN and cip % 128 == 0)


PREP_ITEMS = 512   # items per block of nsm_prep_weights (nsm_prep_items rounds to it)


def run_jobs(jobs, device):
    """One nsm_prep_weights call over a list of NsmPrepJob (consecutive bases,
    shared jobs with a[6] = the source job's first block + 1): the table and
    the max|w| word per block made here (tests, standalone layouts)."""
    total = sum(int(lib.nsm_prep_items(ctypes.byref(j))) for j in jobs)
    raw = (NsmPrepJob * len(jobs))(*jobs)
    table = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8).to(device)
    pmax = torch.empty(total // PREP_ITEMS, dtype=torch.int32, device=device)
    max_pass = int(any(j.kind in (KIND_WINO_H2, KIND_PACK_H2, KIND_WINO_F16) for j in jobs))
    call("nsm_prep_weights", ptr(table), len(jobs), total, max_pass, ptr(pmax), None, 0, None, 0,
         stream())
    return table, pmax


class LazyBlockWeights:
    """Layouts of one DoubleConv computed on demand (one launch each)."""

    def __init__(self, blk, dtype):
        self.blk, self.dtype = blk, dtype
        self.cip = ops.pad32(blk.conv[0].in_channels)
        self.cop = ops.pad32(blk.conv[4].out_channels)

    def vec(self, name):
        c0, bn1, c4, bn2 = (self.blk.conv[i] for i in (0, 1, 4, 5))
        t, n = {"b1": (c0.bias, self.cip), "g1": (bn1.weight, self.cip), "be1": (bn1.bias, self.cip),
                "b2": (c4.bias, self.cop), "g2": (bn2.weight, self.cop),
                "be2": (bn2.bias, self.cop)}[name]
        return ops.pad_vec(t.detach(), n)

    def U1(self, tile, flip):
        return ops.wino_weight(self.blk.conv[0].weight.detach(), self.cip, self.cip, flip=flip,
                               tile=tile)

    def amax_U1(self, flip):
        return None      # no recorded maximum: the bf16 split runs

    def amax_w2(self, mode):
        return None

    def amax_w1(self, mode):
        return None

    def w1(self, mode):
        return ops.pack_conv_weight(self.blk.conv[0].weight.detach(), self.cip, self.cip, mode,
                                    self.dtype)

    def w2(self, mode):
        return ops.pack_conv_weight(self.blk.conv[4].weight.detach(), self.cop, self.cip, mode,
                                    self.dtype)


class _PreparedBlock:
    __slots__ = ("t",)

    def __init__(self):
        self.t = {}

    def vec(self, name):
        return self.t[name]

    def U1(self, tile, flip):
        return self.t[("U1", flip)]

    def amax_U1(self, flip):
        """max|U| of the step's Winograd weight (written by the prep launch);
        for an h2 U (float16 storage) max|w| of the filters, its scale source."""
        return self.t.get(("amaxU1", flip))

    def amax_w2(self, mode):
        """max|packed 1x1 weight| (fp32 packs; written by the prep launch)."""
        return self.t.get(("amaxw2", mode))

    def amax_w1(self, mode):
        """max|packed direct 3x3 weight| (fp32 packs; written by the prep launch)."""
        return self.t.get(("amaxw1", mode))

    def w1(self, mode):
        return self.t[("w1", mode)]

    def w2(self, mode):
        return self.t[("w2", mode)]

    def Uf16(self, flip=False):
        """the bf16 path's F(4x4) filters (prep kind 6; flip: the input
        gradient's), or None"""
        return self.t.get("Uf16d" if flip else "Uf16")

    def amax_Uf16(self):
        return self.t.get("amaxUf16")


class StepWeights:
    """All layouts of a Unet for one (dtype, input size, train/eval) signature.
    `run()` launches the single preparation kernel; `block(k)` returns the
    layouts of DoubleConv k. Valid while the parameters keep their storage
    (`valid()` checks the pointers)."""

    def __init__(self, mod, dtype, shapes, training, wino_min, wino_tile, h2=False):
        dev = mod.conv10.weight.device
        self.params = [p for p in mod.parameters()]
        self.ptrs = [p.data_ptr() for p in self.params]
        self.blocks = {}
        jobs, keep = [], []
        base = 0
        # slots: Winograd U (fwd, dgrad) and the packed 1x1 weights (fwd, dgrad)
        # (fwd + dgrad of each block's 3x3 and 1x1 weight)
        n_wino = len(shapes) * 4
        # per-step maxima of the Winograd weights (the f16x2 GEMMs' operand
        # scales), zeroed by run() before the prep launch refills them
        self.amax = ops.amax_slots(max(n_wino, 1), dev)
        n_am = 0
        first = min(shapes)   # the block whose input the forward writes (conv2)

        def add(kind, a, src, shape_numel, out_dtype, amax=None):
            nonlocal base
            out = torch.empty(shape_numel, dtype=out_dtype, device=dev)
            j = NsmPrepJob()
            j.kind = kind
            for i, v in enumerate(a):
                j.a[i] = int(v)
            if kind in (KIND_WINO_H2, KIND_PACK_H2, KIND_WINO_F16) and len(a) > 6 and a[6]:
                # shares the maximum of the job just before it (same filters):
                # a[6] = that job's first block + 1 (include/nsm.h)
                j.a[6] = int(jobs[-1].base // PREP_ITEMS + 1)
            j.base = base
            j.src = src.data_ptr()
            j.dst = out.data_ptr()
            j.amax = amax.data_ptr() if amax is not None else None
            n = int(lib.nsm_prep_items(ctypes.byref(j)))
            assert n > 0, (kind, a)
            base += n
            jobs.append(j)
            keep.append(out)
            return out

        for k, (h, w) in shapes.items():
            blk = mod.block(k)
            c0, bn1, c4, bn2 = (blk.conv[i] for i in (0, 1, 4, 5))
            ci, co = c0.in_channels, c4.out_channels
            cip, cop = ops.pad32(ci), ops.pad32(co)
            pb = _PreparedBlock()
            for name, t, n in (("b1", c0.bias, cip), ("g1", bn1.weight, cip), ("be1", bn1.bias, cip),
                               ("b2", c4.bias, cop), ("g2", bn2.weight, cop),
                               ("be2", bn2.bias, cop)):
                pb.t[name] = (t.detach() if t.numel() == n else
                              add(KIND_PAD, (t.numel(), n), t, n, torch.float32))
            pk = {torch.bfloat16: KIND_PACK_BF16, ops.F16S: KIND_PACK_F16}.get(dtype, KIND_PACK_F32)
            modes = (ops.PACK_FWD, ops.PACK_DGRAD) if training else (ops.PACK_FWD,)
            if cip >= wino_min and dtype == torch.float32:
                tile = wino_tile(cip, h, w)
                for flip in ((False, True) if training else (False,)):
                    if h2 and training and flip:
                        # max|w| of the same filters: the un-flipped job's slot,
                        # filled once (a[6] = 1: phase 0 skips this job)
                        am = pb.t[("amaxU1", False)]
                    else:
                        am = ops.amax_slot(self.amax, n_am)
                        n_am += 1
                    pb.t[("amaxU1", flip)] = am
                    if h2 and training:   # pre-split U [alpha^2][cip][2 cip] float16 (nsm_conv_h2.inc)
                        pb.t[("U1", flip)] = add(KIND_WINO_H2, (ci, ci, cip, cip, int(flip), tile,
                                                                int(flip)),
                                                 c0.weight, (tile + 2) ** 2 * cip * 2 * cip,
                                                 ops.H2, amax=am)
                    else:
                        pb.t[("U1", flip)] = add(KIND_WINO, (ci, ci, cip, cip, int(flip), tile),
                                                 c0.weight, (tile + 2) ** 2 * cip * cip,
                                                 torch.float32, amax=am)
            else:
                # the direct 3x3 (conv2) of the fp32 train step on h2 operands:
                # kind-5 packs, the DGRAD job sharing the FWD job's max|w| slot.
                # Only the first block: its input is the one written as h2
                # (ops.input_prep_h2); a later direct 3x3 (NSM_WINOGRAD=0 or a
                # raised NSM_WINO_MIN) reads the fp32 output of the block before
                h2_3x3 = h2 and training and H2_1X1 and k == first

                wf16 = bf16_wino(cip, dtype, training)
                if wf16:   # Winograd F(4x4) forward: single-plane f16 U (kind 6)
                    am = ops.amax_slot(self.amax, n_am)
                    n_am += 1
                    pb.t["amaxUf16"] = am
                    pb.t["Uf16"] = add(KIND_WINO_F16, (ci, ci, cip, cip, 0, 4, 0), c0.weight,
                                       36 * cip * cip, ops.H2, amax=am)
                    if training:   # the input gradient's filters (flipped; the forward job's slot)
                        pb.t["Uf16d"] = add(KIND_WINO_F16, (ci, ci, cip, cip, 1, 4, 1), c0.weight,
                                            36 * cip * cip, ops.H2, amax=am)
                for mode in modes:
                    if wf16:
                        continue   # forward and input gradient read Uf16 / Uf16d
                    am = None
                    if h2_3x3 and mode != ops.PACK_FWD:
                        am = pb.t[("amaxw1", ops.PACK_FWD)]
                    elif dtype == torch.float32:
                        am = ops.amax_slot(self.amax, n_am)
                        n_am += 1
                    if am is not None:
                        pb.t[("amaxw1", mode)] = am
                    if h2_3x3:
                        pb.t[("w1", mode)] = add(KIND_PACK_H2, (ci, ci, 9, cip, cip, mode,
                                                                int(mode != ops.PACK_FWD)),
                                                 c0.weight, 2 * cip * 9 * cip, ops.H2, amax=am)
                    else:
                        pb.t[("w1", mode)] = add(pk, (ci, ci, 9, cip, cip, mode), c0.weight,
                                                 cip * 9 * cip, dtype, amax=am)
            h2_1x1 = h2 and training and H2_1X1
            for mode in modes:
                am = None
                if h2_1x1 and mode != ops.PACK_FWD:
                    am = pb.t[("amaxw2", ops.PACK_FWD)]   # max|w| of the same weight
                elif dtype == torch.float32:
                    am = ops.amax_slot(self.amax, n_am)
                    n_am += 1
                if am is not None:
                    pb.t[("amaxw2", mode)] = am
                if h2_1x1:   # h2 packs [rows][2 K] float16 (prep kind 5, nsm_conv_h2d.inc)
                    pb.t[("w2", mode)] = add(KIND_PACK_H2, (co, ci, 1, cop, cip, mode,
                                                            int(mode != ops.PACK_FWD)),
                                             c4.weight, 2 * cop * cip, ops.H2, amax=am)
                else:
                    pb.t[("w2", mode)] = add(pk, (co, ci, 1, cop, cip, mode), c4.weight, cop * cip,
                                             dtype, amax=am)
            self.blocks[k] = pb
        # every slot handed out lies inside self.amax (a slice past its end
        # would aim the producers' atomics outside the buffer)
        assert n_am <= max(n_wino, 1), (n_am, n_wino)
        self.total = base
        self.njobs = len(jobs)
        # the max|w| pass (phase 0) runs only for the h2 jobs' scale sources
        self.max_pass = int(any(j.kind in (KIND_WINO_H2, KIND_PACK_H2, KIND_WINO_F16) for j in jobs))
        raw = (NsmPrepJob * len(jobs))(*jobs)
        host = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8)
        self.table = host.to(dev)
        self.keep = keep
        # one max|w| word per block of the launch (the h2 / f16 jobs' phase 0)
        self.pmax = torch.empty(self.total // PREP_ITEMS, dtype=torch.int32, device=dev)

    def valid(self, mod):
        ps = list(mod.parameters())
        return len(ps) == len(self.ptrs) and all(p.data_ptr() == q for p, q in zip(ps, self.ptrs))

    def run(self, act_slots=None):
        """The step's preparation launches. They zero this object's weight
        slots and `act_slots` (the forward's activation-maximum slots, an
        int32 tensor) before anything writes them: no fill launches."""
        call("nsm_prep_weights", ptr(self.table), self.njobs, self.total, self.max_pass,
             ptr(self.pmax), ptr(self.amax), self.amax.numel(), ptr(act_slots),
             act_slots.numel() if act_slots is not None else 0, stream())

    def block(self, k):
        return self.blocks[k]
