"""VGG19 perceptual loss (`customLoss.MultiLayerVGGLoss`, customLoss.py:7-90)
on the libnsm kernels — SURVEY.md §8(f) next-row #1.

The reference runs five prefixes `features[:idx+1]` for idx in (2, 7, 12, 21,
30) separately on output and on target (243.9 GMAC per 512^2 image). Here the
stack runs ONCE per call, incrementally, on output and target batched
together (2B images, 97.1 GMAC per image pair member), and taps the pre-ReLU
conv outputs on the way:

  * input: `nsm_vgg_prep` — clamp/nan_to_num, x3 repeat, (x-0.485)/(0.229+1e-8),
    NHWC padded to 32 channels (customLoss.py:44-62);
  * conv 3x3 + bias: Cin >= 128 through Winograd F(4x4,3x3) (`nsm_wino_*`), the
    rest through the implicit-GEMM conv; the ReLU after each conv is never a
    pass of its own: the next conv's operand loader (or Winograd input
    transform) applies max(x, 0);
  * MaxPool2d(2,2): `nsm_maxpool2_fwd` on the pre-ReLU tensor
    (max(relu(x)) == relu(max(x)); the pending ReLU moves past it);
  * per tap: `nsm_l1_loss_fwd` of the output half against the target half,
    scaled by the normalised layer weight.

Forward only (the reference computes it under no_grad and returns a detached
constant, customLoss.py:66-90). Weights: torchvision's `vgg19().features`
layout (`features.<idx>.weight/bias`); ImageNet weights are a download the
reference does at construction — offline, pass a local checkpoint
(`from_torchvision_checkpoint`) or a state_dict. Without one the module is
randomly initialised (He normal, zero bias): the VALUE is then not the
reference's (parity-unpinned offline), the work is identical.
"""
import os

import numpy as np
import torch
import torch.nn as nn

from . import ops
from ._lib import require_gpu
from .unet import WINO_TILE

# VGG19's 3x3 convs with >= 128 input channels run Winograd F(4x4,3x3)
WINOGRAD_MIN_CHANNELS = 128
# NSM_VGG_F16X2=0: the Winograd GEMMs on the exact three-way bf16 split (6
# products) instead of the f16x2 split (3 products; fp32 accuracy,
# nsm_conv_split16.inc) whose operand maxima the input transform (max|V|) and
# the plan (max|U|, once per weight set) record
VGG_F16X2 = os.environ.get("NSM_VGG_F16X2", "1") != "0"

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M",
             512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def _features():
    mods, c = [], 3
    for v in VGG19_CFG:
        if v == "M":
            mods.append(nn.MaxPool2d(2, 2))
        else:
            mods += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*mods)


class MultiLayerVGGLoss(nn.Module):
    def __init__(self, device=None, feature_layers=(2, 7, 12, 21, 30),
                 weights=(0.25, 0.25, 0.3, 0.1, 0.1), state_dict=None, seed=0):
        super().__init__()
        assert len(feature_layers) == len(weights), "feature_layers and weights differ in length"
        self.feature_layers = tuple(int(i) for i in feature_layers)
        for i in self.feature_layers:
            if not isinstance(_features()[i], nn.Conv2d):
                raise ValueError(f"feature layer {i} is not a conv output")
        self.features = _features()
        if state_dict is not None:
            self.load_vgg_state(state_dict)
        else:
            g = torch.Generator().manual_seed(seed)
            with torch.no_grad():
                for m in self.features:
                    if isinstance(m, nn.Conv2d):
                        fan_in = m.in_channels * 9
                        m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5)
                        m.bias.zero_()
        for p in self.features.parameters():
            p.requires_grad_(False)
        w = torch.tensor(weights)                        # customLoss.py:31-33 (float32)
        self.register_buffer("weights", w / w.sum())
        self._wts = (w / w.sum()).tolist()               # host copy: no device sync per call
        self.mean = 0.485
        # ATen: (std_tensor + 1e-8) in float32, then a true division
        self.denom = float(np.float32(0.229) + np.float32(1e-8))
        self._packed = None
        if device is not None:
            self.to(device)

    @classmethod
    def from_torchvision_checkpoint(cls, path, device=None, **kw):
        """Local copy of torchvision's vgg19 IMAGENET1K_V1 weights (.pth)."""
        sd = torch.load(path, map_location="cpu", weights_only=True)
        return cls(device, state_dict=sd, **kw)

    def load_vgg_state(self, sd):
        feats = {}
        for k, v in sd.items():
            if k.startswith("features."):
                k = k[len("features."):]
            elif k.startswith("classifier."):
                continue
            feats[k] = v
        self.features.load_state_dict(feats)
        self._packed = None

    def _plan(self):
        """Packed operands of every conv up to the last tap, cached while the
        weights do not change (frozen in the reference)."""
        key = tuple((m.weight.data_ptr(), m.weight._version) for m in self.features
                    if isinstance(m, nn.Conv2d))
        if self._packed is not None and self._packed[0] == key:
            return self._packed[1]
        plan, last = [], max(self.feature_layers)
        cin_p = 32
        for idx, m in enumerate(self.features):
            if idx > last:
                break
            if isinstance(m, nn.Conv2d):
                co = m.out_channels
                cop = ops.pad32(co)
                w, b = m.weight.detach().float(), ops.pad_vec(m.bias.detach().float(), cop)
                if cin_p >= WINOGRAD_MIN_CHANNELS:
                    U = ops.wino_weight(w, cop, cin_p, flip=False, tile=WINO_TILE)
                    op = ("wino", U, b, cop, ops.absmax(U) if VGG_F16X2 else None)
                else:
                    op = ("conv", ops.pack_conv_weight(w, cop, cin_p, ops.PACK_FWD), b, cop)
                plan.append((idx,) + op)
                cin_p = cop
            elif isinstance(m, nn.MaxPool2d):
                plan.append((idx, "pool"))
            else:
                plan.append((idx, "relu"))
        self._packed = (key, plan)
        return plan

    @torch.no_grad()
    def forward(self, output, target):
        require_gpu(output, "VGG loss input")
        o = output.detach().to(torch.float32).contiguous()
        t = target.detach().to(device=o.device, dtype=torch.float32).contiguous()
        if o.shape != t.shape or o.dim() != 4 or o.shape[1] != 1:
            raise ValueError(f"VGG loss expects [B,1,H,W] pairs, got {tuple(o.shape)}, {tuple(t.shape)}")
        with ops.stage("vgg.fwd"):
            return self._forward(o, t)

    def _forward(self, o, t):
        B, _, H, W = o.shape
        n2 = 2 * B
        cur = ops.vgg_prep(o, t, self.mean, self.denom)
        h, w = H, W
        relu = False
        ones = zeros = None
        terms = []
        wts = self._wts
        plan = self._plan()
        n_w = sum(1 for st in plan if st[1] == "wino")
        # max|V| of every Winograd conv's input transform (zeroed once per call)
        am_v = ops.amax_slots(n_w, o.device) if VGG_F16X2 and n_w else None
        i_w = 0
        for step in plan:
            idx, kind = step[0], step[1]
            if kind == "conv":
                _, _, wpk, bias, cop = step
                pro = None
                if relu:
                    cp = cur.shape[1]
                    if ones is None or ones.numel() != cp:
                        ones = torch.ones(cp, device=o.device)
                        zeros = torch.zeros(cp, device=o.device)
                    pro = (ones, zeros, None)
                cur = ops.conv_fwd(cur, n2, h, w, wpk, bias, cop, 3, pro=pro, slope=0.0,
                                   tag=f"vgg.{idx}")
                relu = False
            elif kind == "wino":
                _, _, U, bias, cop, am_u = step
                cur = ops.conv3x3_wino(cur, n2, h, w, U, bias, cop, tile=WINO_TILE, relu=relu,
                                       tag=f"vgg.{idx}", amax_v=ops.amax_slot(am_v, i_w)
                                       if am_v is not None else None, amax_u=am_u)
                i_w += 1
                relu = False
            elif kind == "relu":
                relu = True
            else:
                cur = ops.maxpool2(cur, n2, h, w)
                h, w = h // 2, w // 2
            if idx in self.feature_layers:
                half = B * h * w
                i = self.feature_layers.index(idx)
                terms.append(ops.l1_mean(cur[:half], cur[half:], wts[i]))
        self.last_terms = terms        # weighted per-tap terms (device scalars)
        self.f16x2 = am_v is not None
        total = terms[0]
        for v in terms[1:]:
            total = total + v
        return total
