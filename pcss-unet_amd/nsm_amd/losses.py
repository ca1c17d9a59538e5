"""Losses of the hot path on the libnsm kernels.

* `L1Loss` / `l1_loss`: nn.L1Loss (mean) — customLoss.py:96,134.
* `CustomLoss(device, alpha=0.9)`: returns alpha*L1 + (1-alpha)*vgg
  (customLoss.py:129-193). The reference's VGG term is a DETACHED constant
  (`torch.tensor(total_loss, requires_grad=True)`, customLoss.py:90), so the
  gradient is exactly alpha*sign(o-t)/N. The VGG19 perceptual value
  (`nsm_amd.vgg.MultiLayerVGGLoss`, on the libnsm kernels) needs the ImageNet
  weights the reference downloads at construction (customLoss.py:20,97). By
  default (`vgg_weights="auto"`) the torchvision checkpoint is taken from
  $NSM_VGG19_WEIGHTS or torch.hub's cache (`<hub>/checkpoints/
  vgg19-dcbb9e9d.pth`, loaded with weights_only=True); when neither exists the
  loss warns once that its VGG term is 0. Other values: a .pth path, a
  state_dict, a MultiLayerVGGLoss, "random", or False (term off, no warning);
  any `vgg=<callable(out, target)>` overrides. The gradient is the same either
  way.
* The reference asserts `output.min() >= 0 and output.max() <= 1`
  (customLoss.py:131) with a host sync per call. Here a range-check kernel
  sets a sticky device flag that is copied to pinned host memory
  asynchronously; the next call raises the same AssertionError once that copy
  has landed (at most one step late, never a sync), and `check_range()`
  checks it immediately (synchronising).
* `PerturbationLoss(perturbation_count=3)`: pert_loss.py:7-90 — three
  no-grad forwards of the model on inputs perturbed by per-channel
  std * 0.01 Gaussian noise, mean L1 to the original output.
* `EnhancedCustomLoss(device, alpha=0.9, perturb_weight=0.5)`: the wired
  perturbation-training loss of pert_loss.py:92-163 (§8f next-row #4). The
  reference's class cannot be constructed (it imports a `VGGLoss` that
  customLoss.py does not define); this one uses the `MultiLayerVGGLoss`
  CustomLoss uses and otherwise follows the reference: returns
  (total, {'l1_loss', 'vgg_loss', 'perturbation_loss', 'total_loss'}),
  total = alpha*L1 + (1-alpha)*vgg [+ perturb_weight*perturbation while
  training].
* `measure_temporal_instability(frames, motion_vectors=None, alpha=5.0)`:
  pert_loss.py:166-199, mean over consecutive frame pairs of
  mean(exp(alpha*|f_t - f_{t-1}|) - 1) (`nsm_expdiff_mean`).
"""
import os
import warnings

import torch
import torch.nn as nn

from ._lib import call, lib, ptr, require_gpu, stream

VGG19_FILE = "vgg19-dcbb9e9d.pth"   # torchvision IMAGENET1K_V1 (customLoss.py:20)
_VGG_WARNED = []


def find_vgg19_checkpoint():
    """A locally cached torchvision VGG19 ImageNet checkpoint, or None."""
    env = os.environ.get("NSM_VGG19_WEIGHTS")
    cands = [env] if env else []
    try:
        cands.append(os.path.join(torch.hub.get_dir(), "checkpoints", VGG19_FILE))
    except Exception:  # noqa: BLE001  (hub dir unresolvable: no cache)
        pass
    for c in cands:
        if c and os.path.isfile(c):
            return c
    return None


class _RangeCheck:
    """Sticky device flag for `assert 0 <= output <= 1` (customLoss.py:131,
    pert_loss.py:131) without a host synchronisation."""

    def __init__(self, what):
        self.what = what
        self.flag = None
        self.host = None
        self.event = None

    def _raise_if_set(self):
        if self.host is not None and int(self.host[0]) != 0:
            self.host[0] = 0
            self.flag.zero_()
            raise AssertionError(f"{self.what}: output must be in [0, 1] (sigmoid output), "
                                 "customLoss.py:131")

    def prepare(self, device):
        """Allocate the flag, its pinned host copy and the event on `device`
        (outside any graph capture: a capture would record the flag's zeroing
        into every replay, which would make it non-sticky)."""
        if self.flag is None or self.flag.device != torch.device(device):
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"{self.what}: the range flag must be allocated before graph "
                                   "capture (call prepare_capture(device) first)")
            self.flag = torch.zeros(1, dtype=torch.int32, device=device)
            self.host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self.event = torch.cuda.Event()

    def launch(self, o):
        self.prepare(o.device)
        if torch.cuda.is_current_stream_capturing():
            # a captured step (GraphedTrainStep): the sticky device flag only —
            # no event, no copy; check() reads the flag itself
            call("nsm_range_flag", ptr(o), o.numel(), 0.0, 1.0, ptr(self.flag), stream())
            self.captured = True
            return
        if self.event.query():
            self._raise_if_set()
        # eager: the kernel stores the sticky 1 straight into the pinned host
        # word (mapped into the device's address space; it only ever writes 1),
        # so no device-to-host copy is queued; the event orders the host's read
        call("nsm_range_flag", ptr(o), o.numel(), 0.0, 1.0, ptr(self.host), stream())
        self.event.record()

    def check(self):
        if getattr(self, "captured", False):
            torch.cuda.current_stream().synchronize()
            self.host.copy_(self.flag)
            self._raise_if_set()
        elif self.event is not None:
            self.event.synchronize()
            self._raise_if_set()


class _L1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, o, t, alpha):
        require_gpu(o, "L1 input")
        o_ = o.detach().contiguous().to(torch.float32)
        t_ = t.detach().contiguous().to(device=o.device, dtype=torch.float32)
        n = o_.numel()
        if t_.numel() != n:
            raise ValueError(f"l1: shape mismatch {tuple(o.shape)} vs {tuple(t.shape)}")
        nb = lib.nsm_loss_blocks(n)
        partial = torch.empty(nb, dtype=torch.float32, device=o.device)
        out = torch.empty((), dtype=torch.float32, device=o.device)
        call("nsm_l1_loss_fwd", ptr(o_), ptr(t_), n, float(alpha), ptr(partial), ptr(out), stream())
        ctx.save_for_backward(o_, t_)
        ctx.alpha = float(alpha)
        ctx.oshape = o.shape
        return out

    @staticmethod
    def backward(ctx, g):
        o_, t_ = ctx.saved_tensors
        grad = torch.empty_like(o_)
        g_ = g.detach().contiguous().to(torch.float32)
        call("nsm_l1_loss_bwd", ptr(o_), ptr(t_), o_.numel(), ctx.alpha, ptr(g_), ptr(grad), 0,
             stream())
        return grad.view(ctx.oshape), None, None


def l1_loss(output, target, alpha=1.0):
    return _L1Fn.apply(output, target, alpha)


class L1Loss(nn.Module):
    def forward(self, output, target):
        return l1_loss(output, target)


class CustomLoss(nn.Module):
    def __init__(self, device=None, alpha=0.9, vgg=None, vgg_weights="auto", check_range=True):
        super().__init__()
        self.alpha = alpha
        self.l1 = L1Loss()
        if vgg is not None and isinstance(vgg_weights, str) and vgg_weights == "auto":
            vgg_weights = None           # an explicit vgg callable wins
        if vgg is None and isinstance(vgg_weights, str) and vgg_weights == "auto":
            vgg_weights = find_vgg19_checkpoint()
            if vgg_weights is None and not _VGG_WARNED:
                _VGG_WARNED.append(True)
                warnings.warn(
                    "nsm_amd.CustomLoss: no VGG19 ImageNet checkpoint found ($NSM_VGG19_WEIGHTS "
                    f"or torch.hub cache {VGG19_FILE}); the perceptual term (customLoss.py:137, "
                    "weight 1-alpha) is 0 — the loss VALUE differs from the reference's, its "
                    "gradient (alpha*sign/N) does not", RuntimeWarning, stacklevel=2)
        if vgg_weights is False:
            vgg_weights = None
        if vgg_weights is not None:
            from .vgg import MultiLayerVGGLoss
            if isinstance(vgg_weights, MultiLayerVGGLoss):
                self.vgg_loss = vgg_weights
            elif isinstance(vgg_weights, str) and vgg_weights == "random":
                self.vgg_loss = MultiLayerVGGLoss(device)
            elif isinstance(vgg_weights, str):
                self.vgg_loss = MultiLayerVGGLoss.from_torchvision_checkpoint(vgg_weights, device)
            else:
                self.vgg_loss = MultiLayerVGGLoss(device, state_dict=vgg_weights)
            vgg = self.vgg_loss
        self.vgg = vgg
        self.device = device
        self.check_range = check_range
        self._range = _RangeCheck("CustomLoss")

    def forward(self, output, target, inputs=None):
        if self.check_range:
            require_gpu(output, "CustomLoss output")
            self._range.launch(output.detach().contiguous().to(torch.float32))
        loss = l1_loss(output, target, self.alpha)
        if self.vgg is not None:
            v = self.vgg(output, target)
            loss = loss + (1 - self.alpha) * torch.as_tensor(v, device=loss.device).detach()
        return loss

    def check_range_now(self):
        """Raise now (host sync) if any output seen so far left [0, 1]."""
        self._range.check()

    def prepare_capture(self, device):
        """Allocate the range assert's device state before a graph capture
        (GraphedTrainStep calls it)."""
        if self.check_range:
            self._range.prepare(device)


class PerturbationLoss(nn.Module):
    def __init__(self, perturbation_count=3, alpha=0.9, std_factor=0.01):
        super().__init__()
        self.perturbation_count = perturbation_count
        self.alpha = alpha
        self.std_factor = std_factor
        self.loss_fn = L1Loss()

    def perturb_input(self, x, noises=None):
        """Per-channel unbiased std over the batch, then x + n*std*0.01
        (pert_loss.py:26-59); `noises` (list of tensors shaped like x) may be
        supplied for parity, else drawn from torch.randn."""
        require_gpu(x, "perturbation input")
        x_ = x.detach().contiguous().to(torch.float32)
        B, C, H, W = x_.shape
        std = torch.empty(C, dtype=torch.float32, device=x.device)
        call("nsm_channel_std", ptr(x_), B, C, H, W, None, ptr(std), stream())
        outs = []
        for i in range(self.perturbation_count):
            n = noises[i] if noises is not None else torch.randn_like(x_)
            n = n.to(device=x.device, dtype=torch.float32).contiguous()
            o = torch.empty_like(x_)
            call("nsm_perturb", ptr(x_), ptr(n), ptr(std), B, C, H, W, self.std_factor, ptr(o),
                 stream())
            outs.append(o)
        return outs

    def forward(self, model, original_input, original_output, noises=None):
        pins = self.perturb_input(original_input, noises)
        with torch.no_grad():
            pouts = [model(p) for p in pins]
        total = 0
        for po in pouts:
            total = total + l1_loss(original_output, po)
        return total / len(pouts)


class EnhancedCustomLoss(nn.Module):
    def __init__(self, device=None, alpha=0.9, perturb_weight=0.5, vgg=None, vgg_weights="auto"):
        super().__init__()
        self.alpha = alpha
        self.perturb_weight = perturb_weight
        self.l1 = L1Loss()
        self.base = CustomLoss(device, alpha, vgg=vgg, vgg_weights=vgg_weights)
        self.vgg_loss = getattr(self.base, "vgg_loss", None) or vgg
        self.perturbation_loss = PerturbationLoss()

    def prepare_capture(self, device):
        self.base._range.prepare(device)

    def check_range_now(self):
        self.base._range.check()

    def forward(self, model, output, target, inputs, noises=None):
        # pert_loss.py:131: the same [0, 1] assertion, as CustomLoss's device flag
        require_gpu(output, "EnhancedCustomLoss output")
        self.base._range.launch(output.detach().contiguous().to(torch.float32))
        l1 = l1_loss(output, target)
        if self.vgg_loss is not None:
            vgg = torch.as_tensor(self.vgg_loss(output, target), device=l1.device).detach()
        else:
            vgg = torch.zeros((), device=l1.device)
        # d(alpha*l1)/do reaches the L1 backward as gscale = alpha: alpha*sign/N
        basic = self.alpha * l1 + (1 - self.alpha) * vgg
        losses = {"l1_loss": l1, "vgg_loss": vgg}
        if self.training and self.perturb_weight > 0:
            pert = self.perturbation_loss(model, inputs, output, noises=noises)
            total = basic + self.perturb_weight * pert
            losses["perturbation_loss"] = pert
        else:
            total = basic
            losses["perturbation_loss"] = torch.zeros((), device=l1.device)
        losses["total_loss"] = total
        return total, losses


def measure_temporal_instability(frames, motion_vectors=None, alpha=5.0):
    """frames: sequence of same-shape tensors on the GPU (e.g. [B,1,H,W] outputs)."""
    if len(frames) < 2:
        return torch.tensor(0.0)
    # motion_vectors: the reference accepts them but does not use them (pert_loss.py:184-187)
    dev = frames[0].device
    require_gpu(frames[0], "temporal-instability frames")
    n = frames[0].numel()
    partial = torch.empty(lib.nsm_loss_blocks(n), dtype=torch.float32, device=dev)
    total = torch.zeros((), dtype=torch.float32, device=dev)
    for t in range(1, len(frames)):
        a = frames[t].detach().contiguous().to(torch.float32)
        b = frames[t - 1].detach().contiguous().to(torch.float32)
        out = torch.empty((), dtype=torch.float32, device=dev)
        call("nsm_expdiff_mean", ptr(a), ptr(b), n, float(alpha), ptr(partial), ptr(out), stream())
        total = total + out
    return total / (len(frames) - 1)
