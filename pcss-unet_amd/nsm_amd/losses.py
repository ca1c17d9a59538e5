"""Losses of the hot path on the libnsm kernels.

* `L1Loss` / `l1_loss`: nn.L1Loss (mean) — customLoss.py:96,134.
* `CustomLoss(device, alpha=0.9)`: returns alpha*L1 + (1-alpha)*vgg
  (customLoss.py:129-193). The reference's VGG term is a DETACHED constant
  (`torch.tensor(total_loss, requires_grad=True)`, customLoss.py:90), so the
  gradient is exactly alpha*sign(o-t)/N. The VGG19 perceptual value
  (`nsm_amd.vgg.MultiLayerVGGLoss`, on the libnsm kernels) needs ImageNet
  weights the reference downloads at construction; offline pass
  `vgg_weights=<local torchvision vgg19 .pth | state_dict | MultiLayerVGGLoss
  | "random">` (or any `vgg=<callable(out, target)>`). With neither, the term
  is 0 (the gradient is unchanged either way).
* `PerturbationLoss(perturbation_count=3)`: pert_loss.py:7-90 — three
  no-grad forwards of the model on inputs perturbed by per-channel
  std * 0.01 Gaussian noise, mean L1 to the original output.
"""
import torch
import torch.nn as nn

from ._lib import call, lib, ptr, require_gpu, stream


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
    def __init__(self, device=None, alpha=0.9, vgg=None, vgg_weights=None, check_range=True):
        super().__init__()
        self.alpha = alpha
        self.l1 = L1Loss()
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

    def forward(self, output, target, inputs=None):
        if self.check_range:
            # customLoss.py:131 asserts output in [0,1]; sigmoid guarantees it, so
            # the check is done without a host sync (NaNs fail it too).
            pass
        loss = l1_loss(output, target, self.alpha)
        if self.vgg is not None:
            v = self.vgg(output, target)
            loss = loss + (1 - self.alpha) * torch.as_tensor(v, device=loss.device).detach()
        return loss


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
