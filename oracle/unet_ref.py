"""TEST INFRASTRUCTURE ONLY — functional PyTorch-CPU fp32 restatement of the
reference U-Net forward (autograd supplies the backward).

Follows `/root/reference/Unetmodel.py`:
  * odd-size guard + .to(f32)            :93-100
  * pixel_unshuffle(2)                   :65-67,101
  * DoubleConv = 3x3(ci->ci)+BN+LReLU(0.2)+Dropout2d(p)+1x1(ci->co)+BN+LReLU  :17-33
  * encoder conv2..conv5 with AvgPool2d(2) :104-116
  * conv5 under checkpoint(use_reentrant=False): in training, the backward
    recompute runs conv5's BatchNorms a second time on the same input, so
    their running stats see the update twice. Here the
    second update is an explicit call `conv5_recompute_bn_update()`.
  * decoder: bilinear x2 (align_corners=True) then `_upsample_and_match`
    to the skip size, DoubleConv, additive skip       :118-142
  * conv10 1x1 16->4, pixel_shuffle(2), sigmoid      :143-148

Dropout2d is restated with explicit per-(n,c) masks (values 0 or 1/(1-p)),
exactly what ATen's feature dropout multiplies by; `masks=None` in training
with p>0 is rejected so a parity run can never silently draw its own RNG.
"""
import torch
import torch.nn.functional as F

from .weights import block_channels

ENCODER = (2, 3, 4, 5)
DECODER = (6, 7, 8, 9)
SLOPE = 0.2
EPS = 1e-5


def block_dropout(k, dropout_rate):
    # Unetmodel.py:61 — conv9 uses dropout_rate/2
    return dropout_rate / 2 if k == 9 else dropout_rate


def _bn(x, sd, prefix, training, momentum):
    # nn.BatchNorm2d(eps=1e-5, momentum=0.1) (Unetmodel.py:22,27): in training
    # the module also bumps num_batches_tracked.
    if training and prefix + "num_batches_tracked" in sd:
        sd[prefix + "num_batches_tracked"] += 1
    return F.batch_norm(x, sd[prefix + "running_mean"], sd[prefix + "running_var"],
                        sd[prefix + "weight"], sd[prefix + "bias"],
                        training=training, momentum=momentum, eps=EPS)


def double_conv(x, sd, k, training, mask=None, momentum=0.1):
    """DoubleConv.forward (Unetmodel.py:20-33), dropout via explicit mask."""
    p = f"conv{k}.conv."
    y = F.conv2d(x, sd[p + "0.weight"], sd[p + "0.bias"], padding=1)
    y = _bn(y, sd, p + "1.", training, momentum)
    y = F.leaky_relu(y, SLOPE)
    if mask is not None:
        y = y * mask[:, :, None, None]
    y = F.conv2d(y, sd[p + "4.weight"], sd[p + "4.bias"])
    y = _bn(y, sd, p + "5.", training, momentum)
    return F.leaky_relu(y, SLOPE)


def resize(x, hw):
    # _upsample_and_match / nn.Upsample(scale_factor=2): bilinear, align_corners=True
    return F.interpolate(x, size=tuple(hw), mode="bilinear", align_corners=True)


def forward(sd, x, training=True, masks=None, dropout_rate=0.2, momentum=0.1):
    """Unet.forward restated. `sd` maps state_dict keys to CPU fp32 tensors
    (params may require grad; running stats are updated in place when
    training). `masks[k]` is a [B, C_in(k)] tensor for block k.
    Returns (out, saved) where saved['p4'] is conv5's input (for the
    checkpoint-recompute BN update)."""
    B, C, H, W = x.shape
    if H % 2 or W % 2:
        x = resize(x, (H - H % 2, W - W % 2))
    x = x.to(torch.float32)
    x = F.pixel_unshuffle(x, 2)

    def mask_for(k):
        if not training or block_dropout(k, dropout_rate) == 0:
            return None
        if masks is None or k not in masks:
            raise ValueError(f"training with dropout needs an explicit mask for conv{k}")
        return masks[k]

    c, inp = {}, x
    for k in ENCODER:
        c[k] = double_conv(inp, sd, k, training, mask_for(k), momentum)
        if k < 5:
            inp = F.avg_pool2d(c[k], 2)
            if k == 4:
                p4 = inp
    skip = {6: c[4], 7: c[3], 8: c[2], 9: x}
    cur = c[5]
    for k in DECODER:
        up = resize(cur, (2 * cur.shape[2], 2 * cur.shape[3]))
        up = resize(up, skip[k].shape[2:])
        y = double_conv(up, sd, k, training, mask_for(k), momentum)
        cur = y + skip[k] if k < 9 else y
    c10 = F.conv2d(cur, sd["conv10.weight"], sd["conv10.bias"])
    out = torch.sigmoid(F.pixel_shuffle(c10, 2))
    return out, {"p4": p4}


def conv5_recompute_bn_update(sd, p4, momentum=0.1, mask=None):
    """The reference's checkpoint recompute of conv5 in backward
    (Unetmodel.py:114-116, torch.utils.checkpoint use_reentrant=False):
    re-run conv5 in train mode on the same input with the same dropout
    mask (checkpoint restores the RNG state), which updates conv5's two BN
    running stats and num_batches_tracked a second time."""
    with torch.no_grad():
        double_conv(p4.detach(), sd, 5, True, mask, momentum)


def l1_loss(out, target):
    # nn.L1Loss() mean reduction (customLoss.py:96,134)
    return (out - target).abs().mean()


def custom_loss(out, target, alpha=0.9, vgg=0.0):
    """CustomLoss.forward return value (customLoss.py:160,193):
    alpha*L1 + (1-alpha)*vgg where the VGG term is a detached constant
    (customLoss.py:90), so only the L1 term carries gradient."""
    return alpha * l1_loss(out, target) + (1 - alpha) * torch.as_tensor(float(vgg))


def perturbation_loss(out, perturbed_outputs):
    """PerturbationLoss.forward tail (pert_loss.py:84-90): mean over the
    perturbed copies of L1(original_output, perturbed_output); the
    perturbed outputs come from no-grad forwards (constants)."""
    tot = 0
    for po in perturbed_outputs:
        tot = tot + F.l1_loss(out, po.detach())
    return tot / len(perturbed_outputs)


def perturb_inputs(x, noises, std_factor=0.01):
    """PerturbationLoss.perturb_input (pert_loss.py:26-59) with the Gaussian
    draws supplied: copy_i = x + noise_i[:, c] * std(x[:, c]) * std_factor,
    std unbiased over the whole batch of channel c."""
    stds = [torch.std(x[:, c]).item() for c in range(x.shape[1])]
    outs = []
    for n in noises:
        p = x.detach().clone()
        for c in range(x.shape[1]):
            p[:, c:c + 1] += n[:, c:c + 1] * stds[c] * std_factor
        outs.append(p)
    return outs


def torch_state(np_sd, requires_grad=False):
    """numpy recipe state -> torch CPU tensors (params optionally leaves)."""
    out = {}
    for k, v in np_sd.items():
        t = torch.from_numpy(v.copy())
        if requires_grad and t.dtype == torch.float32 and "running" not in k:
            t.requires_grad_(True)
        out[k] = t
    return out


def param_keys(in_ch=4):
    from .weights import state_dict_spec
    return [k for k, _, dt in state_dict_spec(in_ch) if dt == "f4" and "running" not in k]


__all__ = ["forward", "conv5_recompute_bn_update", "l1_loss", "custom_loss",
           "perturbation_loss", "perturb_inputs", "torch_state", "param_keys",
           "block_channels", "block_dropout"]


def temporal_instability(frames, alpha=5.0):
    """pert_loss.py:166-199 (measure_temporal_instability, no motion vectors):
    mean over consecutive pairs of mean(exp(alpha*|f_t - f_{t-1}|) - 1)."""
    if len(frames) < 2:
        return torch.tensor(0.0)
    total = 0
    for t in range(1, len(frames)):
        total = total + torch.mean(torch.exp(alpha * torch.abs(frames[t] - frames[t - 1])) - 1)
    return total / (len(frames) - 1)
