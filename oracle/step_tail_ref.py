"""CPU restatement of the reference training-step tail (TEST INFRASTRUCTURE).

Only tests/ and the golden-fixture scripts use this module; nothing in the
product path (pcss-unet_amd/) imports it. It restates, on PyTorch CPU tensors,
what /root/reference/main.py does between `backward()` and
`optimizer.step()`:

  * main.py:295-317  per-parameter NaN/Inf census; a parameter with more than
                     20 % invalid entries skips the step;
  * main.py:320-354  otherwise repair every parameter: NaN -> valid mean +
                     randn * valid std * 0.1, +-Inf -> sign * max|valid| * 10,
                     zero the gradient if it is still not finite;
  * main.py:357-358  max_norm = 1.0, or max(0.1, 1 - epoch/num_epochs) from
                     half the epochs on;
  * main.py:361-365  per-parameter clip to 1000 * scale before unscaling;
  * main.py:368-402  unscale, then per parameter: NaN/Inf -> skip,
                     norm > 1e5 -> skip, norm > 1e3 -> rescale to 1e3;
  * main.py:405      clip_grad_norm_(max_norm);
  * main.py:408-418  skip if any clipped per-parameter norm exceeds 10;
  * main.py:421-423  optimizer step (AdamW, main.py:954-955).

`scale` is the GradScaler scale; on the reference's CPU path (and on our
fp32/bf16 GPU path, which needs no loss scaling) the scaler is disabled and
its scale is 1.0 (main.py:175: `enabled=(device.type == 'cuda')`).

Pinned by tests/golden/tail_steps.npz, which tests/golden/make_golden_tail.py
produced by running the reference's own `train_model` (main.py:132-581) on a
stub model whose gradients are injected; test_oracle.py replays it here.
"""
import math

import torch


def max_norm_for(epoch, num_epochs):
    ratio = epoch / num_epochs
    return 1.0 if ratio < 0.5 else max(0.1, 1.0 - ratio)


def lr_lambda(warmup_epochs, num_epochs):
    """main.py:959-967."""
    def f(epoch):
        if epoch < warmup_epochs:
            return float(epoch) / float(max(1, warmup_epochs))
        d = 0.5 * (1.0 + math.cos(math.pi * (epoch - warmup_epochs) / (num_epochs - warmup_epochs)))
        return max(0.01, d)
    return f


FLT_MAX = 3.4028234663852886e38


def fp32_norm(t):
    """torch.norm of an fp32 gradient as the reference's device computes it
    (main.py:95, CUDA): the squares accumulate in fp32, so a sum of squares
    above FLT_MAX (a norm above ~1.8e19) reads +inf. Below that the value is
    torch.norm's. (Some hosts' CPU kernels sum in double and return a finite
    norm up to FLT_MAX; this restatement fixes the fp32 behaviour so the
    decision does not depend on the host.)"""
    n = torch.norm(t)
    if torch.isfinite(n) and t.double().pow(2).sum().item() > FLT_MAX:
        return torch.tensor(float("inf"))
    return n


def sanitize_and_clip(params, epoch, num_epochs, scale=1.0, noise=None):
    """Apply main.py:287-418 to `params` (each with .grad) in place.
    Returns True when the reference would skip the optimizer step. `noise`
    (one tensor per parameter, like its grad) replaces the randn draws of the
    NaN repair; None draws them with torch.randn_like as the reference does."""
    # census (:295-312); a severe parameter stops the scan
    fixable = False
    for p in params:
        g = p.grad
        if g is None:
            continue
        bad_nan, bad_inf = torch.isnan(g), torch.isinf(g)
        if bad_nan.any() or bad_inf.any():
            frac = (bad_nan.sum() + bad_inf.sum()).item() / g.numel()
            if frac > 0.2:
                return True
            fixable = True
    # repair (:320-354)
    if fixable:
        for i, p in enumerate(params):
            g = p.grad
            if g is None:
                continue
            g = g.data
            ok = ~(torch.isnan(g) | torch.isinf(g))
            if ok.sum() > 0:
                vals = g[ok]
                mu = vals.mean().item()
                sd = vals.std().item() if vals.numel() > 1 else 0.01
                nan = torch.isnan(g)
                if nan.any():
                    z = torch.randn_like(g[nan]) if noise is None else noise[i][nan]
                    g[nan] = mu + z * sd * 0.1
                inf = torch.isinf(g)
                if inf.any():
                    big = vals.abs().max().item()
                    g[inf] = torch.sign(g[inf]) * big * 10.0
            else:
                g.zero_()
            if torch.isnan(g).any() or torch.isinf(g).any():
                g.zero_()
    max_norm = max_norm_for(epoch, num_epochs)
    # pre-unscale clip (:361-365)
    if math.isfinite(scale):
        for p in params:
            if p.grad is not None:
                n = fp32_norm(p.grad.data)
                p.grad.data.mul_(torch.clamp(torch.tensor(1.0 / max(1.0, n / (1000.0 * scale))),
                                             max=1.0))
    # unscale_ (a no-op multiply by 1/scale when the scaler is disabled)
    if scale != 1.0:
        for p in params:
            if p.grad is not None:
                p.grad.data.mul_(1.0 / scale)
    # per-parameter checks (:371-397)
    for p in params:
        if p.grad is None:
            continue
        if torch.isnan(p.grad).any() or torch.isinf(p.grad).any():
            return True
        n = fp32_norm(p.grad)
        if n > 1e3:
            if n > 1e5:
                return True
            p.grad.data.mul_(min(1.0, 1e3 / n))
    # global clip (:405) and the post-clip check (:408-418)
    torch.nn.utils.clip_grad_norm_([p for p in params], max_norm=max_norm)
    worst = 0.0
    for p in params:
        if p.grad is not None:
            worst = max(worst, torch.norm(p.grad).item())
    return worst > 10.0


def replay_noise(rng_state, grads, severe):
    """The randn draws of the repair (main.py:336) in the order the reference
    makes them: one randn_like per parameter that has NaNs, from the RNG state
    the step started with. Returns flat noise tensors (zeros elsewhere)."""
    out = [torch.zeros_like(g) for g in grads]
    if severe:
        return out
    torch.set_rng_state(rng_state)
    for g, o in zip(grads, out):
        nan = torch.isnan(g)
        if nan.any():
            o[nan] = torch.randn(int(nan.sum()))
    return out
