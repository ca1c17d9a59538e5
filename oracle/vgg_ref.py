"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's VGG19
perceptual loss (customLoss.py:7-90, `MultiLayerVGGLoss`), the checker for
nsm_amd.vgg. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
may import it.

The reference builds torchvision's `vgg19(IMAGENET1K_V1).features` and, for
each feature index in (2, 7, 12, 21, 30), a prefix `features[:idx+1]`; the
features are therefore the PRE-ReLU outputs of conv layers 2, 7, 12, 21, 30.
Loss = sum_i w_i * mean|f_i(o) - f_i(t)| with w normalised to sum 1
(customLoss.py:31-33,71-83) on inputs clamp(., 0, 1) (nan_to_num), repeated
to 3 channels and normalised by (x - 0.485) / (0.229 + 1e-8)
(customLoss.py:44-62). It is computed under no_grad and returned as a fresh
tensor (customLoss.py:90): a detached constant.

ImageNet weights are a network download (unavailable offline): the
`standin_state` recipe (seeded randn, He scale, zero bias) is the one
tests/golden/make_golden.py installs in place of torchvision, so the fixtures'
`vgg` values pin this restatement against the reference code path.
"""
import torch
import torch.nn.functional as F

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M",
             512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
FEATURE_LAYERS = (2, 7, 12, 21, 30)
LAYER_WEIGHTS = (0.25, 0.25, 0.3, 0.1, 0.1)
MEAN, STD, EPS = 0.485, 0.229, 1e-8


def layers():
    """torchvision vgg19().features index order: [(idx, kind, cin, cout)]."""
    out, c, idx = [], 3, 0
    for v in VGG19_CFG:
        if v == "M":
            out.append((idx, "pool", c, c))
            idx += 1
        else:
            out.append((idx, "conv", c, v))
            out.append((idx + 1, "relu", v, v))
            idx += 2
            c = v
    return out


def standin_state(seed=19):
    """{'<idx>.weight', '<idx>.bias'} of the stand-in VGG19 (make_golden.py recipe)."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for idx, kind, ci, co in layers():
        if kind == "conv":
            sd[f"{idx}.weight"] = torch.randn(co, ci, 3, 3, generator=g) * (2.0 / (9 * ci)) ** 0.5
            sd[f"{idx}.bias"] = torch.zeros(co)
    return sd


def features(sd, x, taps=FEATURE_LAYERS):
    """Run the stack once (incrementally) and return {idx: output of layer idx}."""
    out, last = {}, max(taps)
    for idx, kind, ci, co in layers():
        if idx > last:
            break
        if kind == "conv":
            x = F.conv2d(x, sd[f"{idx}.weight"], sd[f"{idx}.bias"], padding=1)
        elif kind == "relu":
            x = F.relu(x)          # not in place: the recorded pre-ReLU tap must survive
        else:
            x = F.max_pool2d(x, 2, 2)
        if idx in taps:
            out[idx] = x
    return out


def prep(img):
    """customLoss.py:44-62 on a [B,1,H,W] image."""
    x = torch.clamp(img.to(torch.float32), 0.0, 1.0)
    x = torch.nan_to_num(x, nan=0.5, posinf=1.0, neginf=0.0)
    mean = torch.tensor([MEAN]).view(1, 1, 1, 1)
    std = torch.tensor([STD]).view(1, 1, 1, 1)
    return (x.repeat(1, 3, 1, 1) - mean) / (std + EPS)


def normalized_weights(weights=LAYER_WEIGHTS):
    w = torch.tensor(weights)
    return w / w.sum()


def layer_losses(sd, output, target, feature_layers=FEATURE_LAYERS):
    """[mean|f_i(o) - f_i(t)|] per feature layer (unweighted)."""
    with torch.no_grad():
        fo = features(sd, prep(output), feature_layers)
        ft = features(sd, prep(target), feature_layers)
    vals = []
    for idx in feature_layers:
        a = torch.nan_to_num(fo[idx], nan=0.0, posinf=1.0, neginf=-1.0)
        b = torch.nan_to_num(ft[idx], nan=0.0, posinf=1.0, neginf=-1.0)
        vals.append(F.l1_loss(a, b))
    return vals


def vgg_loss(sd, output, target, feature_layers=FEATURE_LAYERS, weights=LAYER_WEIGHTS):
    w = normalized_weights(weights)
    total = 0.0
    for i, v in enumerate(layer_losses(sd, output, target, feature_layers)):
        total = total + w[i] * v
    return torch.as_tensor(total).detach()
