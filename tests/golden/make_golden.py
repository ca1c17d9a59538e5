"""Generate the golden fixtures in tests/golden/ by running the REFERENCE code
(/root/reference, read-only) in the survey/build container.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference modules as-is with three import-only stubs, exactly
as SURVEY.md §8(c) records:
  * `visualize` (needs graphviz; `make_dot` is never called, Unetmodel.py:4)
  * `torchvision.models.vgg19` (IMAGENET1K_V1 weights are a network download:
    a locally built VGG19 'E' stack with seeded random weights stands in, so
    the VGG *value* is parity-unpinned; it is a detached constant anyway,
    customLoss.py:90)
  * `pytorch_msssim` (imported, unused: customLoss.py:5)

Weights come from oracle/weights.py's numpy recipe (loaded into the
reference Unet with load_state_dict). Dropout masks are recovered by
replaying the reference's RNG stream (ATen feature dropout draws one
bernoulli_(1-p) tensor of shape [B,C,1,1] per DoubleConv with p>0, in
forward order; conv5's checkpoint restores the RNG state for its recompute)
and checked by re-running the oracle with them.

Fixtures hold inputs and expected outputs only (no reference source).
This script is never shipped to or run on the GPU box.
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from oracle import unet_ref as O  # noqa: E402
from oracle.weights import make_state, synthetic_batch, block_channels  # noqa: E402


def install_stubs():
    sys.modules["visualize"] = types.SimpleNamespace(make_dot=None)
    sys.modules["pytorch_msssim"] = types.SimpleNamespace(ssim=None)
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")

    class _W:
        IMAGENET1K_V1 = "IMAGENET1K_V1"

    def vgg19(weights=None):
        cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M",
               512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
        layers, c = [], 3
        g = torch.Generator().manual_seed(19)
        for v in cfg:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                conv = nn.Conv2d(c, v, 3, padding=1)
                with torch.no_grad():
                    conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * (2.0 / (9 * c)) ** 0.5)
                    conv.bias.zero_()
                layers += [conv, nn.ReLU(inplace=True)]
                c = v
        return types.SimpleNamespace(features=nn.Sequential(*layers))

    models.vgg19 = vgg19
    models.VGG19_Weights = _W
    tv.models = models
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = models
    sys.path.insert(0, REF)


def ref_model(in_ch, dropout, np_sd):
    import Unetmodel
    m = Unetmodel.Unet(dropout_rate=dropout)
    if in_ch != 4:
        # the 7-ch generalisation uses the reference's own DoubleConv
        m.conv2 = Unetmodel.DoubleConv(4 * in_ch, 64, dropout)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in np_sd.items()})
    return m


def calibrate(m, x):
    """Make the running stats meaningful for eval fixtures: one train-mode
    no-grad forward with BN momentum 1.0 copies the batch stats in."""
    for mod in m.modules():
        if isinstance(mod, nn.BatchNorm2d):
            mod.momentum = 1.0
    m.train()
    with torch.no_grad():
        m(x)
    for mod in m.modules():
        if isinstance(mod, nn.BatchNorm2d):
            mod.momentum = 0.1
            mod.num_batches_tracked.zero_()


def running_state(m):
    return {k: v.detach().numpy().copy() for k, v in m.state_dict().items()
            if "running" in k or "num_batches" in k}


def proj_vector(idx, n):
    return np.random.default_rng([7, idx]).standard_normal(n).astype(np.float32)


def grad_summary(m, prefix="g/"):
    out = {}
    for idx, (k, p) in enumerate(m.named_parameters()):
        g = p.grad.detach().numpy().astype(np.float64).ravel()
        if g.size <= 4096:
            out[prefix + k] = g.astype(np.float32)
        else:
            out[prefix + k + "/sum"] = np.array(g.sum())
            out[prefix + k + "/l2"] = np.array(np.sqrt((g * g).sum()))
            out[prefix + k + "/head"] = g[:64].astype(np.float32)
            out[prefix + k + "/proj"] = np.array((g * proj_vector(idx, g.size)).sum())
    return out


def replay_masks(seed, B, in_ch, p):
    torch.manual_seed(seed)
    masks = {}
    for k, (ci, _) in block_channels(in_ch).items():
        pk = O.block_dropout(k, p)
        if pk > 0:
            masks[k] = torch.empty(B, ci, 1, 1).bernoulli_(1 - pk).div_(1 - pk).view(B, ci)
    return masks


def train_case(name, in_ch, B, H, W, dropout, seed_w=42, mask_seed=1234):
    np_sd = make_state(in_ch, seed_w)
    x_np, y_np = synthetic_batch(B, in_ch, H, W)
    m = ref_model(in_ch, dropout, np_sd)
    m.train()
    import customLoss
    crit = customLoss.CustomLoss("cpu", alpha=0.9)
    x = torch.from_numpy(x_np.copy()).requires_grad_(True)   # setdata.py:325-326
    y = torch.from_numpy(y_np.copy())
    torch.manual_seed(mask_seed)
    out = m(x)
    loss = crit(out, y, x)
    l1 = crit.l1(out, y)
    vgg = (loss - crit.alpha * l1) / (1 - crit.alpha)        # main.py:276-277
    loss.backward()
    rec = {"x": x_np, "y": y_np, "out": out.detach().numpy(), "loss": np.array(loss.item()),
           "l1": np.array(l1.item()), "vgg": np.array(vgg.item()), "x_grad": x.grad.numpy(),
           "meta/in_ch": np.array(in_ch), "meta/dropout": np.array(dropout),
           "meta/seed_w": np.array(seed_w)}
    masks = replay_masks(mask_seed, B, in_ch, dropout) if dropout > 0 else {}
    for k, v in masks.items():
        rec[f"mask/{k}"] = v.numpy()
    rec.update(grad_summary(m))
    rec.update({"run/" + k: v for k, v in running_state(m).items()})
    # cross-check the oracle restatement against the reference right here
    sd = O.torch_state(np_sd, requires_grad=True)
    xo = torch.from_numpy(x_np.copy()).requires_grad_(True)
    oo, saved = O.forward(sd, xo, True, masks, dropout)
    O.custom_loss(oo, y, 0.9, vgg.item()).backward()
    O.conv5_recompute_bn_update(sd, saved["p4"], mask=masks.get(5))
    err = (oo.detach() - out.detach()).abs().max().item()
    gerr = (xo.grad - x.grad).abs().max().item() / (x.grad.abs().max().item() + 1e-30)
    rerr = max((sd[k].float() - torch.from_numpy(v).float()).abs().max().item()
               for k, v in running_state(m).items())
    print(f"{name}: out max|d|={err:.3e}  x_grad rel={gerr:.3e}  running max|d|={rerr:.3e}")
    assert err < 1e-5 and gerr < 1e-3 and rerr < 1e-5, name
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)


def eval_case(name, in_ch, B, H, W, seed_w=42):
    np_sd = make_state(in_ch, seed_w)
    x_np, _ = synthetic_batch(B, in_ch, H, W)
    m = ref_model(in_ch, 0.2, np_sd)
    x = torch.from_numpy(x_np.copy())
    calibrate(m, x)
    m.eval()
    with torch.no_grad():
        out = m(x)
    rec = {"x": x_np, "out": out.numpy(), "meta/in_ch": np.array(in_ch), "meta/seed_w": np.array(seed_w)}
    rec.update({"run/" + k: v for k, v in running_state(m).items()})
    sd = O.torch_state(np_sd)
    for k, v in running_state(m).items():
        sd[k] = torch.from_numpy(v.copy())
    with torch.no_grad():
        oo, _ = O.forward(sd, x, False)
    err = (oo - out).abs().max().item()
    print(f"{name}: out max|d|={err:.3e}  out range [{out.min():.3f},{out.max():.3f}] std {out.std():.3f}")
    assert err < 1e-5, name
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)


def perturb_case(name, in_ch=4, B=1, H=64, W=64, seed_w=42, noise_seed=77):
    """PerturbationLoss (pert_loss.py:7-90) on a train-mode, dropout-0 model."""
    import pert_loss
    np_sd = make_state(in_ch, seed_w)
    x_np, _ = synthetic_batch(B, in_ch, H, W)
    m = ref_model(in_ch, 0.0, np_sd)
    m.train()
    x = torch.from_numpy(x_np.copy())
    with torch.no_grad():
        out0 = m(x)
    out = out0.clone().requires_grad_(True)
    run_before = running_state(m)
    torch.manual_seed(noise_seed)
    pl = pert_loss.PerturbationLoss()
    loss = pl(m, x, out)
    loss.backward()
    torch.manual_seed(noise_seed)
    noises = [torch.stack([torch.randn_like(x[:, c:c + 1]) for c in range(x.shape[1])], 0)
              for _ in range(3)]
    noises = [n.permute(1, 0, 2, 3, 4).reshape(x.shape) for n in noises]
    rec = {"x": x_np, "out": out0.numpy(), "loss": np.array(loss.item()), "out_grad": out.grad.numpy(),
           "noise": np.stack([n.numpy() for n in noises]), "meta/in_ch": np.array(in_ch),
           "meta/seed_w": np.array(seed_w)}
    rec.update({"run_before/" + k: v for k, v in run_before.items()})
    rec.update({"run/" + k: v for k, v in running_state(m).items()})
    # oracle check
    sd = O.torch_state(np_sd)
    for k, v in run_before.items():
        sd[k] = torch.from_numpy(v.copy())
    ps = O.perturb_inputs(x, noises)
    with torch.no_grad():
        pouts = [O.forward(sd, p, True, None, 0.0)[0] for p in ps]
    oo = out0.clone().requires_grad_(True)
    lo = O.perturbation_loss(oo, pouts)
    lo.backward()
    print(f"{name}: loss ref {loss.item():.8e} oracle {lo.item():.8e}  grad max|d| "
          f"{(oo.grad - out.grad).abs().max().item():.3e}")
    assert abs(lo.item() - loss.item()) <= 1e-6 * abs(loss.item()) + 1e-9
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)


def vgg_case(name, B, H, W, seed=11):
    """MultiLayerVGGLoss (customLoss.py:7-90) value and per-layer L1 terms on the
    stand-in VGG19 weights (install_stubs), for sigmoid-range images."""
    import customLoss
    vl = customLoss.MultiLayerVGGLoss("cpu")
    g = torch.Generator().manual_seed(seed)
    o = torch.sigmoid(torch.randn(B, 1, H, W, generator=g) * 2)
    t = torch.randint(0, 256, (B, 1, H, W), generator=g).float() / 255.0
    o[0, 0, 0, :3] = torch.tensor([-0.5, 1.5, float("nan")])   # clamp / nan_to_num paths
    val = vl(o, t)
    per = []
    with torch.no_grad():
        on = (torch.nan_to_num(torch.clamp(o, 0, 1), nan=0.5).repeat(1, 3, 1, 1) - vl.mean) / (vl.std + 1e-8)
        tn = (torch.clamp(t, 0, 1).repeat(1, 3, 1, 1) - vl.mean) / (vl.std + 1e-8)
        for ext in vl.feature_extractors:
            per.append(torch.nn.functional.l1_loss(ext(on), ext(tn)).item())
    from oracle import vgg_ref as V
    sd = V.standin_state()
    ov = V.vgg_loss(sd, o, t).item()
    oper = [v.item() for v in V.layer_losses(sd, o, t)]
    print(f"{name}: vgg ref {val.item():.8e} oracle {ov:.8e} per-layer max|d| "
          f"{max(abs(a - b) for a, b in zip(per, oper)):.3e}")
    assert abs(ov - val.item()) <= 1e-6 * abs(val.item())
    rec = {"output": o.numpy(), "target": t.numpy(), "vgg": np.array(val.item()),
           "layer_l1": np.array(per), "weights": vl.weights.numpy()}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)


def temporal_case(name="temporal_b2_5f"):
    """measure_temporal_instability (pert_loss.py:166-199) on 5 frames."""
    import pert_loss
    g = torch.Generator().manual_seed(21)
    frames = [torch.sigmoid(torch.randn(2, 1, 48, 40, generator=g)) for _ in range(5)]
    vals = {a: pert_loss.measure_temporal_instability(frames, alpha=a).item() for a in (5.0, 3.0)}
    from oracle import unet_ref as O
    for a, v in vals.items():
        ov = O.temporal_instability(frames, a).item()
        print(f"{name}: alpha {a} ref {v:.8e} oracle {ov:.8e}")
        assert abs(ov - v) <= 1e-6 * abs(v)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), frames=torch.stack(frames).numpy(),
                        value_a5=np.array(vals[5.0]), value_a3=np.array(vals[3.0]))


def dataset_case(name="mmap_norm"):
    """MmapLiverDataset.__getitem__ normalisation (setdata.py:296-328)."""
    import tempfile
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.modules.setdefault("OpenEXR", types.ModuleType("OpenEXR"))
    sys.modules.setdefault("Imath", types.ModuleType("Imath"))
    tvt = types.ModuleType("torchvision.transforms")
    sys.modules["torchvision.transforms"] = tvt
    sys.modules["torchvision"].transforms = tvt
    cwd = os.getcwd()
    rng = np.random.default_rng(5)
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)  # setdata writes dataset_debug.log to CWD at import
        try:
            import setdata
            inputs = (rng.standard_normal((3, 4, 8, 10)) * 3 + 1.5).astype(np.float32)
            labels = rng.integers(0, 256, (3, 1, 8, 10)) / 255.0          # float64 like prepare_dataset.py
            np.save(os.path.join(d, "train_inputs.npy"), inputs)
            np.save(os.path.join(d, "train_labels.npy"), labels)
            means = inputs.transpose(1, 0, 2, 3).reshape(4, -1).astype(np.float64).mean(1)
            stds = inputs.transpose(1, 0, 2, 3).reshape(4, -1).astype(np.float64).std(1)
            np.save(os.path.join(d, "train_stats.npy"), {"means": means.tolist(), "stds": stds.tolist()})
            ds = setdata.MmapLiverDataset(d, "train")
            xs, ys = zip(*[ds[i] for i in range(3)])
            rec = {"inputs": inputs, "labels": labels, "means": means, "stds": stds,
                   "x": torch.stack(xs).detach().numpy(), "y": torch.stack(ys).numpy()}
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)
    print(f"{name}: ok")


if __name__ == "__main__":
    torch.set_num_threads(8)
    install_stubs()
    if sys.argv[1:] == ["temporal"]:
        temporal_case()
        sys.exit(0)
    if sys.argv[1:] == ["vgg"]:
        vgg_case("vgg_b2_96x128", 2, 96, 128)
        vgg_case("vgg_b1_40x72", 1, 40, 72)
        sys.exit(0)
    eval_case("eval_c4_b2_64", 4, 2, 64, 64)
    eval_case("eval_c7_b1_odd_41x73", 7, 1, 41, 73)
    train_case("train_c7_p0_b2_64", 7, 2, 64, 64, 0.0)
    train_case("train_c4_drop_b2_64", 4, 2, 64, 64, 0.2)
    train_case("train_c4_p0_b1_40x72", 4, 1, 40, 72, 0.0)
    perturb_case("perturb_c4_b1_64")
    dataset_case()
    vgg_case("vgg_b2_96x128", 2, 96, 128)
    vgg_case("vgg_b1_40x72", 1, 40, 72)
    temporal_case()
