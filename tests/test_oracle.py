"""CPU: pin the oracle restatement (oracle/unet_ref.py) against the golden
fixtures produced by the reference code itself (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from oracle import unet_ref as O
from oracle.weights import make_state, state_dict_spec
from util import LOSS_REL, OUT_ABS, check_grads, load

torch.set_num_threads(8)


def _state_with_running(fx, in_ch, prefix="run/"):
    sd = O.torch_state(make_state(in_ch, int(fx["meta/seed_w"])))
    for k in list(sd):
        if prefix + k in fx and "running" in k:
            sd[k] = torch.from_numpy(fx[prefix + k].copy())
    return sd


def test_state_spec_matches_reference_layout():
    spec = state_dict_spec(4)
    assert len(spec) == 114
    n = sum(int(np.prod(s)) for k, s, dt in spec if dt == "f4" and "running" not in k)
    assert n == 15739556
    assert len([1 for k, s, dt in spec if dt == "f4" and "running" not in k]) == 66


@pytest.mark.parametrize("name", ["eval_c4_b2_64", "eval_c7_b1_odd_41x73"])
def test_oracle_eval(name):
    fx = load(name)
    in_ch = int(fx["meta/in_ch"])
    sd = _state_with_running(fx, in_ch)
    with torch.no_grad():
        out, _ = O.forward(sd, torch.from_numpy(fx["x"]), training=False)
    assert np.abs(out.numpy() - fx["out"]).max() <= OUT_ABS


@pytest.mark.parametrize("name", ["train_c7_p0_b2_64", "train_c4_drop_b2_64", "train_c4_p0_b1_40x72"])
def test_oracle_train_step(name):
    fx = load(name)
    in_ch, p = int(fx["meta/in_ch"]), float(fx["meta/dropout"])
    np_sd = make_state(in_ch, int(fx["meta/seed_w"]))
    sd = O.torch_state(np_sd, requires_grad=True)
    masks = {int(k.split("/")[1]): torch.from_numpy(fx[k]) for k in fx if k.startswith("mask/")}
    x = torch.from_numpy(fx["x"]).requires_grad_(True)
    out, saved = O.forward(sd, x, True, masks, p)
    loss = O.custom_loss(out, torch.from_numpy(fx["y"]), 0.9, float(fx["vgg"]))
    loss.backward()
    O.conv5_recompute_bn_update(sd, saved["p4"], mask=masks.get(5))
    assert np.abs(out.detach().numpy() - fx["out"]).max() <= OUT_ABS
    assert abs(loss.item() - float(fx["loss"])) <= LOSS_REL * abs(float(fx["loss"]))
    keys = O.param_keys(in_ch)
    fails = check_grads([(k, sd[k].grad.numpy()) for k in keys], fx)
    assert not fails, fails
    xg = x.grad.numpy()
    assert np.linalg.norm(xg - fx["x_grad"]) / np.linalg.norm(fx["x_grad"]) <= 1e-3
    for k in fx:
        if k.startswith("run/"):
            a = sd[k[4:]].numpy().astype(np.float64)
            assert np.abs(a - fx[k]).max() <= 1e-5, k


def test_oracle_perturbation_loss():
    fx = load("perturb_c4_b1_64")
    sd = _state_with_running(fx, 4, prefix="run_before/")
    x = torch.from_numpy(fx["x"])
    noises = [torch.from_numpy(n) for n in fx["noise"]]
    ps = O.perturb_inputs(x, noises)
    with torch.no_grad():
        pouts = [O.forward(sd, p, True, None, 0.0)[0] for p in ps]
    o = torch.from_numpy(fx["out"]).requires_grad_(True)
    loss = O.perturbation_loss(o, pouts)
    loss.backward()
    assert abs(loss.item() - float(fx["loss"])) <= 1e-6 * abs(float(fx["loss"]))
    assert np.abs(o.grad.numpy() - fx["out_grad"]).max() <= 1e-9
    for k in fx:
        if k.startswith("run/") and "running" in k:
            assert np.abs(sd[k[4:]].numpy() - fx[k]).max() <= 1e-5, k


def test_l1_grad_is_alpha_sign_over_n():
    """customLoss.py:90,160: d(loss)/d(out) = 0.9*sign(o-t)/N exactly."""
    fx = load("train_c7_p0_b2_64")
    o = torch.from_numpy(fx["out"]).requires_grad_(True)
    t = torch.from_numpy(fx["y"])
    O.custom_loss(o, t, 0.9, float(fx["vgg"])).backward()
    ref = 0.9 * torch.sign(o.detach() - t) / o.numel()
    assert torch.equal(o.grad, ref)


@pytest.mark.parametrize("name", ["vgg_b2_96x128", "vgg_b1_40x72"])
def test_oracle_vgg_loss_vs_reference(name):
    """oracle/vgg_ref.py restates MultiLayerVGGLoss: bitwise on the fixtures."""
    from oracle import vgg_ref as V
    fx = load(name)
    sd = V.standin_state()
    o, t = torch.from_numpy(fx["output"]), torch.from_numpy(fx["target"])
    assert V.vgg_loss(sd, o, t).item() == float(fx["vgg"])
    per = [v.item() for v in V.layer_losses(sd, o, t)]
    assert per == list(fx["layer_l1"])


def test_oracle_vgg_matches_train_fixture_vgg_term():
    """the stand-in VGG term inside the reference's CustomLoss (train fixture)."""
    from oracle import vgg_ref as V
    fx = load("train_c7_p0_b2_64")
    v = V.vgg_loss(V.standin_state(), torch.from_numpy(fx["out"]), torch.from_numpy(fx["y"])).item()
    assert abs(v - float(fx["vgg"])) <= 1e-6 * abs(v)


def test_oracle_temporal_instability():
    fx = load("temporal_b2_5f")
    frames = [torch.from_numpy(f) for f in fx["frames"]]
    assert O.temporal_instability(frames, 5.0).item() == float(fx["value_a5"])
    assert O.temporal_instability(frames, 3.0).item() == float(fx["value_a3"])
