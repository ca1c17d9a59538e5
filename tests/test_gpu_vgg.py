"""VGG19 perceptual loss (customLoss.py:7-90) on the libnsm kernels vs the
reference's own values (tests/golden/vgg_*.npz, made by running
customLoss.MultiLayerVGGLoss with the stand-in VGG19 weights) and vs the
oracle restatement at a larger size."""
import numpy as np
import pytest
import torch

from oracle import vgg_ref as V
from util import load

pytestmark = pytest.mark.gpu

VGG_REL = 2e-5   # fp32; Winograd F(4x4) feature error ~1e-6 relative, averaged by the L1 mean


def module(device):
    import nsm_amd
    return nsm_amd.MultiLayerVGGLoss(device, state_dict=V.standin_state())


@pytest.mark.parametrize("name", ["vgg_b2_96x128", "vgg_b1_40x72"])
def test_vgg_vs_reference_fixture(device, name):
    g = load(name)
    m = module(device)
    o = torch.from_numpy(g["output"]).to(device)
    t = torch.from_numpy(g["target"]).to(device)
    val = m(o, t).item()
    ref = float(g["vgg"])
    per = np.array([v.item() for v in m.last_terms]) / np.asarray(g["weights"], np.float64)
    print(f"{name}: vgg {val:.8e} ref {ref:.8e}; per-layer rel "
          f"{np.abs(per - g['layer_l1']) / np.abs(g['layer_l1'])}")
    assert abs(val - ref) <= VGG_REL * abs(ref)
    np.testing.assert_allclose(per, g["layer_l1"], rtol=VGG_REL)


def test_vgg_vs_oracle_256(device):
    gen = torch.Generator().manual_seed(3)
    o = torch.sigmoid(torch.randn(2, 1, 256, 256, generator=gen))
    t = torch.rand(2, 1, 256, 256, generator=gen)
    ref = V.vgg_loss(V.standin_state(), o, t).item()
    val = module(device)(o.to(device), t.to(device)).item()
    assert abs(val - ref) <= VGG_REL * abs(ref)


@pytest.mark.parametrize("name", ["train_c7_p0_b2_64", "train_c4_drop_b2_64"])
def test_custom_loss_with_vgg_vs_reference(device, name):
    """CustomLoss value incl. the VGG term = the reference's loss on the same
    (output, label) pair (the fixture's loss used the same stand-in VGG)."""
    import nsm_amd
    g = load(name)
    crit = nsm_amd.CustomLoss(device, alpha=0.9, vgg_weights=V.standin_state())
    o = torch.from_numpy(g["out"]).to(device).requires_grad_(True)
    y = torch.from_numpy(g["y"]).to(device)
    loss = crit(o, y, None)
    assert abs(loss.item() - float(g["loss"])) <= 1e-5 * abs(float(g["loss"]))
    loss.backward()   # the VGG term is a detached constant: grad = 0.9*sign(o-y)/N
    ref = 0.9 * torch.sign(o.detach() - y) / o.numel()
    torch.testing.assert_close(o.grad, ref, rtol=1e-6, atol=0)
