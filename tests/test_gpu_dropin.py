"""GPU: drop-in behaviours of the reference surface that are not arithmetic.

  * the `assert output.min() >= 0 and output.max() <= 1` of CustomLoss
    (customLoss.py:131) and EnhancedCustomLoss (pert_loss.py:131): a device flag
    here; an out-of-range or NaN output raises AssertionError at the next call
    once the flag has landed in host memory, and at once via check_range_now();
  * the VGG19 perceptual loss built from a torchvision-layout checkpoint file
    (customLoss.py:20: `models.vgg19(weights=IMAGENET1K_V1)`; here a local .pth
    loaded with weights_only=True) equals the module built from the same
    weights directly;
  * main.py:257's fp16 autocast region: this path has fp32 and bf16 kernels,
    so it warns and runs fp32 (bitwise the fp32 result)."""

import pytest
import torch

from oracle import vgg_ref as V

pytestmark = pytest.mark.gpu


def _crit(device):
    import nsm_amd
    return nsm_amd.CustomLoss(device, alpha=0.9, vgg_weights=False)


@pytest.mark.parametrize("bad", [1.5, -0.25, float("nan")])
def test_range_assert_check_now(device, bad):
    crit = _crit(device)
    y = torch.rand(2, 1, 32, 32, device=device)
    o = torch.rand(2, 1, 32, 32, device=device)
    crit(o, y, None)
    crit.check_range_now()            # in range: nothing raised
    o[1, 0, 3, 5] = bad
    crit(o, y, None)
    with pytest.raises(AssertionError, match=r"customLoss.py:131"):
        crit.check_range_now()
    crit.check_range_now()            # the flag is cleared once reported


def test_range_assert_raises_at_next_call(device):
    crit = _crit(device)
    y = torch.rand(1, 1, 16, 16, device=device)
    o = torch.rand(1, 1, 16, 16, device=device)
    o[0, 0, 0, 0] = 2.0
    crit(o, y, None)
    torch.cuda.synchronize()          # the flag's async copy has landed
    with pytest.raises(AssertionError):
        crit(torch.rand(1, 1, 16, 16, device=device), y, None)


def test_enhanced_loss_range_assert(device):
    import nsm_amd
    crit = nsm_amd.EnhancedCustomLoss(device, vgg_weights=False).eval()
    o = torch.rand(1, 1, 16, 16, device=device)
    o[0, 0, 2, 2] = 1.01
    crit(None, o, torch.rand_like(o), None)
    with pytest.raises(AssertionError):
        crit.base.check_range_now()


def test_vgg_from_torchvision_checkpoint(device, tmp_path):
    """A torchvision vgg19 state_dict layout ('features.N.*' + 'classifier.*'),
    torch.save'd and loaded through from_torchvision_checkpoint / CustomLoss's
    path argument, reproduces the module built from the same weights."""
    import nsm_amd
    sd = V.standin_state()
    tv = {f"features.{k}": v for k, v in sd.items()}
    g = torch.Generator().manual_seed(5)
    tv.update({"classifier.0.weight": torch.randn(8, 8, generator=g),
               "classifier.0.bias": torch.zeros(8)})
    path = tmp_path / "vgg19-dcbb9e9d.pth"
    torch.save(tv, path)
    o = torch.sigmoid(torch.randn(2, 1, 64, 96, generator=g)).to(device)
    t = torch.rand(2, 1, 64, 96, generator=g).to(device)
    want = nsm_amd.MultiLayerVGGLoss(device, state_dict=sd)(o, t).item()
    got = nsm_amd.MultiLayerVGGLoss.from_torchvision_checkpoint(str(path), device)(o, t).item()
    assert got == want
    crit = nsm_amd.CustomLoss(device, alpha=0.9, vgg_weights=str(path))
    loss = crit(o, t, None).item()
    l1 = (o - t).abs().mean().item()
    assert abs(loss - (0.9 * l1 + 0.1 * want)) <= 1e-6 * abs(loss)
    ref = V.vgg_loss(sd, o.cpu(), t.cpu()).item()   # the oracle on the same weights
    assert abs(got - ref) <= 2e-5 * abs(ref)
