"""GPU: the drop-in Unet / CustomLoss / PerturbationLoss (HIP path through the
C ABI) against the golden fixtures made by the reference code, and against
the CPU oracle at full resolution."""
import numpy as np
import pytest
import torch

from oracle import unet_ref as O
from oracle.weights import make_state, synthetic_batch
from util import GRAD_REL_L2, LOSS_REL, OUT_ABS, RUN_TOL, check_grads, load

pytestmark = pytest.mark.gpu
torch.set_num_threads(16)


def build(device, in_ch, dropout, np_sd, running=None):
    from nsm_amd import Unet
    m = Unet(in_ch=in_ch, dropout_rate=dropout)
    sd = {k: torch.from_numpy(v.copy()) for k, v in np_sd.items()}
    if running:
        sd.update({k: torch.from_numpy(v.copy()) for k, v in running.items()})
    m.load_state_dict(sd)
    return m.to(device)


def running_from(fx, prefix="run/"):
    return {k[len(prefix):]: v for k, v in fx.items() if k.startswith(prefix) and "running" in k}


@pytest.mark.parametrize("name", ["eval_c4_b2_64", "eval_c7_b1_odd_41x73"])
def test_eval_fixture(device, name):
    fx = load(name)
    in_ch = int(fx["meta/in_ch"])
    m = build(device, in_ch, 0.2, make_state(in_ch, int(fx["meta/seed_w"])), running_from(fx)).eval()
    with torch.no_grad():
        out = m(torch.from_numpy(fx["x"]).to(device)).cpu().numpy()
    assert out.shape == fx["out"].shape
    assert np.abs(out - fx["out"]).max() <= OUT_ABS


def train_step(device, fx):
    from nsm_amd import CustomLoss
    in_ch, p = int(fx["meta/in_ch"]), float(fx["meta/dropout"])
    m = build(device, in_ch, p, make_state(in_ch, int(fx["meta/seed_w"]))).train()
    masks = {int(k.split("/")[1]): torch.from_numpy(fx[k]) for k in fx if k.startswith("mask/")}
    if masks:
        m._inject_masks = masks
    x = torch.from_numpy(fx["x"]).to(device).requires_grad_(True)
    out = m(x)
    vgg = float(fx["vgg"])
    crit = CustomLoss(device, alpha=0.9, vgg=lambda o, t: vgg)
    loss = crit(out, torch.from_numpy(fx["y"]).to(device), x)
    loss.backward()
    torch.cuda.synchronize()
    return m, x, out, loss


@pytest.mark.parametrize("name", ["train_c7_p0_b2_64", "train_c4_drop_b2_64", "train_c4_p0_b1_40x72"])
def test_train_fixture(device, name):
    fx = load(name)
    m, x, out, loss = train_step(device, fx)
    assert np.abs(out.detach().cpu().numpy() - fx["out"]).max() <= OUT_ABS
    assert abs(loss.item() - float(fx["loss"])) <= LOSS_REL * abs(float(fx["loss"]))
    report = []
    fails = check_grads([(k, p.grad.cpu().numpy()) for k, p in m.named_parameters()], fx, report)
    assert not fails, (fails, sorted(report, key=lambda r: -r[1])[:8])
    xg = x.grad.cpu().numpy()
    assert np.linalg.norm(xg - fx["x_grad"]) / np.linalg.norm(fx["x_grad"]) <= GRAD_REL_L2
    sd = m.state_dict()
    for k in fx:
        if k.startswith("run/"):
            a = sd[k[4:]].cpu().numpy()
            if a.dtype == np.int64:
                assert (a == fx[k]).all(), k          # conv5 reads 2 (checkpoint recompute)
            else:
                assert np.abs(a - fx[k]).max() <= RUN_TOL * (1 + np.abs(fx[k]).max()), k


def test_train_deterministic(device):
    fx = load("train_c7_p0_b2_64")
    m1, x1, o1, _ = train_step(device, fx)
    m2, x2, o2, _ = train_step(device, fx)
    assert torch.equal(o1, o2)
    for (k, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a.grad, b.grad), k
    assert torch.equal(x1.grad, x2.grad)


def test_grads_share_one_flat_buffer(device):
    from nsm_amd import flat_grad
    fx = load("train_c4_p0_b1_40x72")
    m, _, _, _ = train_step(device, fx)
    g = flat_grad(list(m.parameters()))
    assert g is not None and g.numel() == sum(p.numel() for p in m.parameters())


def test_perturbation_fixture(device):
    from nsm_amd import PerturbationLoss
    fx = load("perturb_c4_b1_64")
    m = build(device, 4, 0.0, make_state(4, int(fx["meta/seed_w"])), running_from(fx, "run_before/")).train()
    x = torch.from_numpy(fx["x"]).to(device)
    out = torch.from_numpy(fx["out"]).to(device).requires_grad_(True)
    noises = [torch.from_numpy(n).to(device) for n in fx["noise"]]
    loss = PerturbationLoss()(m, x, out, noises=noises)
    loss.backward()
    ref = float(fx["loss"])
    # the loss is a mean |difference| of two nearly equal outputs: compare at the
    # output tolerance scale
    assert abs(loss.item() - ref) <= 2e-5 + 1e-2 * ref
    g = out.grad.cpu().numpy()
    agree = np.mean(np.sign(g) == np.sign(fx["out_grad"]))
    assert agree >= 0.99
    sd = m.state_dict()
    for k, v in running_from(fx).items():
        assert np.abs(sd[k].cpu().numpy() - v).max() <= RUN_TOL * (1 + np.abs(v).max()), k


@pytest.mark.parametrize("B,in_ch,H,W", [(2, 7, 512, 512)])
def test_train_full_res_vs_oracle(device, B, in_ch, H, W):
    """BASELINE config shape (7x512x512) at B=2: HIP train step vs CPU oracle."""
    from nsm_amd import CustomLoss
    np_sd = make_state(in_ch, 42)
    x_np, y_np = synthetic_batch(B, in_ch, H, W)
    m = build(device, in_ch, 0.0, np_sd).train()
    x = torch.from_numpy(x_np).to(device).requires_grad_(True)
    out = m(x)
    loss = CustomLoss(device, 0.9)(out, torch.from_numpy(y_np).to(device))
    loss.backward()
    sd = O.torch_state(np_sd, requires_grad=True)
    xo = torch.from_numpy(x_np).requires_grad_(True)
    oo, saved = O.forward(sd, xo, True, None, 0.0)
    lo = O.custom_loss(oo, torch.from_numpy(y_np), 0.9)
    lo.backward()
    assert (out.detach().cpu() - oo.detach()).abs().max().item() <= OUT_ABS
    assert abs(loss.item() - lo.item()) <= LOSS_REL * lo.item()
    worst = []
    for k, p in m.named_parameters():
        a, b = p.grad.cpu().double(), sd[k].grad.double()
        if k.endswith(".0.bias") or k.endswith(".4.bias"):
            assert (a - b).abs().max().item() <= 1e-6, k
            continue
        e = ((a - b).norm() / b.norm()).item()
        worst.append((e, k))
        assert e <= GRAD_REL_L2, (k, e)
    e = ((x.grad.cpu() - xo.grad).norm() / xo.grad.norm()).item()
    assert e <= GRAD_REL_L2


def test_eval_1080p_vs_oracle(device):
    """config 5 shape (7x1080x1920 inference): odd decoder resize at up6."""
    np_sd = make_state(7, 42)
    x_np, _ = synthetic_batch(1, 7, 1080, 1920)
    m = build(device, 7, 0.2, np_sd).eval()
    with torch.no_grad():
        out = m(torch.from_numpy(x_np).to(device)).cpu()
        ref, _ = O.forward(O.torch_state(np_sd), torch.from_numpy(x_np), training=False)
    assert out.shape == (1, 1, 1080, 1920)
    assert (out - ref).abs().max().item() <= OUT_ABS


@pytest.mark.gpu
def test_graphed_inference_matches_eager(device):
    """config 5 path: the hipGraph-captured eval forward equals the eager one bitwise
    and follows new inputs on replay."""
    import nsm_amd
    np_sd = make_state(7, 42)
    m = build(device, 7, 0.2, np_sd).eval()
    x1 = torch.from_numpy(synthetic_batch(1, 7, 96, 160)[0]).to(device)
    x2 = torch.randn(1, 7, 96, 160, device=device)
    g = nsm_amd.GraphedUnet(m, x1)
    with torch.no_grad():
        e1, e2 = m(x1), m(x2)
    assert torch.equal(g(x1), e1)
    assert torch.equal(g(x2), e2)
