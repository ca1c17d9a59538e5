"""GPU: the fp32 train step's numerics outside the random-init regime (VERDICT
r03, weak #1 / next #2). The h2 GEMM operands carry ONE power-of-two scale per
tensor (csrc/nsm_conv_split16.inc), so channels far below a tensor's maximum
get tensor-relative precision; train-mode BN (Unetmodel.py:22,27) renormalises
each channel. Here every conv weight's output channels and every BN gamma are
rescaled by 2^U(-12, 0), the input channels likewise, and a 5-step trajectory
(Dropout2d masks, CustomLoss, backward, the main.py:287-423 tail + AdamW) runs
in all three fp32 GEMM arithmetics (NSM_F32_SPLIT 0 = fp32 MFMA, 1 = bf16
split, 2 = f16x2 / h2 operands):
  * lockstep: at every step the GPU model is loaded with the oracle's
    trajectory state and must match its output (<= 1e-4 max-abs), loss
    (<= 1e-5 rel) and every gradient (<= 2e-2 rel-L2);
  * its own trajectory (FlatAdamW, sanitize + clip on the device): five
    AdamW steps amplify summation-order noise in every arithmetic (exact fp32
    included), so the h2 and bf16-split trajectories must stay within 1.5x the
    divergence of the fp32-MFMA trajectory from the oracle's.
Margins go to gpurun_out/parity_margins.json (profiles/r04/)."""
import numpy as np
import pytest
import torch

from oracle import unet_ref as O
from oracle.step_tail_ref import max_norm_for, sanitize_and_clip
from oracle.weights import block_channels, make_state, synthetic_batch
from test_gpu_model import build
from util import GRAD_REL_L2, LOSS_REL, OUT_ABS, is_pre_bn_bias, record_margin

pytestmark = pytest.mark.gpu
torch.set_num_threads(16)

B, C, H, W, P, STEPS, LR, WD, EPOCHS = 1, 7, 128, 128, 0.2, 5, 1e-3, 1e-3, 10


def spread_state(seed=3):
    """make_state(7, 42) with conv output channels and BN gammas scaled by 2^U(-12, 0)."""
    sd = make_state(C, 42)
    rng = np.random.default_rng(seed)
    for k, v in sd.items():
        if k.startswith("conv10"):
            continue
        if k.endswith(("conv.0.weight", "conv.4.weight")):
            sd[k] = (v * 2.0 ** rng.uniform(-12, 0, (v.shape[0], 1, 1, 1))).astype(np.float32)
        elif k.endswith(("conv.1.weight", "conv.5.weight")):
            sd[k] = (v * 2.0 ** rng.uniform(-12, 0, v.shape)).astype(np.float32)
    return sd


def batch(seed=4):
    x, y = synthetic_batch(B, C, H, W)
    rng = np.random.default_rng(seed)
    return (x * 2.0 ** rng.uniform(-12, 0, (1, C, 1, 1))).astype(np.float32), y


def step_masks(step):
    g = torch.Generator().manual_seed(100 + step)
    out = {}
    for k, (ci, _) in block_channels(C).items():
        pk = O.block_dropout(k, P)
        if pk > 0:
            out[k] = (torch.rand(B, ci, generator=g) >= pk).float() / (1 - pk)
    return out


_REF = {}


def oracle_trajectory():
    """The CPU oracle's 5 steps: per step (state before it, output, loss, grads)
    and the final state."""
    if _REF:
        return _REF
    np_sd = spread_state()
    x_np, y_np = batch()
    sd = O.torch_state(np_sd, requires_grad=True)
    keys = O.param_keys(C)
    params = [sd[k] for k in keys]
    opt = torch.optim.AdamW(params, lr=LR, weight_decay=WD)
    steps = []
    for s in range(STEPS):
        before = {k: v.detach().clone() for k, v in sd.items()}
        masks = step_masks(s)
        xo = torch.from_numpy(x_np)
        out, saved = O.forward(sd, xo, True, masks, P)
        loss = O.custom_loss(out, torch.from_numpy(y_np), 0.9)
        loss.backward()
        O.conv5_recompute_bn_update(sd, saved["p4"], mask=masks[5])
        grads = {k: sd[k].grad.detach().clone() for k in keys}
        steps.append((before, out.detach().clone(), loss.item(), grads, masks))
        skip = sanitize_and_clip(params, 0, EPOCHS)
        assert not skip
        opt.step()
        opt.zero_grad(set_to_none=True)
    _REF.update(steps=steps, final={k: v.detach().clone() for k, v in sd.items()},
                init={k: torch.from_numpy(v.copy()) for k, v in np_sd.items()}, x=x_np, y=y_np)
    return _REF


@pytest.fixture(params=[0, 1, 2], ids=["fp32mfma", "bf16x3", "h2"])
def split_mode(request, device):
    from nsm_amd import ops
    prev = ops.set_f32_split(request.param)
    yield request.param
    ops.set_f32_split(prev)


def test_spread_lockstep(device, split_mode):
    """At every step of the oracle's trajectory, from its state: output,
    loss and every gradient within the fp32 bounds."""
    import nsm_amd
    ref = oracle_trajectory()
    x = torch.from_numpy(ref["x"]).to(device)
    y = torch.from_numpy(ref["y"]).to(device)
    crit = nsm_amd.CustomLoss(device, 0.9, vgg_weights=False)
    worst_out, worst_loss, worst_g = 0.0, 0.0, []
    lock = build(device, C, P, {k: v.numpy() for k, v in ref["init"].items()}).train()
    for s, (before, out_r, loss_r, grads_r, masks) in enumerate(ref["steps"]):
        lock.load_state_dict({k: v.to(device) for k, v in before.items()})
        lock.zero_grad(set_to_none=True)
        lock._inject_masks = dict(masks)
        out = lock(x)
        loss = crit(out, y)
        loss.backward()
        torch.cuda.synchronize()
        e = (out.detach().cpu() - out_r).abs().max().item()
        le = abs(loss.item() - loss_r) / loss_r
        assert e <= OUT_ABS, (s, e)
        assert le <= LOSS_REL, (s, le)
        worst_out, worst_loss = max(worst_out, e), max(worst_loss, le)
        for k, prm in lock.named_parameters():
            a, b = prm.grad.cpu().double(), grads_r[k].double()
            if is_pre_bn_bias(k):     # analytically 0 (train-mode BN follows)
                assert (a - b).abs().max().item() <= 1e-6, (s, k)
                continue
            ge = ((a - b).norm() / b.norm()).item()
            assert ge <= GRAD_REL_L2, (s, k, ge)
            worst_g.append((ge, s, k))
    worst_g.sort(reverse=True)
    print(f"split {split_mode}: out {worst_out:.2e} loss {worst_loss:.2e} grads {worst_g[:3]}")
    record_margin(f"spread_lockstep_split{split_mode}", out_max_abs=worst_out, out_bound=OUT_ABS,
                  loss_rel=worst_loss, loss_bound=LOSS_REL,
                  worst_grad_rel_l2=[[k, s, e] for e, s, k in worst_g[:5]], grad_bound=GRAD_REL_L2,
                  steps=STEPS, spread="conv output channels, BN gamma, input channels x 2^U(-12,0)")


def _own_trajectory(device, mode, ref):
    """5 steps of the GPU model on its own gradients (FlatAdamW, the device
    tail) in fp32 GEMM arithmetic `mode`: divergence from the oracle's
    trajectory (parameter updates, final train-mode output)."""
    import nsm_amd
    from nsm_amd import ops
    prev = ops.set_f32_split(mode)
    try:
        x = torch.from_numpy(ref["x"]).to(device)
        y = torch.from_numpy(ref["y"]).to(device)
        crit = nsm_amd.CustomLoss(device, 0.9, vgg_weights=False)
        own = build(device, C, P, {k: v.numpy() for k, v in ref["init"].items()}).train()
        opt = nsm_amd.FlatAdamW(list(own.parameters()), lr=LR, weight_decay=WD,
                                max_grad_norm=max_norm_for(0, EPOCHS), sanitize=True, seed=1)
        for s in range(STEPS):
            own._inject_masks = dict(ref["steps"][s][4])
            opt.zero_grad(set_to_none=True)
            crit(own(x), y).backward()
            opt.step()
        torch.cuda.synchronize()
        assert opt.steps_taken() == STEPS
        own._inject_masks = dict(ref["steps"][0][4])
        with torch.no_grad():
            out_own = own(x).cpu()
    finally:
        ops.set_f32_split(prev)
    num = den = 0.0
    msd = own.state_dict()
    for k, v in ref["final"].items():
        if "running" in k or "num_batches" in k:
            continue
        du = msd[k].detach().cpu().double() - ref["init"][k].double()
        dr = v.double() - ref["init"][k].double()
        num += (du - dr).pow(2).sum().item()
        den += dr.pow(2).sum().item()
    sd_f = {k: v.clone() for k, v in ref["final"].items()}
    out_fin, _ = O.forward(sd_f, torch.from_numpy(ref["x"]), True, ref["steps"][0][4], P)
    return (num / den) ** 0.5, (out_own - out_fin).abs().max().item()


def test_spread_own_trajectory_no_worse_than_fp32(device):
    """Five Adam steps on the device's own gradients diverge from the CPU
    oracle's trajectory in EVERY arithmetic, exact fp32 MFMA included
    (measured: ~17 % of the update, 4 % of the elements' update signs, 0.06-0.09
    output max-abs): with channels spread over 2^12 many gradient elements sit
    at the summation-order noise of the large ones, and AdamW's first steps
    move each element by ~lr sign(g). The fp32 tolerance therefore applies to
    the lockstep comparison above; here the h2 (and bf16-split) trajectories
    must diverge no more than the exact fp32 MFMA trajectory does."""
    ref = oracle_trajectory()
    res = {m: _own_trajectory(device, m, ref) for m in (0, 1, 2)}
    print("own trajectory vs oracle (update rel-L2, final out max-abs):", res)
    record_margin("spread_own_trajectory", **{f"split{m}": list(v) for m, v in res.items()},
                  note="divergence from the oracle's trajectory; bound: 1.5x the fp32-MFMA run's")
    for m in (1, 2):
        assert res[m][0] <= 1.5 * res[0][0] + 1e-3, (m, res)
        assert res[m][1] <= 1.5 * res[0][1] + 1e-4, (m, res)
