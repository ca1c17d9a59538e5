"""The fp16-autocast mode (the reference's own GPU precision: main.py:175,
257-259 run the step under torch.amp.autocast(float16) with a GradScaler,
281/368): direct convolutions on IEEE-half operands, f16 activations and
activation gradients (csrc/nsm_conv_s16.inc compiled for f16, NSM_F16
elementwise kernels), fp32 accumulation / BN statistics / parameters / weight
gradients.

Anchor: the reference's own fp16-autocast deviation from fp32, measured on the
CPU oracle under torch.autocast('cpu', float16) with the same 2^16 loss scale
(GradScaler's initial scale), as test_gpu_configs.py anchors bf16."""
import numpy as np
import pytest
import torch

from oracle import unet_ref as O
from oracle.weights import make_state, synthetic_batch
from test_gpu_configs import masks_for
from test_gpu_model import _rel, build
from util import record_margin

pytestmark = pytest.mark.gpu
torch.set_num_threads(16)
SCALE = 65536.0   # GradScaler's initial scale (main.py:175)


@pytest.mark.parametrize("spread", [False, True], ids=["init", "spread"])
def test_f16_b64_small_res_vs_fp16_autocast_oracle(device, spread):
    """B=64 7x128x128 train step in f16 vs the fp32 oracle, within 1.5x of the
    reference's fp16-autocast deviation (output, x-grad, every weight grad;
    spread: test_gpu_spread.py's channel scales 2^U(-12,0))."""
    import nsm_amd
    from nsm_amd import ops
    B, C, H, W, p = 64, 7, 128, 128, 0.2
    np_sd = make_state(C, 42)
    x_np, y_np = synthetic_batch(B, C, H, W)
    if spread:
        from test_gpu_spread import spread_state
        np_sd = spread_state()
        rng = np.random.default_rng(4)
        x_np = (x_np * 2.0 ** rng.uniform(-12, 0, (1, C, 1, 1))).astype(np.float32)
    masks = masks_for(B, C, p, 6)
    m = build(device, C, p, np_sd).train().set_compute_dtype(torch.float16)
    assert m.activation_dtype() == ops.F16S
    m._inject_masks = dict(masks)
    x = torch.from_numpy(x_np).to(device).requires_grad_(True)
    out = m(x)
    loss = nsm_amd.CustomLoss(device, 0.9, vgg_weights=False)(out, torch.from_numpy(y_np).to(device), x)
    (loss * SCALE).backward()
    our_g = {k: prm.grad.cpu() / SCALE for k, prm in m.named_parameters()}
    our_xg = x.grad.cpu() / SCALE

    def oracle(autocast):
        sd = O.torch_state(np_sd, requires_grad=True)
        xo = torch.from_numpy(x_np).requires_grad_(True)
        with torch.autocast("cpu", dtype=torch.float16, enabled=autocast):
            oo, _ = O.forward(sd, xo, True, masks, p)
        oo = oo.float()
        (O.custom_loss(oo, torch.from_numpy(y_np), 0.9) * SCALE).backward()
        return (oo.detach(), xo.grad / SCALE,
                {k: sd[k].grad / SCALE for k in O.param_keys(C)})

    o32, xg32, g32 = oracle(False)
    o16, xg16, g16 = oracle(True)
    ref_out = (o16 - o32).abs().max().item()
    our_out = (out.detach().cpu() - o32).abs().max().item()
    ref_xg, ours_xg = _rel(xg16, xg32), _rel(our_xg, xg32)
    print(f"f16 B=64 128^2: out ours {our_out:.2e} ref-autocast {ref_out:.2e}; "
          f"x_grad ours {ours_xg:.2e} ref {ref_xg:.2e}")
    keys = [k for k in our_g if not (k.endswith(".0.bias") or k.endswith(".4.bias"))]
    ratios = sorted((((_rel(our_g[k], g32[k]) - 1e-2) / max(_rel(g16[k], g32[k]), 1e-12), k,
                      round(_rel(our_g[k], g32[k]), 4), round(_rel(g16[k], g32[k]), 4))
                     for k in keys), reverse=True)
    print("worst grad ratios (ours - 0.01) / ref-autocast:", ratios[:6])
    worst = ratios[0][:2]
    record_margin("f16_b64_128" + ("_spread" if spread else ""), out_max_abs=our_out,
                  out_bound=1.5 * ref_out, x_grad_rel_l2=ours_xg, x_grad_bound=1.5 * ref_xg,
                  worst_grad_ratio=worst[0], worst_grad=worst[1], grad_ratio_bound=1.5)
    assert our_out <= 1.5 * ref_out
    assert ours_xg <= 1.5 * ref_xg
    for k in keys:
        ours, ref = _rel(our_g[k], g32[k]), _rel(g16[k], g32[k])
        assert ours <= 1.5 * ref + 1e-2, (k, ours, ref)
    med = float(np.median([r[0] for r in ratios]))
    print(f"median grad ratio {med:.3f}")
    assert med <= 1.25, med


def test_fp16_autocast_runs_the_f16_kernels(device):
    """An unchanged main.py-style forward under torch.autocast('cuda',
    float16) runs the f16 path: the same output, bitwise, as
    set_compute_dtype(torch.float16), and fp32-close within f16 rounding."""
    import nsm_amd
    from nsm_amd import ops
    torch.manual_seed(0)
    m = nsm_amd.Unet(in_ch=4, dropout_rate=0.0).to(device).eval()
    x = torch.randn(1, 4, 64, 64, device=device)
    with torch.no_grad():
        ref = m(x)
        with torch.autocast("cuda", dtype=torch.float16):
            assert m.activation_dtype() == ops.F16S
            out = m(x)
        pinned = m.set_compute_dtype(torch.float16)(x)
    m.set_compute_dtype(None)
    assert out.dtype == torch.float32
    assert torch.equal(out, pinned)
    assert (out - ref).abs().max().item() < 2e-2


def test_f16_train_step_with_grad_scaler_semantics(device):
    """main.py's step at a tiny size: scaled loss backward, the device tail
    told the scale (FlatAdamW(grad_scale=...), main.py:361-368) — finite
    parameters after three steps, and a scale-invariant update (loss scales
    2^10 and 2^16 give the same parameters up to AdamW's sign sensitivity on
    near-zero gradients: |dp| <= 2 lr per step)."""
    import nsm_amd
    outs = []
    for scale in (1024.0, 65536.0):
        torch.manual_seed(3)
        m = nsm_amd.Unet(in_ch=7, dropout_rate=0.0).to(device).train()
        m.set_compute_dtype(torch.float16)
        opt = nsm_amd.FlatAdamW(m.parameters(), lr=1e-4, max_grad_norm=1.0, sanitize=True,
                                grad_scale=scale, seed=5)
        crit = nsm_amd.CustomLoss(device, 0.9, vgg_weights=False)
        g = torch.Generator(device=device).manual_seed(7)
        x = torch.randn(4, 7, 64, 64, device=device, generator=g)
        y = torch.rand(4, 1, 64, 64, device=device, generator=g)
        for _ in range(3):
            (crit(m(x), y, x) * scale).backward()
            opt.step()
            opt.zero_grad()
        flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        assert torch.isfinite(flat).all()
        outs.append(flat)
    d = (outs[0] - outs[1]).abs()
    assert d.max().item() <= 6e-4, d.max().item()
    assert d.mean().item() <= 1e-5, d.mean().item()
