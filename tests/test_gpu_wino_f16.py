"""GPU: the bf16 path's Winograd F(4x4,3x3) forward on single-plane scaled
f16 operands (ops.conv3x3_wino_f16: nsm_wino_input_f16, prep kind 6,
nsm_wino_gemm_f16 on gemm_h2p/h2q in single-plane mode, nsm_wino_output_bf16)
against a float64 conv2d of the same bf16 input: its error stays within that of
the direct bf16 implicit GEMM it replaces (the reference's bf16-autocast
arithmetic for Unetmodel.py:21), and the BN partials written by the output
transform are those of the bf16-rounded outputs."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _prep_u(ops, w, cin_p, cout_p, device):
    """prep kind 6 (single-plane f16 U) through nsm_prep_weights, one job."""
    from nsm_amd import prep
    am = ops.amax_slots(1, device)
    U = torch.empty(36 * cout_p * cin_p, dtype=ops.H2, device=device)
    j = prep.NsmPrepJob()
    j.kind = prep.KIND_WINO_F16
    for i, v in enumerate((w.shape[0], w.shape[1], cout_p, cin_p, 0, 4, 0)):
        j.a[i] = v
    j.base = 0
    j.src = w.data_ptr()
    j.dst = U.data_ptr()
    j.amax = am.data_ptr()
    prep.run_jobs([j], device)
    torch.cuda.synchronize()
    return U, am


@pytest.mark.parametrize("m16", [False, True])
# (2, 32, 32, 512, 1024): the shape of the r04 fault record (call_r4_27, a
# pre-commit library; tests/test_gpu_guard.py audits it with guard regions);
# (3, 21, 27, 512, 1024): ragged tiles with co > ci
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 32, 32, 512, 512), (1, 37, 29, 512, 1024),
                                        (2, 32, 32, 512, 1024), (3, 21, 27, 512, 1024),
                                        (4, 16, 16, 1024, 512), (64, 8, 8, 512, 1024)])
def test_conv3x3_wino_f16_vs_direct_bf16(device, B, H, W, ci, co, m16):
    from nsm_amd import ops
    g = torch.Generator().manual_seed(B * H + W + ci)
    x = torch.randn(B, ci, H, W, generator=g) * torch.pow(2.0, torch.rand(1, ci, 1, 1, generator=g) * 4 - 2)
    w = torch.randn(co, ci, 3, 3, generator=g) / (9 * ci) ** 0.5
    b = torch.randn(co, generator=g) * 0.1
    xb = x.to(torch.bfloat16)
    ref = F.conv2d(xb.double(), w.double(), b.double(), padding=1)
    nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).contiguous()  # noqa: E731
    xd = nhwc(xb).to(device)
    ax = ops.amax_slots(1, device)
    ops.absmax(xd.float(), ax)   # (x's producer records it in the model path)
    U, au = _prep_u(ops, w.to(device).contiguous(), ci, co, device)
    y, part = ops.conv3x3_wino_f16(xd, B, H, W, U, b.to(device), co, amax=(ax, au), m16=m16)
    wp = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_FWD, torch.bfloat16)
    y0 = ops.conv_fwd(xd, B, H, W, wp, b.to(device), co, 3)
    torch.cuda.synchronize()
    r = nhwc(ref)
    e1 = (y.double().cpu() - r)
    e0 = (y0.double().cpu() - r)
    rms1, rms0 = e1.pow(2).mean().sqrt().item(), e0.pow(2).mean().sqrt().item()
    mx1, mx0 = e1.abs().max().item(), e0.abs().max().item()
    print(f"wino f16 (M16 {m16}) rms {rms1:.3e} max {mx1:.3e} | direct bf16 rms {rms0:.3e} "
          f"max {mx0:.3e} | ratio {rms1 / rms0:.3f} {mx1 / mx0:.3f}")
    assert rms1 <= 1.5 * rms0 and mx1 <= 2.0 * mx0, (rms1, rms0, mx1, mx0)
    if part is not None:
        bn = torch.nn.BatchNorm2d(co).to(device)
        st = ops.bn_train(y, bn, co, 0.1, 1e-5, part=part)
        yr = y.double()
        torch.testing.assert_close(st.mean.double(), yr.mean(0), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,H,W,c", [(2, 32, 32, 512), (1, 37, 29, 512), (4, 16, 16, 1024)])
def test_wgrad_wino_f16_vs_direct_bf16(device, B, H, W, c):
    """The weight gradient in the F(4x4) domain (nsm_wino_dout_f16 + the
    single-plane KM GEMMs + the filter transform) against a float64 weight
    gradient of the unrounded fp32 operands: within 2x the error of the direct
    bf16 weight gradient (whose error is the bf16 rounding of x and dY, as in
    the reference's bf16 autocast; the F(4x4) f16 operands add theirs)."""
    from nsm_amd import ops
    g = torch.Generator().manual_seed(B * H + W + c)
    x32 = torch.randn(B, c, H, W, generator=g)
    dy32 = torch.randn(B, c, H, W, generator=g) * 0.01
    x, dy = x32.to(torch.bfloat16), dy32.to(torch.bfloat16)
    w = torch.randn(c, c, 3, 3, generator=g) / (9 * c) ** 0.5
    xr = x32.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    F.conv2d(xr, wr, None, padding=1).backward(dy32.double())
    nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).contiguous()  # noqa: E731
    xd, dyd = nhwc(x).to(device), nhwc(dy).to(device)
    ax, ady = ops.amax_slots(1, device), ops.amax_slots(1, device)
    ops.absmax(xd.float(), ax)
    ops.absmax(dyd.float(), ady)
    U, au = _prep_u(ops, w.to(device).contiguous(), c, c, device)
    _, _, V = ops.conv3x3_wino_f16(xd, B, H, W, U, None, c, amax=(ax, au), stats=False, keep_v=True)
    dM = ops.wino_dout_f16(dyd, B, H, W, ady)
    dw = torch.empty(c, c, 3, 3, device=device)
    ops.conv3x3_wgrad_wino_f16(dM, V, B, H, W, c, c, c, c, dw, amax=(ady, ax))
    dw0 = torch.empty_like(dw)
    ops.conv_wgrad(dyd, xd, B, H, W, 3, c, c, dw0)
    torch.cuda.synchronize()
    r = wr.grad
    e1, e0 = dw.double().cpu() - r, dw0.double().cpu() - r
    rms1, rms0 = e1.pow(2).mean().sqrt().item(), e0.pow(2).mean().sqrt().item()
    print(f"wgrad wino f16 rms {rms1:.3e} | direct bf16 rms {rms0:.3e} | ref rms {r.pow(2).mean().sqrt().item():.3e}")
    assert rms1 <= 2.0 * rms0, (rms1, rms0)


@pytest.mark.parametrize("B,H,W,c", [(2, 32, 32, 512), (1, 37, 29, 128), (3, 13, 22, 256)])
def test_wino_dual_f16_matches_separate_transforms(device, B, H, W, c):
    """nsm_wino_dual_f16 (one read of dY) writes exactly the V of
    nsm_wino_input_f16 and the dM of nsm_wino_dout_f16 (same arithmetic,
    same scale slot), ragged edges included."""
    from nsm_amd import ops
    g = torch.Generator().manual_seed(B * H * W + c)
    dy = (torch.randn(B * H * W, c, generator=g) * 1e-3).to(torch.bfloat16).to(device)
    am = ops.amax_slots(1, device)
    ops.absmax(dy.float(), am)
    V, dM = ops.wino_dual_f16(dy, B, H, W, am)
    V0 = torch.empty_like(V)
    ops.call("nsm_wino_input_f16", ops.ptr(dy), dy.stride(0), B, H, W, c, 4, ops.ptr(V0), ops.ptr(am),
             ops.stream())
    dM0 = ops.wino_dout_f16(dy, B, H, W, am)
    torch.cuda.synchronize()
    assert torch.equal(V.view(torch.int16), V0.view(torch.int16))
    assert torch.equal(dM.view(torch.int16), dM0.view(torch.int16))
    assert V.abs().max().item() > 0 and dM.abs().max().item() > 0


@pytest.mark.parametrize("drop", [False, True])
@pytest.mark.parametrize("B,H,W,c", [(2, 32, 32, 512), (1, 37, 29, 128), (3, 13, 22, 256)])
def test_wino_dual_bn_f16_matches_apply_then_dual(device, B, H, W, c, drop):
    """nsm_wino_dual_bn_f16 (the bf16 path's lazy dY1: the first BN's backward
    formed per element inside the F(4x4) dual transform) writes the V and dM
    of nsm_bn_bwd_apply's stored dY1 followed by nsm_wino_dual_f16, under the
    same scale slot (the finalize's dY1 bound, which dominates max|dY1|):
    equal up to FMA-contraction ulps of the per-element dY1."""
    from nsm_amd import ops
    g = torch.Generator().manual_seed(B * H * W + c + int(drop))
    M = B * H * W
    y = (torch.randn(M, c, generator=g) * 2 + 0.5).to(torch.bfloat16).to(device)
    gr = (torch.randn(M, c, generator=g) * 1e-2).to(torch.bfloat16).to(device)
    mask = ((torch.rand(B, c, generator=g) > 0.2).float() / 0.8).to(device) if drop else None
    bn = torch.nn.BatchNorm2d(c).to(device)
    with torch.no_grad():
        bn.weight.copy_(torch.randn(c, generator=g))
        bn.bias.uniform_(-0.2, 0.2)
    st = ops.bn_train(y, bn, c, 0.1, 1e-5)
    slots = ops.amax_slots(2, device)
    k1dz, bnd = ops.amax_slot(slots, 0), ops.amax_slot(slots, 1)
    z = [torch.zeros(c, device=device) for _ in range(6)]
    d = ops.bn_bwd(gr, y, st, H * W, mask, c, *z[:3], defer=True, h2=(k1dz, bnd))
    V1, dM1 = ops.wino_dual_bn_f16(d, y, st, mask, B, H, W, bnd)
    dy = ops.bn_bwd(gr, y, st, H * W, mask, c, *z[3:])
    V0, dM0 = ops.wino_dual_f16(dy, B, H, W, bnd)
    torch.cuda.synchronize()
    bound = torch.frombuffer(bytearray(bnd.cpu().numpy().tobytes()), dtype=torch.float32).max().item()
    assert bound >= dy.float().abs().max().item()
    for name, a, b in (("V", V1, V0), ("dM", dM1, dM0)):
        a, b = a.float(), b.float()
        diff = (a - b).abs()
        frac = (diff > 0).float().mean().item()
        print(f"{name}: mismatched {frac:.2e}, max diff {diff.max().item():.3e} of {b.abs().max().item():.3e}")
        assert torch.isfinite(a).all() and b.abs().max().item() > 0
        assert frac <= 2e-3 and diff.max().item() <= 2.0 ** -5 * b.abs().max().item(), (name, frac)


@pytest.mark.parametrize("B,hi,wi,c", [(2, 16, 16, 512), (1, 17, 30, 512), (3, 8, 11, 1024)])
def test_wino_input_f16_resize_matches_materialised_upsample(device, B, hi, wi, c):
    """nsm_wino_input_f16_resize (the decoder's x2 upsample sampled inside the
    F(4x4) input transform, each value rounded to bf16) equals the transform
    of the materialised bf16 upsample (nsm_resize_fwd, then nsm_wino_input_f16)
    under the same scale slot, up to FMA-contraction ulps of the interpolation."""
    from nsm_amd import ops
    g = torch.Generator().manual_seed(B * hi * wi + c)
    x = torch.randn(B * hi * wi, c, generator=g).to(torch.bfloat16).to(device)
    H, W = 2 * hi, 2 * wi
    am = ops.amax_slots(1, device)
    ops.absmax(x, am)
    T = ops.wino_tiles(B, H, W, 4)
    V1 = torch.empty(36 * T * c, dtype=ops.H2, device=device)
    ops.call("nsm_wino_input_f16_resize", ops.ptr(x), x.stride(0), B, hi, wi, H, W, c, 4, ops.ptr(V1),
             ops.ptr(am), ops.stream())
    up = ops.resize(x, B, hi, wi, H, W)
    V0 = torch.empty_like(V1)
    ops.call("nsm_wino_input_f16", ops.ptr(up), up.stride(0), B, H, W, c, 4, ops.ptr(V0), ops.ptr(am),
             ops.stream())
    torch.cuda.synchronize()
    a, b = V1.float(), V0.float()
    diff = (a - b).abs()
    frac = (diff > 0).float().mean().item()
    print(f"mismatched {frac:.2e}, max diff {diff.max().item():.3e} of {b.abs().max().item():.3e}")
    assert b.abs().max().item() > 0 and torch.isfinite(a).all()
    assert frac <= 2e-3 and diff.max().item() <= 2.0 ** -6 * b.abs().max().item()
