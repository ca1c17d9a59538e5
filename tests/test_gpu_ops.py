"""GPU: each libnsm kernel family against the PyTorch-CPU fp32 op it replaces
(same seeded inputs), through the C ABI (nsm_amd.ops -> ctypes -> libnsm.so)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

torch.set_num_threads(8)


def nhwc(x):  # [B,C,H,W] -> [B*H*W, C]
    B, C, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(B * H * W, C).contiguous()


def nchw(y, B, H, W):
    return y.reshape(B, H, W, -1).permute(0, 3, 1, 2).contiguous()


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ops(device):
    from nsm_amd import ops as O
    return O


@pytest.mark.parametrize("B,H,W,ci,co,k", [(2, 9, 11, 32, 64, 3), (1, 16, 16, 64, 32, 3),
                                           (2, 8, 8, 128, 128, 3), (3, 7, 5, 32, 128, 1),
                                           (2, 32, 32, 64, 512, 1), (1, 5, 67, 32, 32, 3)])
def test_conv_fwd(ops, device, B, H, W, ci, co, k):
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + ci + co + k)
    x = torch.randn(B, ci, H, W, generator=g)
    w = torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5
    b = torch.randn(co, generator=g)
    ref = F.conv2d(x, w, b, padding=k // 2)
    wp = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_FWD)
    y = ops.conv_fwd(nhwc(x).to(device), B, H, W, wp, b.to(device), co, k)
    out = nchw(y.cpu(), B, H, W)
    assert (out - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("B,H,W,ci,co", [(2, 6, 7, 32, 64), (2, 16, 16, 128, 64)])
def test_conv1x1_prologue(ops, device, B, H, W, ci, co):
    g = torch.Generator().manual_seed(7)
    y1 = torch.randn(B, ci, H, W, generator=g)
    sc, sh = torch.rand(ci, generator=g) + 0.5, torch.randn(ci, generator=g)
    mask = (torch.rand(B, ci, generator=g) > 0.2).float() / 0.8
    w = torch.randn(co, ci, 1, 1, generator=g) / ci ** 0.5
    a = F.leaky_relu(y1 * sc[None, :, None, None] + sh[None, :, None, None], 0.2) * mask[:, :, None, None]
    ref = F.conv2d(a, w)
    wp = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_FWD)
    y = ops.conv_fwd(nhwc(y1).to(device), B, H, W, wp, None, co, 1,
                     pro=(sc.to(device), sh.to(device), mask.to(device)))
    assert (nchw(y.cpu(), B, H, W) - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()


@pytest.mark.parametrize("B,H,W,ci,co,k", [(2, 9, 11, 32, 64, 3), (2, 8, 8, 64, 64, 3),
                                           (2, 12, 12, 64, 128, 1)])
def test_conv_dgrad(ops, device, B, H, W, ci, co, k):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, ci, H, W, generator=g, requires_grad=True)
    w = torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5
    dy = torch.randn(B, co, H, W, generator=g)
    F.conv2d(x, w, padding=k // 2).backward(dy)
    wd = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_DGRAD)
    dx = ops.conv_fwd(nhwc(dy).to(device), B, H, W, wd, None, ci, k)
    assert rel(nchw(dx.cpu(), B, H, W), x.grad) <= 1e-5


@pytest.mark.parametrize("B,H,W,ci,co,k,pro", [(2, 9, 11, 32, 64, 3, False), (2, 16, 16, 64, 32, 3, False),
                                               (1, 33, 35, 128, 128, 3, False), (2, 8, 8, 32, 64, 1, True),
                                               (2, 16, 16, 128, 512, 1, True), (2, 64, 64, 32, 32, 3, False)])
def test_conv_wgrad(ops, device, B, H, W, ci, co, k, pro):
    g = torch.Generator().manual_seed(13)
    x = torch.randn(B, ci, H, W, generator=g)
    sc, sh = torch.rand(ci, generator=g) + 0.5, torch.randn(ci, generator=g)
    mask = (torch.rand(B, ci, generator=g) > 0.2).float() / 0.8
    a = F.leaky_relu(x * sc[None, :, None, None] + sh[None, :, None, None], 0.2) * mask[:, :, None, None] if pro else x
    w = (torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5).requires_grad_(True)
    dy = torch.randn(B, co, H, W, generator=g)
    F.conv2d(a, w, padding=k // 2).backward(dy)
    dw = torch.empty(co, ci, k, k, device=device)
    ops.conv_wgrad(nhwc(dy).to(device), nhwc(x).to(device), B, H, W, k, ci, co, dw,
                   pro=(sc.to(device), sh.to(device), mask.to(device)) if pro else None)
    assert rel(dw.cpu(), w.grad) <= 1e-5


# fp32 Winograd error grows with the tile: F(2x2) ~2x direct-conv rounding,
# F(4x4) (points 0, +-1, 1/2, -2) ~10x (measured with tools/wino_coeffs.py points
# in numpy fp32 vs float64: 2.1e-5 max-abs at unit-variance outputs, K=9216),
# F(6x6) (points 0, +-1, +-2, +-1/2) ~3-4x F(4x4) (1.25e-4 max-abs, 8.8e-6 rms
# at unit-variance outputs, K=4608).
WINO_TOL = {2: dict(fwd=5e-5, dgrad=2e-5, wgrad=2e-5), 4: dict(fwd=2e-4, dgrad=1e-4, wgrad=1e-4),
            6: dict(fwd=8e-4, dgrad=4e-4, wgrad=4e-4)}


@pytest.mark.parametrize("tile", [2, 4, 6])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 9, 11, 32, 64), (1, 16, 16, 256, 128), (2, 7, 5, 64, 32),
                                        (2, 32, 32, 512, 256), (1, 67, 120, 64, 64)])
def test_conv3x3_winograd(ops, device, B, H, W, ci, co, tile):
    """Winograd F(tile x tile, 3x3) forward and input-gradient vs F.conv2d / autograd."""
    g = torch.Generator().manual_seed(ci + co + H)
    x = torch.randn(B, ci, H, W, generator=g, requires_grad=True)
    w = torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5
    b = torch.randn(co, generator=g)
    ref = F.conv2d(x, w, b, padding=1)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    tol = WINO_TOL[tile]
    U = ops.wino_weight(w.to(device), co, ci, flip=False, tile=tile)
    y = ops.conv3x3_wino(nhwc(x.detach()).to(device), B, H, W, U, b.to(device), co, tile=tile)
    err = (nchw(y.cpu(), B, H, W) - ref.detach()).abs().max().item() / max(1.0, ref.abs().max().item())
    Ud = ops.wino_weight(w.to(device), ci, co, flip=True, tile=tile)
    dx = ops.conv3x3_wino(nhwc(dy).to(device), B, H, W, Ud, None, ci, tile=tile)
    derr = rel(nchw(dx.cpu(), B, H, W), x.grad)
    print(f"wino F({tile}) fwd max-rel {err:.2e} dgrad rel-l2 {derr:.2e}")
    assert err <= tol["fwd"]
    assert derr <= tol["dgrad"]


@pytest.mark.parametrize("tile", [2, 4, 6])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 9, 11, 32, 64), (1, 16, 16, 256, 128), (2, 7, 5, 64, 32),
                                        (2, 32, 32, 512, 256), (4, 64, 64, 64, 64)])
def test_conv3x3_wgrad_winograd(ops, device, B, H, W, ci, co, tile):
    """Winograd weight gradient (reusing the forward's V) vs autograd."""
    g = torch.Generator().manual_seed(ci * 3 + co + W)
    x = torch.randn(B, ci, H, W, generator=g)
    w = (torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5).requires_grad_(True)
    dy = torch.randn(B, co, H, W, generator=g)
    F.conv2d(x, w, padding=1).backward(dy)
    U = ops.wino_weight(w.detach().to(device), co, ci, flip=False, tile=tile)
    _, V = ops.conv3x3_wino(nhwc(x).to(device), B, H, W, U, None, co, tile=tile, keep_v=True)
    dw = torch.empty(co, ci, 3, 3, device=device)
    ops.conv3x3_wgrad_wino(nhwc(dy).to(device), V, B, H, W, ci, ci, co, dw, tile=tile)
    err = rel(dw.cpu(), w.grad)
    print(f"wino F({tile}) wgrad rel-l2 {err:.2e}")
    assert err <= WINO_TOL[tile]["wgrad"]


@pytest.mark.parametrize("tile", [2, 4, 6])
@pytest.mark.parametrize("B,hi,wi,H,W,ci,co", [(2, 8, 10, 16, 20, 64, 32), (1, 16, 16, 32, 32, 128, 128),
                                              (2, 5, 7, 10, 14, 32, 64), (1, 67, 120, 134, 240, 64, 32),
                                              (2, 4, 5, 7, 9, 32, 32)])
def test_wino_input_fused_resize(ops, device, B, hi, wi, H, W, ci, co, tile):
    """Winograd conv sampling a bilinear align_corners resize inside its input
    transform (nsm_wino_input_resize) == resize then Winograd conv, and == the
    PyTorch reference of interpolate + conv2d."""
    g = torch.Generator().manual_seed(hi * wi + ci + tile)
    x = torch.randn(B, ci, hi, wi, generator=g)
    w = torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5
    b = torch.randn(co, generator=g)
    ref = F.conv2d(F.interpolate(x, size=(H, W), mode="bilinear", align_corners=True), w, b,
                   padding=1)
    U = ops.wino_weight(w.to(device), co, ci, flip=False, tile=tile)
    xl = nhwc(x).to(device)
    y_f, V_f = ops.conv3x3_wino(xl, B, H, W, U, b.to(device), co, tile=tile, keep_v=True,
                                src_hw=(hi, wi))
    up = ops.resize(xl, B, hi, wi, H, W)
    y_u, V_u = ops.conv3x3_wino(up, B, H, W, U, b.to(device), co, tile=tile, keep_v=True)
    # the same interpolation formula; only FMA contraction may differ (1 ulp),
    # which the F(6x6) transforms amplify a few times
    assert rel(V_f.cpu(), V_u.cpu()) <= 2e-6
    assert rel(y_f.cpu(), y_u.cpu()) <= 1e-5
    err = (nchw(y_f.cpu(), B, H, W) - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err <= WINO_TOL[tile]["fwd"]


@pytest.mark.parametrize("tile", [2, 4, 6])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 9, 11, 32, 64), (1, 16, 16, 128, 128), (3, 7, 5, 64, 32),
                                        (2, 32, 32, 256, 1024), (8, 64, 64, 64, 64),
                                        (1, 67, 120, 32, 96), (8, 256, 256, 64, 64)])
def test_wino_output_bn_stats(ops, device, B, H, W, ci, co, tile):
    """BN batch statistics written by the Winograd output transform (counted
    partials, merged when > 1024 slots) == float64 statistics of the stored y,
    and the running-stat update of bn_train on them: the tuned slot count where
    it applies, the smallest valid one, and one > 1024 (merge)."""
    import math
    from nsm_amd._lib import lib
    g = torch.Generator().manual_seed(ci + co + H * tile)
    x = torch.randn(B, ci, H, W, generator=g)
    w = torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5
    b = torch.randn(co, generator=g) * 2 + 1  # a large mean, as a pre-BN conv output has
    U = ops.wino_weight(w.to(device), co, ci, flip=False, tile=tile)
    step = int(lib.nsm_wino_stat_step(co, tile))   # from the library's channels per thread
    assert step > 0
    tuned = int(lib.nsm_wino_stat_slots(B, H, W, co, tile))
    if (B, H, W) == (8, 256, 256):
        assert tuned > 1024  # conv8 / conv9 geometry: the stats form with a merge
    T = B * -(-H // tile) * -(-W // tile)
    if T >= step and os.environ.get("NSM_WINO_STAT_SMALL", "1") != "0":
        # every layer with a slot's worth of tiles takes the statistics form
        # (below the policy's slot count: one slot per tile, no bn_stats pass)
        assert tuned > 0 and tuned % step == 0, (T, step, tuned)
    for ns in sorted({tuned, step, step * -(-1100 // step)} - {0}):
        y, _, part = ops.conv3x3_wino(nhwc(x).to(device), B, H, W, U, b.to(device), co, tile=tile,
                                      stats=True, nslot=ns)
        assert part is not None and part.rpc == 0 and part.nchunk == ns
        yc = y.cpu().double()
        bn = torch.nn.BatchNorm2d(co).to(device)
        st = ops.bn_train(y, bn, co, 0.1, 1e-5, part=part)
        mean, var_b, var_u = yc.mean(0), yc.var(0, unbiased=False), yc.var(0, unbiased=True)
        inv = 1 / (var_b + 1e-5).sqrt()
        assert (st.mean.cpu().double() - mean).abs().max() <= 2e-6 * max(1.0, mean.abs().max().item())
        assert (st.invstd.cpu().double() - inv).abs().max() <= 2e-5 * inv.max()
        assert (bn.running_var.cpu().double() - (0.9 + 0.1 * var_u)).abs().max() <= 1e-4 * max(1.0, var_u.max().item())


def test_conv_padded_channels(ops, device):
    """conv2 of the 7-channel model: 28 real channels padded to 32."""
    B, H, W, ci, co = 2, 10, 12, 28, 28
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, ci, H, W, generator=g)
    w = torch.randn(co, ci, 3, 3, generator=g) / 16
    b = torch.randn(co, generator=g)
    ref = F.conv2d(x, w, b, padding=1)
    xp = F.pad(nhwc(x), (0, 4)).to(device)
    wp = ops.pack_conv_weight(w.to(device), 32, 32, ops.PACK_FWD)
    y = ops.conv_fwd(xp, B, H, W, wp, ops.pad_vec(b.to(device), 32), 32, 3).cpu()
    assert (nchw(y[:, :28], B, H, W) - ref).abs().max() <= 1e-4
    assert y[:, 28:].abs().max() == 0


@pytest.mark.parametrize("M,C", [(7, 32), (1000, 64), (4096 * 8 + 3, 128), (65536, 1024)])
def test_bn_train_stats(ops, device, M, C):
    g = torch.Generator().manual_seed(M)
    y = torch.randn(M, C, generator=g) * 3 + 5
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.1, 0.1)
    st = ops.bn_train(y.to(device), bn, C, 0.1, 1e-5)
    mean = y.double().mean(0)
    var_b = y.double().var(0, unbiased=False)
    var_u = y.double().var(0, unbiased=True)
    assert (st.mean.cpu().double() - mean).abs().max() <= 1e-5 * 5
    assert (st.invstd.cpu().double() - 1 / (var_b + 1e-5).sqrt()).abs().max() <= 1e-5
    assert (bn.running_mean.cpu().double() - 0.1 * mean).abs().max() <= 1e-5
    assert (bn.running_var.cpu().double() - (0.9 + 0.1 * var_u)).abs().max() <= 1e-4
    assert int(bn.num_batches_tracked.item()) == 1


def test_bn_act_and_bwd(ops, device):
    """bn_train -> bn_act -> bn_bwd against autograd of F.batch_norm+lrelu*mask."""
    B, C, H, W = 2, 64, 6, 5
    g = torch.Generator().manual_seed(5)
    y = (torch.randn(B, C, H, W, generator=g) * 2 + 1).requires_grad_(True)
    gamma = (torch.rand(C, generator=g) + 0.5).requires_grad_(True)
    beta = torch.randn(C, generator=g).requires_grad_(True)
    mask = (torch.rand(B, C, generator=g) > 0.3).float() / 0.7
    z = F.leaky_relu(F.batch_norm(y, None, None, gamma, beta, training=True), 0.2) * mask[:, :, None, None]
    gz = torch.randn(B, C, H, W, generator=g)
    z.backward(gz)
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    yd = nhwc(y.detach()).to(device)
    st = ops.bn_train(yd, bn, C, 0.1, 1e-5)
    zz = ops.bn_act(yd, st)
    zref = F.leaky_relu(F.batch_norm(y.detach(), None, None, gamma.detach(), beta.detach(), training=True), 0.2)
    assert (nchw(zz.cpu(), B, H, W) - zref).abs().max() <= 1e-5
    dg = torch.empty(C, device=device)
    db = torch.empty(C, device=device)
    dbias = torch.empty(C, device=device)
    dy = ops.bn_bwd(nhwc(gz).to(device), yd, st, H * W, mask.to(device), C, dg, db, dbias)
    assert rel(nchw(dy.cpu(), B, H, W), y.grad) <= 1e-5
    assert rel(dg.cpu(), gamma.grad) <= 1e-5
    assert rel(db.cpu(), beta.grad) <= 1e-5
    assert dbias.abs().max().item() <= 1e-5


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("recompute", [False, True])
@pytest.mark.parametrize("B,H,W,cip,cop,drop", [(2, 9, 11, 32, 64, True), (2, 16, 16, 64, 32, False),
                                                (2, 16, 16, 128, 64, True), (1, 32, 32, 512, 128, True),
                                                (2, 8, 8, 1024, 512, False), (2, 24, 40, 128, 512, True),
                                                (9, 128, 128, 64, 32, True)])
def test_conv1x1_dgrad_bn_bwd(ops, device, B, H, W, cip, cop, drop, recompute, dtype):
    """1x1 input gradient with the first BN's backward in the GEMM epilogue
    (nsm_conv1x1_dgrad_bnbwd, both schedules) vs autograd of
    conv1x1(lrelu(BN(y1)) * mask) and vs the unfused conv_fwd + bn_bwd path.
    The last shape has > 512 partial rows (nsm_sum_rows merge)."""
    g = torch.Generator().manual_seed(B * H + cip + cop)
    y1 = (torch.randn(B, cip, H, W, generator=g) * 1.5 + 0.3)
    w2 = torch.randn(cop, cip, 1, 1, generator=g) / cip ** 0.5
    dy2 = torch.randn(B, cop, H, W, generator=g)
    gamma = torch.rand(cip, generator=g) + 0.5
    beta = torch.randn(cip, generator=g) * 0.2
    mask = (torch.rand(B, cip, generator=g) > 0.2).float() / 0.8 if drop else None
    bf = dtype == "bf16"
    tdt = torch.bfloat16 if bf else torch.float32
    if bf:  # the reference sees the same bf16-representable inputs
        y1, w2, dy2 = (t.to(torch.bfloat16).float() for t in (y1, w2, dy2))
    yr = y1.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    a = F.leaky_relu(F.batch_norm(yr, None, None, gr, br, training=True), 0.2)
    if drop:
        a = a * mask[:, :, None, None]
    F.conv2d(a, w2).backward(dy2)

    bn = torch.nn.BatchNorm2d(cip).to(device)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    yd = nhwc(y1).to(device=device, dtype=tdt)
    st = ops.bn_train(yd, bn, cip, 0.1, 1e-5)
    wd = ops.pack_conv_weight(w2.to(device), cop, cip, ops.PACK_DGRAD, tdt)
    dyd = nhwc(dy2).to(device=device, dtype=tdt)
    md = mask.to(device) if drop else None
    outs = {}
    for fused in (True, False):
        dg, db, dbias = (torch.empty(cip, device=device) for _ in range(3))
        if fused:
            dy1 = ops.conv1x1_dgrad_bn_bwd(dyd, B, H, W, wd, yd, st, md, cip, dg, db, dbias,
                                           recompute)
        else:
            dA1 = ops.conv_fwd(dyd, B, H, W, wd, None, cip, 1)
            dy1 = ops.bn_bwd(dA1, yd, st, H * W, md, cip, dg, db, dbias)
        outs[fused] = (nchw(dy1.float().cpu(), B, H, W), dg.cpu(), db.cpu(), dbias.cpu())
    tol = 2e-2 if bf else 1e-5
    for fused in (True, False):
        dy1, dg, db, dbias = outs[fused]
        assert rel(dy1, yr.grad) <= tol, (fused, rel(dy1, yr.grad))
        assert rel(dg, gr.grad) <= tol
        assert rel(db, br.grad) <= tol
        assert dbias.abs().max().item() <= 1e-3 * max(1.0, br.grad.abs().max().item())
    # fused vs unfused: the same rounded dA1 and formulas, only the reduction order differs
    assert rel(outs[True][0], outs[False][0]) <= (4e-3 if bf else 2e-6)
    assert rel(outs[True][1], outs[False][1]) <= 1e-5
    assert rel(outs[True][2], outs[False][2]) <= 1e-5


@pytest.mark.parametrize("Hi,Wi,Ho,Wo", [(4, 5, 8, 10), (8, 10, 4, 5), (2, 4, 4, 8), (4, 8, 5, 9),
                                         (67, 120, 134, 240), (134, 240, 135, 240), (1, 1, 2, 2),
                                         (5, 5, 5, 5), (64, 64, 32, 32)])
def test_resize(ops, device, Hi, Wi, Ho, Wo):
    B, C = 2, 8
    g = torch.Generator().manual_seed(Hi * Wo)
    x = torch.randn(B, C, Hi, Wi, generator=g, requires_grad=True)
    ref = F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=True)
    gy = torch.randn(B, C, Ho, Wo, generator=g)
    ref.backward(gy)
    y = ops.resize(nhwc(x.detach()).to(device), B, Hi, Wi, Ho, Wo)
    assert (nchw(y.cpu(), B, Ho, Wo) - ref.detach()).abs().max() <= 1e-5
    dx = ops.resize_bwd(nhwc(gy).to(device), B, Hi, Wi, Ho, Wo)
    assert (nchw(dx.cpu(), B, Hi, Wi) - x.grad).abs().max() <= 1e-5 * max(1, x.grad.abs().max().item())


@pytest.mark.parametrize("h,w,th,tw", [(8, 10, 8, 10), (32, 32, 32, 32), (2, 4, 5, 9), (67, 120, 135, 240),
                                       (5, 7, 5, 7)])
def test_up2_resize_composite(ops, device, h, w, th, tw):
    """fused up x2 + _upsample_and_match == the two-step reference path."""
    B, C = 2, 8
    g = torch.Generator().manual_seed(h * 31 + tw)
    x = torch.randn(B, C, h, w, generator=g, requires_grad=True)
    ref = F.interpolate(F.interpolate(x, size=(2 * h, 2 * w), mode="bilinear", align_corners=True),
                        size=(th, tw), mode="bilinear", align_corners=True)
    gy = torch.randn(B, C, th, tw, generator=g)
    ref.backward(gy)
    y = ops.up2_resize(nhwc(x.detach()).to(device), B, h, w, th, tw)
    assert (nchw(y.cpu(), B, th, tw) - ref.detach()).abs().max() <= 1e-5
    dx = ops.up2_resize_bwd(nhwc(gy).to(device), B, h, w, th, tw)
    assert (nchw(dx.cpu(), B, h, w) - x.grad).abs().max() <= 2e-5 * max(1, x.grad.abs().max().item())


@pytest.mark.parametrize("kind,B,h,w,C", [("resize", 2, 32, 32, 128), ("resize", 1, 16, 24, 512),
                                          ("resize", 1, 8, 8, 1024), ("up2", 2, 64, 64, 64),
                                          ("up2", 1, 67, 120, 32), ("resize", 1, 270, 480, 16)])
def test_resize_bwd_channel_slices(ops, device, kind, B, h, w, C):
    """The separable backward (and the composite's separable forward) at the
    decoder's channel counts (several channel slices per row, x windows from
    LDS) against PyTorch-CPU fp32 autograd of the reference upsample (+ match
    for the composite); fp32 like the reference, whose source-index rounding
    the kernels reproduce."""
    g = torch.Generator().manual_seed(h * C + w)
    x = torch.randn(B, C, h, w, generator=g, requires_grad=True)
    if kind == "resize":
        th, tw = 2 * h, 2 * w
        ref = F.interpolate(x, size=(th, tw), mode="bilinear", align_corners=True)
    else:
        th, tw = 2 * h - 1, 2 * w + 3
        ref = F.interpolate(F.interpolate(x, size=(2 * h, 2 * w), mode="bilinear", align_corners=True),
                            size=(th, tw), mode="bilinear", align_corners=True)
    gy = torch.randn(B, C, th, tw, generator=g)
    ref.backward(gy)
    xd = nhwc(x.detach()).to(device)
    y = ops.resize(xd, B, h, w, th, tw) if kind == "resize" else ops.up2_resize(xd, B, h, w, th, tw)
    assert (nchw(y.cpu(), B, th, tw) - ref.detach()).abs().max().item() <= 1e-5
    dyd = nhwc(gy).to(device)
    dx = (ops.resize_bwd(dyd, B, h, w, th, tw) if kind == "resize"
          else ops.up2_resize_bwd(dyd, B, h, w, th, tw))
    err = (nchw(dx.cpu(), B, h, w) - x.grad).abs().max().item()
    assert err <= 2e-5 * max(1.0, x.grad.abs().max().item()), err


def test_resize_identity_bitwise(ops, device):
    x = torch.randn(3 * 7 * 9, 16, device=device)
    y = ops.resize(x, 3, 7, 9, 7, 9)
    assert torch.equal(x, y)


@pytest.mark.parametrize("H,W", [(8, 8), (7, 9), (135, 240)])
def test_avgpool(ops, device, H, W):
    B, C = 2, 16
    g = torch.Generator().manual_seed(H)
    x = torch.randn(B, C, H, W, generator=g, requires_grad=True)
    ref = F.avg_pool2d(x, 2)
    gy = torch.randn_like(ref)
    ref.backward(gy)
    skip = torch.randn(B, C, H, W, generator=g)
    y = ops.avgpool2(nhwc(x.detach()).to(device), B, H, W)
    assert (nchw(y.cpu(), B, H // 2, W // 2) - ref.detach()).abs().max() <= 1e-6
    dx = ops.avgpool2_bwd_add(nhwc(gy).to(device), B, H, W, nhwc(skip).to(device))
    assert (nchw(dx.cpu(), B, H, W) - (x.grad + skip)).abs().max() <= 1e-6


def test_input_prep_and_grad(ops, device):
    B, C, H, W = 2, 7, 6, 10
    x = torch.randn(B, C, H, W)
    X = ops.input_prep(x.to(device), 32).cpu()
    ref = nhwc(F.pixel_unshuffle(x, 2))
    assert torch.equal(X[:, :28], ref) and X[:, 28:].abs().max() == 0
    dx = ops.input_grad(X.to(device), B, C, H, W).cpu()
    assert torch.equal(dx, x)


def test_head(ops, device):
    B, Rh, Rw = 2, 5, 6
    g = torch.Generator().manual_seed(9)
    z = torch.randn(B, 16, Rh, Rw, generator=g, requires_grad=True)
    w = (torch.randn(4, 16, 1, 1, generator=g) * 0.3).requires_grad_(True)
    b = torch.randn(4, generator=g).requires_grad_(True)
    out = torch.sigmoid(F.pixel_shuffle(F.conv2d(z, w, b), 2))
    go = torch.randn_like(out)
    out.backward(go)
    zp = F.pad(nhwc(z.detach()), (0, 16)).to(device)
    o = ops.head_fwd(zp, B, Rh, Rw, w.detach().to(device), b.detach().to(device))
    assert (o.cpu() - out.detach()).abs().max() <= 1e-6
    dw = torch.empty(4, 16, 1, 1, device=device)
    db = torch.empty(4, device=device)
    dz = ops.head_bwd(go.to(device), o, zp, B, Rh, Rw, w.detach().to(device), dw, db).cpu()
    assert rel(nchw(dz[:, :16], B, Rh, Rw), z.grad) <= 1e-5 and dz[:, 16:].abs().max() == 0
    assert rel(dw.cpu(), w.grad) <= 1e-5 and rel(db.cpu(), b.grad) <= 1e-5


def test_l1_loss(device):
    from nsm_amd.losses import l1_loss
    g = torch.Generator().manual_seed(1)
    o = torch.rand(2, 1, 64, 64, generator=g)
    t = (torch.randint(0, 256, (2, 1, 64, 64), generator=g) / 255.0)
    t[0, 0, 0, :4] = o[0, 0, 0, :4]  # exact ties: sign(0) = 0
    oo = o.clone().requires_grad_(True)
    ref = 0.9 * F.l1_loss(oo, t)
    ref.backward()
    od = o.to(device).requires_grad_(True)
    loss = l1_loss(od, t.to(device), 0.9)
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 1e-6 * ref.item()
    assert torch.equal(od.grad.cpu(), oo.grad)


def test_adamw_clip(device):
    from nsm_amd.optim import FlatAdamW
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s)) for s in [(64, 16, 3, 3), (64,), (7,)]]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    dps = [torch.nn.Parameter(p.detach().clone().to(device)) for p in ps]
    opt_r = torch.optim.AdamW(ref, lr=7e-4, weight_decay=1e-3)
    opt = FlatAdamW(dps, lr=7e-4, weight_decay=1e-3, max_grad_norm=1.0)
    for step in range(3):
        grads = [torch.randn_like(p) * (step + 1) for p in ps]
        for p, gg in zip(ref, grads):
            p.grad = gg.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt_r.step()
        for p, gg in zip(dps, grads):
            p.grad = gg.to(device)
        opt.step()
    for a, b in zip(dps, ref):
        assert (a.detach().cpu() - b.detach()).abs().max() <= 1e-6


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("kind,B,h,w,C", [("pool", 2, 16, 18, 64), ("pool", 3, 9, 7, 1024),
                                          ("resize", 2, 8, 10, 128), ("resize", 1, 33, 20, 512),
                                          ("up2", 2, 16, 16, 64), ("up2", 1, 67, 120, 32)])
def test_grad_producer_bn_reduce(ops, device, kind, B, h, w, C, dtype):
    """The pooling / resize backward with the next BN's backward reduction fused
    (bnred=): the same gradient, and bn_bwd on its partials == bn_bwd with its
    own reduce pass (values, dgamma, dbeta)."""
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = torch.Generator().manual_seed(h * w + C)
    if kind == "pool":
        dy = torch.randn(B * (h // 2) * (w // 2), C, generator=g)
        skip = torch.randn(B * h * w, C, generator=g)
    elif kind == "resize":
        dy = torch.randn(B * (2 * h) * (2 * w), C, generator=g)
    else:  # up2 composite to a skip size that is not 2h x 2w
        th, tw = 2 * h - 1, 2 * w + 3
        dy = torch.randn(B * th * tw, C, generator=g)
    y2 = (torch.randn(B * h * w, C, generator=g) * 1.5 + 0.2).to(device=device, dtype=tdt)
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    st = ops.bn_train(y2, bn, C, 0.1, 1e-5)
    dyd = dy.to(device=device, dtype=tdt)

    def produce(bnred):
        if kind == "pool":
            return ops.avgpool2_bwd_add(dyd, B, h, w, skip.to(device=device, dtype=tdt), bnred=bnred)
        if kind == "resize":
            return ops.resize_bwd(dyd, B, h, w, 2 * h, 2 * w, bnred=bnred)
        return ops.up2_resize_bwd(dyd, B, h, w, th, tw, bnred=bnred)

    G0 = produce(None)
    G1, part = produce((y2, st))
    assert part is not None
    assert torch.equal(G0, G1)
    outs = []
    for p in (None, part):
        dg, db, dbias = (torch.empty(C, device=device) for _ in range(3))
        d = ops.bn_bwd(G1, y2, st, h * w, None, C, dg, db, dbias, part=p)
        outs.append((d.float().cpu(), dg.cpu(), db.cpu()))
    assert rel(outs[1][0], outs[0][0]) <= (4e-3 if dtype == "bf16" else 2e-6)
    assert rel(outs[1][1], outs[0][1]) <= 1e-5
    assert rel(outs[1][2], outs[0][2]) <= 1e-5


@pytest.mark.parametrize("tile", [2, 4, 6])
@pytest.mark.parametrize("B,H,W,C,drop", [(2, 9, 11, 32, True), (1, 16, 16, 128, False),
                                         (2, 37, 29, 64, True)])
def test_wino_dual_input_bn(ops, device, B, H, W, C, drop, tile):
    """nsm_wino_dual_input_bn (the first BN's backward formed per element
    inside the dual transform, dY1 never stored) == bn_bwd then
    wino_dual_input, and dgamma / dbeta / dbias identical."""
    g = torch.Generator().manual_seed(H * W + C + tile)
    y = (torch.randn(B * H * W, C, generator=g) * 1.3 + 0.4).to(device)
    gr = torch.randn(B * H * W, C, generator=g).to(device)
    mask = ((torch.rand(B, C, generator=g) > 0.2).float() / 0.8).to(device) if drop else None
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    st = ops.bn_train(y, bn, C, 0.1, 1e-5)
    outs = []
    for defer in (False, True):
        dg, db, dbias = (torch.empty(C, device=device) for _ in range(3))
        d = ops.bn_bwd(gr, y, st, H * W, mask, C, dg, db, dbias, defer=defer)
        Vd, dM = (ops.wino_dual_input_bn(d, y, st, mask, B, H, W, tile=tile) if defer
                  else ops.wino_dual_input(d, B, H, W, tile=tile))
        outs.append((Vd.cpu(), dM.cpu(), dg.cpu(), db.cpu(), dbias.cpu()))
    for a, b in zip(outs[0][:2], outs[1][:2]):
        assert rel(b, a) <= 1e-6
    for a, b in zip(outs[0][2:], outs[1][2:]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("tile", [2, 4, 6])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 9, 11, 32, 64), (1, 16, 16, 128, 128), (2, 37, 29, 64, 32)])
def test_wino_dual_input(ops, device, B, H, W, ci, co, tile):
    """nsm_wino_dual_input: both transforms of dy from one read == the separate
    input transform (dgrad) and the weight gradient's own dy transform."""
    g = torch.Generator().manual_seed(H * W + tile)
    x = nhwc(torch.randn(B, ci, H, W, generator=g)).to(device)
    dy = nhwc(torch.randn(B, co, H, W, generator=g)).to(device)
    w = torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5
    U = ops.wino_weight(w.to(device), co, ci, flip=False, tile=tile)
    Ud = ops.wino_weight(w.to(device), ci, co, flip=True, tile=tile)
    _, V = ops.conv3x3_wino(x, B, H, W, U, None, co, tile=tile, keep_v=True)
    Vd, dM = ops.wino_dual_input(dy, B, H, W, tile=tile)
    dx0 = ops.conv3x3_wino(dy, B, H, W, Ud, None, ci, tile=tile)
    dx1 = ops.conv3x3_wino(dy, B, H, W, Ud, None, ci, tile=tile, v_in=Vd)
    assert torch.equal(dx0, dx1)
    dw0 = torch.empty(co, ci, 3, 3, device=device)
    dw1 = torch.empty(co, ci, 3, 3, device=device)
    ops.conv3x3_wgrad_wino(dy, V, B, H, W, ci, ci, co, dw0, tile=tile)
    ops.conv3x3_wgrad_wino(dy, V, B, H, W, ci, ci, co, dw1, tile=tile, dM=dM)
    assert torch.equal(dw0, dw1)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("B,H,W,C", [(2, 16, 18, 64), (1, 9, 7, 128), (2, 5, 9, 512)])
def test_bn_act_pool_and_lazy_resize(ops, device, B, H, W, C, dtype):
    """bn_act_pool == bn_act then avgpool2 (bitwise); resize / up2_resize of a
    Lazy block output == bn_act(+res) then the resize (bitwise)."""
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    g = torch.Generator().manual_seed(H * W + C)
    y = (torch.randn(B * H * W, C, generator=g) * 2).to(device=device, dtype=tdt)
    res = torch.randn(B * H * W, C, generator=g).to(device=device, dtype=tdt)
    st = ops.BNState(C, device)
    st.scale.copy_(torch.rand(C, generator=g) + 0.5)
    st.shift.copy_(torch.randn(C, generator=g))
    z0 = ops.bn_act(y, st, 0.2)
    p0 = ops.avgpool2(z0, B, H, W)
    z1, p1 = ops.bn_act_pool(y, st, B, H, W, 0.2)
    assert torch.equal(z0, z1) and torch.equal(p0, p1)
    zr = ops.bn_act(y, st, 0.2, res=res)
    lazy = ops.Lazy(y, st, res)
    assert torch.equal(ops.resize(zr, B, H, W, 2 * H, 2 * W),
                       ops.resize_act(lazy, B, H, W, 2 * H, 2 * W, 0.2))
    th, tw = 2 * H - 1, 2 * W - 1
    a = ops.up2_resize_act(lazy, B, H, W, th, tw, 0.2)
    assert a is not None and torch.equal(ops.up2_resize(zr, B, H, W, th, tw), a)
