"""GPU: the DoubleConv's 1x1 convolution (Unetmodel.py:26) on pre-split f16x2
operands (csrc/nsm_conv_h2d.inc) — forward with the BN-statistics epilogue,
input gradient with the first BN's backward in its epilogue, weight gradient —
and the producers of its operands: nsm_bn_act_h2 (scale from the Samuelson
bound nsm_bn_finalize_train records), nsm_to_h2, prep kind 5. Against a
float64 reference the error stays within that of the exact fp32-MFMA path on
the same inputs (the bounds of tests/test_gpu_split.py); every shape class of
the tile policy is run."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(device):
    from nsm_amd import ops as O
    prev = O.set_f32_split(2)
    yield O
    O.set_f32_split(prev)


def _errs(a, ref):
    d = (a.double() - ref).abs()
    return d.max().item(), d.pow(2).mean().sqrt().item()


def _slot_max(slot):
    """max of an operand-maximum slot (fp32 bits as uint32)."""
    v = slot.view(torch.int32).cpu().numpy().astype(np.uint32).max()
    return float(np.array(v, dtype=np.uint32).view(np.float32))


def _spread(g, n, lo=-12, hi=0):
    """per-channel scales 2^U(lo, hi)."""
    return torch.pow(2.0, torch.rand(n, generator=g, dtype=torch.float64) * (hi - lo) + lo)


# (M, cin_p, cout_p): the forward tiles 256x256, 256x128, 256x64, 128x128,
# 128x64, 128x32 (nsm_conv_h2d.inc h2d_tile) and the K = 32 / 64 edges
SHAPES = [(32768, 1024, 512), (65536, 512, 128), (131072, 128, 64), (2048, 256, 256),
          (4096, 64, 64), (6000, 64, 32), (8192, 32, 64), (1000, 128, 1024)]


@pytest.mark.parametrize("M,cin_p,cout_p", SHAPES)
def test_conv1x1_h2_fwd_wgrad(ops, device, M, cin_p, cout_p):
    g = torch.Generator().manual_seed(M + cin_p + cout_p)
    x = torch.randn(M, cin_p, generator=g, dtype=torch.float64) * _spread(g, cin_p, -6, 0)
    w = torch.randn(cout_p, cin_p, generator=g, dtype=torch.float64) / cin_p ** 0.5
    b = torch.randn(cout_p, generator=g, dtype=torch.float64) * 0.1
    dy = torch.randn(M, cout_p, generator=g, dtype=torch.float64) * _spread(g, cout_p, -6, 0)
    x, w, b, dy = (t.to(device) for t in (x, w, b, dy))   # float64 references on the GPU
    ref = x @ w.T + b
    dw_ref = dy.T @ x
    xs, ws, bs, dys = (t.float().contiguous() for t in (x, w, b, dy))
    w4 = ws.view(cout_p, cin_p, 1, 1)
    am = ops.amax_slots(3, device)
    ax, aw, ady = (ops.amax_slot(am, i) for i in range(3))
    ops.absmax(xs, ax)
    ops.absmax(ws, aw)
    ops.absmax(dys, ady)
    xh, wh, dyh = ops.to_h2(xs, ax), ops.to_h2(ws, aw), ops.to_h2(dys, ady)
    y, part = ops.conv1x1_h2(xh, wh, bs, cout_p, stats=True, amax=(ax, aw))
    dw = torch.empty(cout_p, cin_p, 1, 1, device=device)
    ops.conv1x1_wgrad_h2(dyh, xh, cin_p, cout_p, dw, amax=(ady, ax))
    # the exact fp32 MFMA path on the same fp32 operands
    prev = ops.set_f32_split(0)
    try:
        wpk = ops.pack_conv_weight(w4, cout_p, cin_p, ops.PACK_FWD)
        y0, part0 = ops.conv_fwd_bn(xs, 1, 1, M, wpk, bs, cout_p, 1, stats=True)
        dw0 = torch.empty_like(dw)
        ops.conv_wgrad(dys, xs, 1, 1, M, 1, cin_p, cout_p, dw0)
    finally:
        ops.set_f32_split(prev)
    torch.cuda.synchronize()
    for got, base, r in ((y, y0, ref), (dw.view(cout_p, cin_p), dw0.view(cout_p, cin_p), dw_ref)):
        r = r.to(device)
        (mx, rms), (mx0, rms0) = _errs(got, r), _errs(base, r)
        assert rms <= 1.5 * rms0 + 1e-12 and mx <= 2.0 * mx0 + 1e-12, (mx, rms, mx0, rms0)
    # BN batch statistics of y from the epilogue's partials
    bn = torch.nn.BatchNorm2d(cout_p).to(device)
    st = ops.bn_train(y, bn, cout_p, 0.1, 1e-5, part=part)
    yd = ref.to(device)
    mean_ref, var_ref = yd.mean(0), yd.var(0, unbiased=False)
    torch.testing.assert_close(st.mean.double(), mean_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st.invstd.double(), (var_ref + 1e-5).rsqrt(), rtol=1e-4, atol=0)


@pytest.mark.parametrize("recompute", [False, True])
@pytest.mark.parametrize("M,HW,cip,cop", [(32768, 4096, 1024, 512), (65536, 4096, 512, 128),
                                          (131072, 16384, 128, 64), (4096, 1024, 64, 32),
                                          (8192, 4096, 32, 64)])
def test_conv1x1_dgrad_bnbwd_h2(ops, device, M, HW, cip, cop, recompute):
    """dY1 = BN1 backward of dA1 = dY2 W2 (h2 GEMM with the EpiBnBwd epilogue)
    against the same op on the exact fp32 MFMA (nsm_conv1x1_dgrad_bnbwd mode
    0 arithmetic), both vs a float64 restatement."""
    g = torch.Generator().manual_seed(M + cip * 3 + cop + int(recompute))
    B = M // HW
    dY2 = torch.randn(M, cop, generator=g, dtype=torch.float64) * _spread(g, cop, -4, 0)
    w = torch.randn(cop, cip, generator=g, dtype=torch.float64) / cop ** 0.5
    Y1 = torch.randn(M, cip, generator=g, dtype=torch.float64) * _spread(g, cip, -4, 2)
    gamma = torch.randn(cip, generator=g, dtype=torch.float64) * _spread(g, cip, -4, 0)
    beta = torch.randn(cip, generator=g, dtype=torch.float64) * 0.1
    mask = (torch.rand(B, cip, generator=g) > 0.2).double() / 0.8
    dY2, w, Y1, gamma, beta, mask = (t.to(device) for t in (dY2, w, Y1, gamma, beta, mask))
    # float64 reference: dA1 = dY2 W, dz = dA1 lrelu'(BN(Y1)) mask, BN backward
    mu, var = Y1.mean(0), Y1.var(0, unbiased=False)
    inv = (var + 1e-5).rsqrt()
    xhat = (Y1 - mu) * inv
    z = xhat * gamma + beta
    dz = (dY2 @ w) * torch.where(z > 0, 1.0, 0.2) * mask.repeat_interleave(HW, 0)
    ref = gamma * inv * (dz - dz.mean(0) - xhat * (dz * xhat).mean(0))
    dev = lambda t: t.float().to(device).contiguous()  # noqa: E731
    dY2s, ws, Y1s = dev(dY2), dev(w), dev(Y1)
    bn = torch.nn.BatchNorm2d(cip).to(device)
    with torch.no_grad():
        bn.weight.copy_(gamma.float())
        bn.bias.copy_(beta.float())
    st = ops.bn_train(Y1s, bn, cip, 0.1, 1e-5)
    maskd = dev(mask)
    am = ops.amax_slots(3, device)
    ady, aw, aout = (ops.amax_slot(am, i) for i in range(3))
    ops.absmax(dY2s, ady)
    w4 = ws.view(cop, cip, 1, 1)
    wd = ops.pack_conv_weight(w4, cop, cip, ops.PACK_DGRAD)   # [cip][cop]
    ops.absmax(wd, aw)
    dY2h, wdh = ops.to_h2(dY2s, ady), ops.to_h2(wd.view(cip, cop), aw)
    outs = {}
    for name in ("h2", "fp32"):
        gr = [torch.zeros(cip, device=device) for _ in range(3)]
        if name == "h2":
            dy = ops.conv1x1_dgrad_bn_bwd_h2(dY2h, HW, wdh, Y1s, st, maskd, cip, *gr, recompute,
                                             amax=(ady, aw), amax_out=aout)
        else:
            prev = ops.set_f32_split(0)
            try:
                dy = ops.conv1x1_dgrad_bn_bwd(dY2s, B, 1, HW, wd, Y1s, st, maskd, cip, *gr,
                                              recompute)
            finally:
                ops.set_f32_split(prev)
        outs[name] = (dy, gr)
    torch.cuda.synchronize()
    r = ref.to(device)
    (mx, rms), (mx0, rms0) = _errs(outs["h2"][0], r), _errs(outs["fp32"][0], r)
    assert rms <= 1.5 * rms0 + 1e-12 and mx <= 2.0 * mx0 + 1e-12, (mx, rms, mx0, rms0)
    dgamma_ref = (dz * xhat).sum(0)
    dbeta_ref = dz.sum(0)
    for k, rr in ((0, dgamma_ref), (1, dbeta_ref)):
        a, b0 = outs["h2"][1][k].double(), outs["fp32"][1][k].double()
        rr = rr.to(device)
        e, e0 = (a - rr).norm().item(), (b0 - rr).norm().item()
        # sums over all M pixels of the BN backward's dz: within the fp32 path's
        # error or 1e-5 relative (measured up to 2.3e-6 at conv6's shape, where
        # the fp32 MFMA chain reads 4e-7: the f16 MFMA sums are not unbiased
        # over 32k pixels; the model's gradient tolerance is 2e-2 rel-L2)
        assert e <= max(1.5 * e0, 1e-5 * rr.norm().item()), (k, e, e0)
    # the recorded max|dY1| bounds what was stored (the h2 scale source of its transforms)
    assert _slot_max(aout) >= outs["h2"][0].abs().max().item()


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_bn_act_h2_bound(ops, device, p):
    """The Samuelson bound nsm_bn_finalize_train records dominates
    max|lrelu(BN(y)) * mask| (with channel scales spread 2^-12..2^0 and a few
    extreme pixels), and the h2 tensor bn_act_h2 writes decodes to the fp32
    bn_act values within the f16x2 bound."""
    g = torch.Generator().manual_seed(11 + int(p * 10))
    M, C, HW = 8192, 256, 1024
    B = M // HW
    y = torch.randn(M, C, generator=g) * _spread(g, C).float() + torch.randn(C, generator=g)
    y[17, :] *= 40.0                     # an outlier row: the bound must still hold
    gamma = torch.randn(C, generator=g) * _spread(g, C).float()
    beta = torch.randn(C, generator=g) * 0.1
    yd = y.to(device)
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    mask = None
    mmax = 1.0
    if p > 0:
        mask = ((torch.rand(B, C, generator=g) > p).float() / (1 - p)).to(device)
        mmax = 1.0 / (1 - p)
    slot = ops.amax_slots(1, device)
    st = ops.bn_train(yd, bn, C, 0.1, 1e-5, bound=(slot, mmax))
    a_h2 = ops.bn_act_h2(yd, st, 0.2, mask=mask, HW=HW, bound=slot)
    a32 = ops.bn_act(yd, st, 0.2, mask=mask, HW=HW)
    torch.cuda.synchronize()
    bound = _slot_max(slot)
    amax = a32.abs().max().item()
    assert bound >= amax, (bound, amax)
    assert bound <= amax * (M ** 0.5) * 20, (bound, amax)   # Samuelson slack only
    import math
    e = max(-126, min(126, 15 - math.ceil(math.log2(bound))))
    h = a_h2.view(M, C // 8, 2, 8).double()
    dec = (h[:, :, 0, :] + h[:, :, 1, :]).reshape(M, C) * 2.0 ** (-e)
    err = (dec - a32.double()).abs()
    # 22 significand bits relative to each element, or the absolute floor 2^-25 / s
    assert (err <= a32.double().abs() * 2.0 ** -21 + 2.0 ** (-25 - e)).all()


def test_prep_kind5_matches_to_h2(ops, device):
    """Prep kind 5 (the step's h2 packs of the 1x1 weights, FWD and DGRAD)
    bitwise equal to nsm_to_h2 of the fp32 packs with the same max|w| slot."""
    import ctypes
    from nsm_amd import prep
    from nsm_amd._lib import lib
    g = torch.Generator().manual_seed(3)
    co, ci, cop, cip = 50, 70, 64, 96
    w = (torch.randn(co, ci, 1, 1, generator=g) * 0.3).to(device)
    am = ops.amax_slots(1, device)
    jobs, outs, base = [], [], 0
    for mode in (ops.PACK_FWD, ops.PACK_DGRAD):
        j = prep.NsmPrepJob()
        j.kind = prep.KIND_PACK_H2
        for i, v in enumerate((co, ci, 1, cop, cip, mode, int(mode != ops.PACK_FWD))):
            j.a[i] = v
        j.base = base
        out = torch.empty(2 * cop * cip, dtype=ops.H2, device=device)
        j.src, j.dst, j.amax = w.data_ptr(), out.data_ptr(), am.data_ptr()
        base += int(lib.nsm_prep_items(ctypes.byref(j)))
        jobs.append(j)
        outs.append(out)
    prep.run_jobs(jobs, device)
    ref_am = ops.absmax(w.reshape(-1))
    for mode, out in zip((ops.PACK_FWD, ops.PACK_DGRAD), outs):
        pk = ops.pack_conv_weight(w, cop, cip, mode)
        rows, cols = (cop, cip) if mode == ops.PACK_FWD else (cip, cop)
        ref = ops.to_h2(pk.view(rows, cols), ref_am)
        assert torch.equal(out.view(torch.int16), ref.reshape(-1).view(torch.int16)), mode
    assert _slot_max(am) == _slot_max(ref_am)


@pytest.mark.parametrize("fused", [False, True])
def test_bn_bwd_h2_bound(ops, device, fused):
    """dY2 written as h2 by the BN backward (nsm_bn_bwd_apply_h2) with the scale
    from the bound its finalize derives (max|k1 dz| recorded by the reduction —
    nsm_bn_bwd_reduce, or the pooling backward that produces g when fused — +
    |k2| sqrt(n-1)/invstd + |k3|): the bound dominates max|dY2|, and the h2
    tensor decodes to the fp32 nsm_bn_bwd_apply values within the f16x2 bound.
    Channel scales of y, g, gamma spread 2^-12..2^0."""
    import math
    g = torch.Generator().manual_seed(7 + int(fused))
    B, H, W, C = 4, 32, 32, 128
    M = B * H * W
    y = torch.randn(M, C, generator=g) * _spread(g, C).float() + torch.randn(C, generator=g)
    gamma = torch.randn(C, generator=g) * _spread(g, C).float()
    beta = torch.randn(C, generator=g) * 0.1
    yd = y.to(device)
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    st = ops.bn_train(yd, bn, C, 0.1, 1e-5)
    if fused:
        # g = the AvgPool2d backward of a pooled gradient, BN-reduced in its producer
        dpool = (torch.randn(B * (H // 2) * (W // 2), C, generator=g) *
                 _spread(g, C).float()).to(device)
    else:
        gg = (torch.randn(M, C, generator=g) * _spread(g, C).float()).to(device)
    outs = {}
    for mode in ("fp32", "h2"):
        grads = [torch.zeros(C, device=device) for _ in range(3)]
        slots = ops.amax_slots(2, device)
        k1dz, bnd = ops.amax_slot(slots, 0), ops.amax_slot(slots, 1)
        part = None
        if fused:
            gg, part = ops.avgpool2_bwd_add(dpool, B, H, W, None,
                                            bnred=(yd, st, k1dz) if mode == "h2" else (yd, st))
            assert part is not None
        if mode == "fp32":
            outs[mode] = ops.bn_bwd(gg, yd, st, H * W, None, C, *grads, part=part)
        else:
            outs[mode] = ops.bn_bwd(gg, yd, st, H * W, None, C, *grads, part=part,
                                    h2=(k1dz, bnd))
            outs["bound"] = bnd
    torch.cuda.synchronize()
    d32 = outs["fp32"].double()
    bound = _slot_max(outs["bound"])
    amax = d32.abs().max().item()
    assert bound >= amax, (bound, amax)
    e = max(-126, min(126, 15 - math.ceil(math.log2(bound))))
    h = outs["h2"].view(M, C // 8, 2, 8).double()
    dec = (h[:, :, 0, :] + h[:, :, 1, :]).reshape(M, C) * 2.0 ** (-e)
    err = (dec - d32).abs()
    assert (err <= d32.abs() * 2.0 ** -21 + 2.0 ** (-25 - e)).all()


@pytest.mark.parametrize("B,H,W,cin_p,cout_p", [(8, 64, 64, 32, 32), (2, 33, 47, 64, 32),
                                                (4, 40, 24, 32, 64)])
def test_conv3x3_h2(ops, device, B, H, W, cin_p, cout_p):
    """The direct 3x3 (conv2's) on h2 operands: forward with BN partials, the
    input gradient (DGRAD pack), the weight gradient (cout_p 32) vs float64,
    within the fp32 MFMA path's error; X through nsm_input_prep_h2 (scale =
    max|x| its own pass records)."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(B * H + W + cin_p)
    C = cin_p // 4
    xin = torch.randn(B, C, 2 * H, 2 * W, generator=g, dtype=torch.float64) * \
        _spread(g, C, -6, 0).view(1, C, 1, 1)
    w = torch.randn(cout_p, cin_p, 3, 3, generator=g, dtype=torch.float64) / (9 * cin_p) ** 0.5
    b = torch.randn(cout_p, generator=g, dtype=torch.float64) * 0.1
    dy = torch.randn(B, cout_p, H, W, generator=g, dtype=torch.float64)
    xin, w, b, dy = (t.to(device) for t in (xin, w, b, dy))
    x = torch.nn.functional.pixel_unshuffle(xin, 2)               # [B, cin_p, H, W]
    x.requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    ref = F.conv2d(x, wr, b, padding=1)
    ref.backward(dy)
    nh = lambda t: t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).contiguous()  # noqa: E731
    am = ops.amax_slots(4, device)
    ax, aw, awd, ady = (ops.amax_slot(am, i) for i in range(4))
    xh = ops.input_prep_h2(xin.float().contiguous(), cin_p, ax)
    ws = w.float().contiguous()
    wf = ops.pack_conv_weight(ws, cout_p, cin_p, ops.PACK_FWD)
    wd = ops.pack_conv_weight(ws, cout_p, cin_p, ops.PACK_DGRAD)
    ops.absmax(wf, aw)
    ops.absmax(wd, awd)
    dys = nh(dy).float()
    ops.absmax(dys, ady)
    y, part = ops.conv3x3_h2(xh, B, H, W, ops.to_h2(wf.view(cout_p, -1), aw), b.float(), cout_p,
                             amax=(ax, aw))
    dyh = ops.to_h2(dys, ady)
    dx, _ = ops.conv3x3_h2(dyh, B, H, W, ops.to_h2(wd.view(cin_p, -1), awd), None, cin_p,
                           stats=False, amax=(ady, awd))
    outs = {"h2": (y, dx)}
    if cout_p == 32:
        dw = torch.empty(cout_p, cin_p, 3, 3, device=device)
        ops.conv3x3_wgrad_h2(dyh, xh, B, H, W, cin_p, cout_p, dw, amax=(ady, ax))
        outs["h2"] += (dw,)
    prev = ops.set_f32_split(0)
    try:
        xs = nh(x.detach()).float()
        y0 = ops.conv_fwd(xs, B, H, W, wf, b.float(), cout_p, 3)
        dx0 = ops.conv_fwd(dys, B, H, W, wd, None, cin_p, 3)
        outs["fp32"] = (y0, dx0)
        if cout_p == 32:
            dw0 = torch.empty_like(dw)
            ops.conv_wgrad(dys, xs, B, H, W, 3, cin_p, cout_p, dw0)
            outs["fp32"] += (dw0,)
    finally:
        ops.set_f32_split(prev)
    torch.cuda.synchronize()
    refs = (nh(ref.detach()), nh(x.grad), wr.grad)
    for got, base, r in zip(outs["h2"], outs["fp32"], refs):
        (mx, rms), (mx0, rms0) = _errs(got.reshape(r.shape), r), _errs(base.reshape(r.shape), r)
        assert rms <= 1.5 * rms0 + 1e-12 and mx <= 2.0 * mx0 + 1e-12, (mx, rms, mx0, rms0)
    bn = torch.nn.BatchNorm2d(cout_p).to(device)
    st = ops.bn_train(y, bn, cout_p, 0.1, 1e-5, part=part)
    yr = nh(ref.detach())
    torch.testing.assert_close(st.mean.double(), yr.mean(0), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("tile", [4, 6])
@pytest.mark.parametrize("B,H,W,C,drop", [(2, 37, 29, 64, True), (1, 16, 16, 128, False),
                                         (2, 40, 52, 32, True), (3, 13, 7, 96, False),
                                         (8, 256, 256, 64, True)])
def test_wino_dual_input_bn_h2(ops, device, B, H, W, C, drop, tile):
    """nsm_wino_dual_input_bn_h2 (the first BN's backward formed per element
    inside the h2 dual transform; F(6x6) through the LDS-region kernel): its Vd
    and dM decode to the fp32 BN-fused dual transform (nsm_wino_dual_input_bn)
    within the f16x2 bound, under the scale of the dY bound the finalize
    derives from max|k1 dz| — which dominates max|dY|. Channel scales of y, g,
    gamma spread 2^-12..2^0; ragged tile grids, multi-block regions."""
    import math
    g = torch.Generator().manual_seed(H * W + C + tile)
    y = (torch.randn(B * H * W, C, generator=g, dtype=torch.float64) * _spread(g, C) +
         torch.randn(C, generator=g, dtype=torch.float64)).float().to(device)
    gr = (torch.randn(B * H * W, C, generator=g, dtype=torch.float64) * _spread(g, C)).float().to(device)
    mask = ((torch.rand(B, C, generator=g) > 0.2).float() / 0.8).to(device) if drop else None
    bn = torch.nn.BatchNorm2d(C).to(device)
    with torch.no_grad():
        bn.weight.copy_(torch.randn(C, generator=g) * _spread(g, C).float())
        bn.bias.uniform_(-0.2, 0.2)
    st = ops.bn_train(y, bn, C, 0.1, 1e-5)
    grads = [[torch.zeros(C, device=device) for _ in range(3)] for _ in range(2)]
    d32 = ops.bn_bwd(gr, y, st, H * W, mask, C, *grads[0], defer=True)
    Vd32, dM32 = ops.wino_dual_input_bn(d32, y, st, mask, B, H, W, tile=tile)
    dy = ops.bn_bwd(gr, y, st, H * W, mask, C, *[torch.zeros(C, device=device) for _ in range(3)])
    slots = ops.amax_slots(2, device)
    k1dz, bnd = ops.amax_slot(slots, 0), ops.amax_slot(slots, 1)
    dh = ops.bn_bwd(gr, y, st, H * W, mask, C, *grads[1], defer=True, h2=(k1dz, bnd))
    Vdh, dMh = ops.wino_dual_input_bn_h2(dh, y, st, mask, B, H, W, tile, bnd)
    torch.cuda.synchronize()
    for a, b in zip(grads[0], grads[1]):
        assert torch.equal(a, b)
    bound = _slot_max(bnd)
    assert bound >= dy.abs().max().item(), (bound, dy.abs().max().item())
    for which, ref, h2t in ((0, Vd32, Vdh), (1, dM32, dMh)):
        sb = float(np.float32(bound) * np.float32(ops.wino_beta(tile, which)))
        e = max(-126, min(126, 15 - math.ceil(math.log2(sb))))
        h = h2t.view(-1, C // 8, 2, 8).double()
        dec = (h[:, :, 0, :] + h[:, :, 1, :]).reshape(-1) * 2.0 ** (-e)
        r = ref.double().reshape(-1)
        err = (dec - r).abs()
        assert (err <= r.abs() * 2.0 ** -20 + 2.0 ** (-22 - e) + 1e-6 * r.abs().max()).all(), \
            (which, err.max().item(), r.abs().max().item())


@pytest.mark.parametrize("up", [False, True])
@pytest.mark.parametrize("B,hi,wi,H,W,C", [(2, 8, 10, 16, 20, 64), (1, 16, 16, 32, 32, 128),
                                          (2, 5, 7, 10, 14, 32), (1, 34, 60, 67, 120, 64),
                                          (3, 20, 20, 40, 40, 96)])
def test_wino_input_h2(ops, device, B, hi, wi, H, W, C, up):
    """nsm_wino_input_h2 (F(6x6): the LDS-region kernel, optionally sampling
    the x2 bilinear upsample) decodes to the fp32 input transform
    (nsm_wino_input_resize) within the f16x2 bound, under the scale of
    max|x| x beta."""
    import math
    if not up:
        hi, wi = H, W
    g = torch.Generator().manual_seed(hi * wi + C + int(up))
    x = (torch.randn(B * hi * wi, C, generator=g, dtype=torch.float64) * _spread(g, C)).float().to(device)
    slots = ops.amax_slots(1, device)
    ax = ops.amax_slot(slots, 0)
    ops.absmax(x, ax)
    T = ops.wino_tiles(B, H, W, 6)
    Vh = torch.empty(64 * T * 2 * C, dtype=ops.H2, device=device)
    ops.call("nsm_wino_input_h2", ops.ptr(x), x.stride(0), B, hi, wi, H, W, C, 6, ops.ptr(Vh),
             ops.ptr(ax), ops.stream())
    V32 = torch.empty(64 * T * C, device=device)
    ops.call("nsm_wino_input_resize", ops.ptr(x), x.stride(0), B, hi, wi, H, W, C, 6, 0,
             ops.ptr(V32), None, ops.stream())
    torch.cuda.synchronize()
    sb = float(np.float32(_slot_max(ax)) * np.float32(ops.wino_beta(6, 0)))
    e = max(-126, min(126, 15 - math.ceil(math.log2(sb))))
    h = Vh.view(-1, C // 8, 2, 8).double()
    dec = (h[:, :, 0, :] + h[:, :, 1, :]).reshape(-1) * 2.0 ** (-e)
    r = V32.double()
    err = (dec - r).abs()
    assert (err <= r.abs() * 2.0 ** -20 + 2.0 ** (-22 - e) + 1e-6 * r.abs().max()).all(), \
        (err.max().item(), r.abs().max().item())
