"""GPU: the fp32 GEMMs of the Winograd layers on the 16-bit matrix cores carry
fp32 accuracy — the exact three-way bf16 split (csrc/nsm_conv_split.inc, mode
1) and the f16x2 split of power-of-two scaled operands (nsm_conv_split16.inc,
mode 2, operand maxima recorded by the producers): against a float64
convolution their error stays within that of the v_mfma_f32_32x32x2_f32 path
on the same inputs (all modes through the C ABI, same seeded data)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def nhwc(x):
    B, C, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(B * H * W, C).contiguous()


def nchw(y, B, H, W):
    return y.reshape(B, H, W, -1).permute(0, 3, 1, 2).contiguous()


@pytest.fixture(scope="module")
def ops(device):
    from nsm_amd import ops as O
    prev = O.set_f32_split(2)
    yield O
    O.set_f32_split(prev)


def _errs(a, ref):
    d = (a.double() - ref).abs()
    return d.max().item(), d.pow(2).mean().sqrt().item()


@pytest.mark.parametrize("tile", [4, 6])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 9, 11, 32, 64), (1, 16, 16, 256, 128), (2, 7, 5, 64, 32),
                                        (2, 32, 32, 512, 256), (1, 40, 36, 128, 64), (2, 24, 30, 64, 128)])
def test_split_matches_fp32_accuracy(ops, device, B, H, W, ci, co, tile):
    g = torch.Generator().manual_seed(ci * 7 + co + H + tile)
    x = torch.randn(B, ci, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) / (ci * 9) ** 0.5
    dy = torch.randn(B, co, H, W, generator=g, dtype=torch.float64)
    x.requires_grad_(True)
    w.requires_grad_(True)
    ref = F.conv2d(x, w, padding=1)
    ref.backward(dy)
    xs, ws, dys = x.detach().float(), w.detach().float(), dy.float()
    res = {}
    for mode in (0, 1, 2):
        ops.set_f32_split(mode)
        # mode 2: the operands' maxima as the model path records them (the
        # transforms fill V / Vd / dM slots, the weights' from nsm_absmax)
        am = ops.amax_slots(3, device) if mode == 2 else None
        sl = (lambda i: ops.amax_slot(am, i)) if mode == 2 else (lambda i: None)
        U = ops.wino_weight(ws.to(device), co, ci, flip=False, tile=tile)
        y, V = ops.conv3x3_wino(nhwc(xs).to(device), B, H, W, U, None, co, tile=tile, keep_v=True,
                                amax_v=sl(0), amax_u=ops.absmax(U) if mode == 2 else None)
        Ud = ops.wino_weight(ws.to(device), ci, co, flip=True, tile=tile)
        dyd = nhwc(dys).to(device)
        Vd, dM = ops.wino_dual_input(dyd, B, H, W, tile=tile, amax=(sl(1), sl(2)))
        dx = ops.conv3x3_wino(dyd, B, H, W, Ud, None, ci, tile=tile, v_in=Vd, amax_v=sl(1),
                              amax_u=ops.absmax(Ud) if mode == 2 else None)
        dw = torch.empty(co, ci, 3, 3, device=device)
        ops.conv3x3_wgrad_wino(dyd, V, B, H, W, ci, ci, co, dw, tile=tile, dM=dM,
                               amax=(sl(2), sl(0)))
        res[mode] = (_errs(nchw(y.cpu(), B, H, W), ref.detach()),
                     _errs(nchw(dx.cpu(), B, H, W), x.grad),
                     _errs(dw.cpu(), w.grad))
    ops.set_f32_split(2)
    for i, name in enumerate(("fwd", "dgrad", "wgrad")):
        (m0, r0), (m1, r1), (m2, r2) = res[0][i], res[1][i], res[2][i]
        print(f"F({tile}) {name}: fp32-MFMA max {m0:.2e} rms {r0:.2e} | bf16 split max {m1:.2e} "
              f"rms {r1:.2e} | f16x2 max {m2:.2e} rms {r2:.2e}")
        # the Winograd transforms dominate all; the GEMM arithmetic must not add
        # error: rms within 1.25x of the fp32 MFMA's (1.5x for the f16x2
        # split: its 2^-22 per-product representation error shows once the
        # GEMM's K is a few tiles — K = 4 in the 7x5 case — where the fp32
        # path adds almost no rounding; at the model's K it is below the fp32
        # MFMA's, tools/bench_split16.py); the max (a statistic of a few
        # elements at these sizes) within 2x
        for m, r, rb in ((m1, r1, 1.25), (m2, r2, 1.5)):
            assert r <= rb * r0 + 1e-9, (name, r0, r)
            assert m <= 2.0 * m0 + 1e-8, (name, m0, m)


@pytest.mark.parametrize("B,H,W,ci,co,k", [(2, 16, 16, 32, 64, 3), (2, 24, 20, 64, 128, 1),
                                           (1, 33, 35, 128, 128, 3), (2, 64, 64, 32, 32, 3)])
def test_split_direct_convs(ops, device, B, H, W, ci, co, k):
    """Direct implicit-GEMM forward, input gradient and split-K weight gradient
    (the non-Winograd fp32 GEMMs) in all three modes against float64 (mode 2
    with the operands' maxima from nsm_absmax)."""
    g = torch.Generator().manual_seed(B * 100 + ci + co + k)
    x = torch.randn(B, ci, H, W, generator=g, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(co, ci, k, k, generator=g, dtype=torch.float64) / (ci * k * k) ** 0.5).requires_grad_(True)
    dy = torch.randn(B, co, H, W, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, padding=k // 2)
    ref.backward(dy)
    xs, ws, dys = x.detach().float(), w.detach().float(), dy.float()
    res = {}
    for mode in (0, 1, 2):
        ops.set_f32_split(mode)
        am = (lambda t: ops.absmax(t)) if mode == 2 else (lambda t: None)
        xd, dyd = nhwc(xs).to(device), nhwc(dys).to(device)
        wp = ops.pack_conv_weight(ws.to(device), co, ci, ops.PACK_FWD)
        y = ops.conv_fwd(xd, B, H, W, wp, None, co, k, amax=(am(xd), am(wp)))
        wd = ops.pack_conv_weight(ws.to(device), co, ci, ops.PACK_DGRAD)
        dx = ops.conv_fwd(dyd, B, H, W, wd, None, ci, k, amax=(am(dyd), am(wd)))
        dw = torch.empty(co, ci, k, k, device=device)
        ops.conv_wgrad(dyd, xd, B, H, W, k, ci, co, dw, amax=(am(dyd), am(xd)))
        res[mode] = (_errs(nchw(y.cpu(), B, H, W), ref.detach()), _errs(nchw(dx.cpu(), B, H, W), x.grad),
                     _errs(dw.cpu(), w.grad))
    ops.set_f32_split(2)
    for i, name in enumerate(("fwd", "dgrad", "wgrad")):
        (m0, r0), (m1, r1), (m2, r2) = res[0][i], res[1][i], res[2][i]
        print(f"direct k{k} {name}: fp32-MFMA max {m0:.2e} rms {r0:.2e} | bf16 split max {m1:.2e} "
              f"rms {r1:.2e} | f16x2 max {m2:.2e} rms {r2:.2e}")
        for m, r in ((m1, r1), (m2, r2)):
            assert r <= 1.5 * r0 + 1e-9, (name, r0, r)
            assert m <= 2.0 * m0 + 1e-8, (name, m0, m)


def test_split_train_step_vs_oracle(ops, device):
    """Model level: a 1x7x256x256 train step with the split GEMMs stays as close
    to the CPU fp32 oracle as the fp32-MFMA path does (output, loss, grads)."""
    from oracle import unet_ref as O
    from oracle.weights import make_state, synthetic_batch
    from nsm_amd import CustomLoss, Unet
    np_sd = make_state(7, 42)
    x_np, y_np = synthetic_batch(1, 7, 256, 256)
    sd = O.torch_state(np_sd, requires_grad=True)
    xo = torch.from_numpy(x_np).requires_grad_(True)
    oo, _ = O.forward(sd, xo, True, None, 0.0)
    O.custom_loss(oo, torch.from_numpy(y_np), 0.9).backward()
    errs = {}
    for mode in (0, 1, 2):
        ops.set_f32_split(mode)
        m = Unet(in_ch=7, dropout_rate=0.0)
        m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in np_sd.items()})
        m = m.to(device).train()
        x = torch.from_numpy(x_np).to(device).requires_grad_(True)
        out = m(x)
        CustomLoss(device, 0.9)(out, torch.from_numpy(y_np).to(device)).backward()
        ge = max(((p.grad.cpu().double() - sd[k].grad.double()).norm() / sd[k].grad.double().norm()).item()
                 for k, p in m.named_parameters() if not k.endswith("bias"))
        errs[mode] = ((out.detach().cpu() - oo.detach()).abs().max().item(), ge)
    ops.set_f32_split(2)
    print(f"train step vs oracle: fp32-MFMA out {errs[0][0]:.2e} grad {errs[0][1]:.2e} | "
          f"bf16 split out {errs[1][0]:.2e} grad {errs[1][1]:.2e} | "
          f"f16x2 out {errs[2][0]:.2e} grad {errs[2][1]:.2e}")
    for mode in (1, 2):
        assert errs[mode][0] <= 2.0 * errs[0][0] + 1e-6
        assert errs[mode][1] <= 2.0 * errs[0][1] + 1e-6


@pytest.mark.parametrize("wino_min", [1 << 30, 256])
def test_train_step_direct_3x3_blocks_vs_oracle(ops, device, monkeypatch, wino_min):
    """fp32 training with some or all 3x3 convs on the direct implicit GEMM
    (NSM_WINOGRAD=0 / a raised NSM_WINO_MIN): only conv2, whose input the
    forward writes as h2, takes the h2 direct path; conv3.. read the fp32
    output of the block before and keep fp32 packs. Output, loss
    and weight grads of a 1x7x128x128 step vs the CPU oracle."""
    from oracle import unet_ref as O
    from oracle.weights import make_state, synthetic_batch
    from nsm_amd import CustomLoss, Unet
    from nsm_amd import unet as U
    monkeypatch.setattr(U, "WINOGRAD_MIN_CHANNELS", wino_min)
    np_sd = make_state(7, 43)
    x_np, y_np = synthetic_batch(1, 7, 128, 128)
    sd = O.torch_state(np_sd, requires_grad=True)
    oo, _ = O.forward(sd, torch.from_numpy(x_np), True, None, 0.0)
    O.custom_loss(oo, torch.from_numpy(y_np), 0.9).backward()
    m = Unet(in_ch=7, dropout_rate=0.0)
    m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in np_sd.items()})
    m = m.to(device).train()
    out = m(torch.from_numpy(x_np).to(device).requires_grad_(True))
    CustomLoss(device, 0.9)(out, torch.from_numpy(y_np).to(device)).backward()
    torch.cuda.synchronize()
    oe = (out.detach().cpu() - oo.detach()).abs().max().item()
    ge = max(((p.grad.cpu().double() - sd[k].grad.double()).norm() / sd[k].grad.double().norm()).item()
             for k, p in m.named_parameters() if not k.endswith("bias"))
    print(f"wino_min {wino_min}: out {oe:.2e} grad rel {ge:.2e}")
    assert oe <= 1e-4 and ge <= 2e-2, (oe, ge)


def _h2(ops, t, rows, C, amax, beta):
    """fp32 [rows][C] -> h2 tensor (nsm_to_h2) with scale source (amax, beta)."""
    from nsm_amd._lib import call, ptr, stream
    out = torch.empty(rows * 2 * C, dtype=ops.H2, device=t.device)
    call("nsm_to_h2", ptr(t), rows, C, ptr(amax), beta, ptr(out), stream())
    return out


@pytest.mark.parametrize("tile", [4, 6])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 9, 11, 32, 64), (1, 16, 16, 256, 128), (2, 7, 5, 64, 32),
                                        (2, 32, 32, 512, 256), (1, 40, 36, 128, 64), (2, 24, 30, 64, 128)])
def test_h2_matches_fp32_accuracy(ops, device, B, H, W, ci, co, tile):
    """The pre-split (h2) Winograd path (csrc/nsm_conv_h2.inc): the input / dual
    transforms write the two fp16 terms scaled from max|x| / max|dy| times the
    transform bound, U from max|w| times the filter bound, and the LDS-DMA f16
    GEMMs run fwd, dgrad and wgrad. Against a float64 convolution the error
    stays within that of the fp32-MFMA path (same bounds as the f16x2 split)."""
    g = torch.Generator().manual_seed(ci * 5 + co + W + tile)
    x = torch.randn(B, ci, H, W, generator=g, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) / (ci * 9) ** 0.5).requires_grad_(True)
    dy = torch.randn(B, co, H, W, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, padding=1)
    ref.backward(dy)
    xs, ws, dys = x.detach().float(), w.detach().float(), dy.float()
    xd, dyd, wd = nhwc(xs).to(device), nhwc(dys).to(device), ws.to(device)
    nb = (tile + 2) ** 2
    res = {}
    for mode in ("fp32", "h2"):
        ops.set_f32_split(0 if mode == "fp32" else 2)
        U = ops.wino_weight(wd, co, ci, flip=False, tile=tile)
        Ud = ops.wino_weight(wd, ci, co, flip=True, tile=tile)
        dw = torch.empty(co, ci, 3, 3, device=device)
        if mode == "fp32":
            y, V = ops.conv3x3_wino(xd, B, H, W, U, None, co, tile=tile, keep_v=True)
            Vd, dM = ops.wino_dual_input(dyd, B, H, W, tile=tile)
            dx = ops.conv3x3_wino(dyd, B, H, W, Ud, None, ci, tile=tile, v_in=Vd)
            ops.conv3x3_wgrad_wino(dyd, V, B, H, W, ci, ci, co, dw, tile=tile, dM=dM)
        else:
            aw, ax, ady = ops.absmax(wd), ops.absmax(xd), ops.absmax(dyd)
            bg = ops.wino_beta(tile, 2)
            Uh = _h2(ops, U, nb * co, ci, aw, bg)
            Udh = _h2(ops, Ud, nb * ci, co, aw, bg)
            y, V = ops.conv3x3_wino(xd, B, H, W, Uh, None, co, tile=tile, keep_v=True,
                                    amax_v=ax, amax_u=aw)
            assert V.dtype == ops.H2
            Vd, dM = ops.wino_dual_input_h2(dyd, B, H, W, tile, ady)
            dx = ops.conv3x3_wino(dyd, B, H, W, Udh, None, ci, tile=tile, v_in=Vd, amax_v=ady,
                                  amax_u=aw)
            ops.conv3x3_wgrad_wino(dyd, V, B, H, W, ci, ci, co, dw, tile=tile, dM=dM,
                                   amax=(ady, ax))
        res[mode] = (_errs(nchw(y.cpu(), B, H, W), ref.detach()),
                     _errs(nchw(dx.cpu(), B, H, W), x.grad), _errs(dw.cpu(), w.grad))
    ops.set_f32_split(2)
    for i, name in enumerate(("fwd", "dgrad", "wgrad")):
        (m0, r0), (m2, r2) = res["fp32"][i], res["h2"][i]
        print(f"h2 F({tile}) {name}: fp32-MFMA max {m0:.2e} rms {r0:.2e} | h2 max {m2:.2e} rms {r2:.2e}")
        assert r2 <= 1.5 * r0 + 1e-9, (name, r0, r2)
        assert m2 <= 2.0 * m0 + 1e-8, (name, m0, m2)


def test_h2_prep_matches_to_h2(ops, device):
    """The step's weight preparation (prep kind 4: max|w| pass, then U written
    pre-split) gives bitwise the h2 tensor of nsm_wino_weight's U scaled from
    max|w| x the filter bound, for the forward and the input-gradient filters."""
    from nsm_amd import Unet
    from nsm_amd.prep import StepWeights
    from nsm_amd.unet import WINOGRAD_MIN_CHANNELS, block_shapes, wino_tile
    torch.manual_seed(3)
    m = Unet(in_ch=7).to(device).train()
    sw = StepWeights(m, torch.float32, block_shapes(64, 64), True, WINOGRAD_MIN_CHANNELS,
                     wino_tile, h2=True)
    sw.run()
    for k in (3, 6, 9):
        blk = m.block(k)
        cip = ops.pad32(blk.conv[0].in_channels)
        h, w_ = block_shapes(64, 64)[k]
        tile = wino_tile(cip, h, w_)
        pb = sw.block(k)
        wt = blk.conv[0].weight.detach()
        aw = ops.absmax(wt.contiguous())
        nb = (tile + 2) ** 2
        for flip in (False, True):
            U = ops.wino_weight(wt, cip, cip, flip=flip, tile=tile)
            ref = _h2(ops, U, nb * cip, cip, aw, ops.wino_beta(tile, 2))
            got = pb.U1(tile, flip)
            assert got.dtype == ops.H2
            assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), (k, flip)
            # the slot the GEMMs read holds max|w|
            assert torch.equal(pb.amax_U1(flip).max(), aw.max()), (k, flip)


@pytest.mark.parametrize("B,H,W,ci,co", [(8, 64, 64, 1024, 1024), (8, 128, 128, 512, 512),
                                        (8, 128, 128, 512, 128)])
def test_h2_persistent_gemm_full_shapes(ops, device, B, H, W, ci, co):
    """The persistent h2 GEMM (gemm_h2p_kernel: one block per CU walking the
    tiles, the K-tile stream running across tiles, buffer-store epilogue) at the
    train step's conv6 / conv7 shapes (256x256 tiles; the last one 256x128):
    components against float64, and the rows past T (outside the epilogue's
    buffer descriptor) never written."""
    from nsm_amd._lib import call, ptr, stream
    t = 6
    T = ops.wino_tiles(B, H, W, t)
    nb = (t + 2) ** 2
    g = torch.Generator(device=device).manual_seed(ci + co)
    cs = (2.0 ** torch.linspace(-3, 3, nb, device=device)).view(nb, 1, 1)
    V = (torch.randn(nb, T, ci, device=device, generator=g) * cs).reshape(-1).contiguous()
    U = (torch.randn(nb, co, ci, device=device, generator=g) * 0.03).reshape(-1).contiguous()
    amax = ops.amax_slots(2, device)
    av, au = ops.absmax(V, ops.amax_slot(amax, 0)), ops.absmax(U, ops.amax_slot(amax, 1))
    Vh = _h2(ops, V, nb * T, ci, av, 100.0)
    Uh = _h2(ops, U, nb * co, ci, au, 1.0)
    guard = 4096
    Mb = torch.full((nb * T * co + guard,), float("nan"), device=device)
    call("nsm_wino_gemm_h2", ptr(Vh), ptr(Uh), B, H, W, ci, co, t, ptr(Mb), ptr(av), 100.0,
         ptr(au), 1.0, stream())
    torch.cuda.synchronize()
    assert torch.isnan(Mb[nb * T * co:]).all()
    for c in (0, nb // 2, nb - 1):
        v = V.view(nb, T, ci)[c].double()
        u = U.view(nb, co, ci)[c].double()
        ref = v @ u.t()
        got = Mb[:nb * T * co].view(nb, T, co)[c].double()
        assert torch.isfinite(got).all(), c
        rms = ref.pow(2).mean().sqrt()
        assert ((got - ref).pow(2).mean().sqrt() / rms).item() < 2e-6, c
        assert ((got - ref).abs().max() / rms).item() < 3e-5, c


def _scale_exp(m, beta):
    """Host mirror of h2_exp / pow2_scale_exp (nsm_conv_split16.inc)."""
    import numpy as np
    b = np.float32(m) * np.float32(beta)
    if np.isfinite(np.float32(m)) and not np.isfinite(b):
        b = np.finfo(np.float32).max
    u = int(np.array(b, dtype=np.float32).view(np.uint32))
    if u == 0 or u >= 0x7f800000:
        return 0
    e = (u >> 23) - 127
    if u & 0x7fffff:
        e += 1
    return max(-126, min(126, 15 - e))


@pytest.mark.parametrize("mx,beta", [(2.0 ** -120, 1.0), (1e36, 3969.0), (3.0e38, 225.0), (1.0, 1.0)])
def test_h2_scale_edges(ops, device, mx, beta):
    """Scale edges of the h2 writers: a maximum below 2^-111 keeps a
    normal undo factor (the data is represented, not flushed to zero), and a
    bound beta * max above FLT_MAX saturates instead of falling back to s = 1
    (which would turn values above 65504 into Inf). Decoding (h + l) / s gives
    back x within the f16x2 bound relative to the maximum."""
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(64, 32, generator=g) * 2 - 1) * mx
    x[0, 0] = mx
    xd = x.to(device)
    am = ops.absmax(xd)
    h2 = _h2(ops, xd, 64, 32, am, beta).view(64, 4, 2, 8).float().cpu()
    e = _scale_exp(mx, beta)
    dec = (h2[:, :, 0, :].double() + h2[:, :, 1, :].double()).reshape(64, 32) * 2.0 ** (-e)
    assert torch.isfinite(dec).all()
    err = (dec - x.double()).abs().max().item()
    assert err <= mx * 2.0 ** -20, (err, mx)
