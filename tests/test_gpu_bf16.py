"""GPU: the bf16 path (BASELINE config 3) kernel by kernel. References are the
fp32 PyTorch-CPU ops applied to the SAME bf16-rounded inputs and weights (the
products of two bf16 numbers are exact in fp32, so the GEMM references differ
from the kernels only by fp32 summation order and the final bf16 rounding of
the output), then rounded to bf16 where the kernel stores bf16."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_ops import nchw, nhwc, rel

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def r(x):  # round to bf16 and back
    return x.to(BF).float()


@pytest.fixture(scope="module")
def ops(device):
    from nsm_amd import ops as O
    return O


def bf_close(got, ref, ulps=2.0):
    """|got - ref| <= ulps * 2^-8 * max|ref|, element-wise bound from bf16 output rounding."""
    tol = ulps * 2.0 ** -8 * max(ref.abs().max().item(), 1e-30)
    err = (got.float() - ref).abs().max().item()
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("B,H,W,ci,co,k", [(2, 9, 11, 32, 64, 3), (1, 16, 16, 64, 32, 3),
                                           (2, 8, 8, 128, 128, 3), (3, 7, 5, 32, 128, 1),
                                           (2, 32, 32, 64, 512, 1), (1, 5, 67, 96, 32, 3),
                                           (4, 32, 32, 256, 256, 3),
                                           # >= 1024 blocks of 256 rows: the LDS-DMA kernel
                                           (4, 128, 128, 64, 512, 3), (3, 97, 93, 64, 1280, 3),
                                           (1, 128, 256, 128, 1024, 3),
                                           # 256x64 LDS-DMA tiles (64-channel layers), 3x3 and 1x1
                                           (4, 256, 256, 64, 64, 3), (4, 256, 255, 128, 64, 1),
                                           # N = 128: 512x128 LDS-DMA tiles, two 256-row
                                           # BN partials per block (last block ragged)
                                           (4, 256, 256, 64, 128, 3), (4, 257, 255, 128, 128, 3),
                                           (4, 256, 256, 512, 128, 1),
                                           # 32-channel 3x3 on the 128x32 LDS-DMA tiles (BK 32),
                                           # ragged last block
                                           (2, 256, 256, 32, 32, 3), (3, 131, 167, 32, 32, 3)])
def test_conv_fwd_bf16(ops, device, B, H, W, ci, co, k):
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + ci + co + k)
    x = r(torch.randn(B, ci, H, W, generator=g))
    w = r(torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5)
    b = torch.randn(co, generator=g)
    ref = F.conv2d(x, w, b, padding=k // 2)
    wp = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_FWD, BF)
    y, part = ops.conv_fwd_bn(nhwc(x).to(device, BF), B, H, W, wp, b.to(device), co, k)
    assert y.dtype == BF
    bf_close(nchw(y.cpu(), B, H, W), ref)
    # fused BN partials are taken on the rounded outputs
    yr = y.float().cpu()
    rpc, n = part.rpc, part.nchunk
    pb = part.buf.view(n, 2, co).cpu().double()
    torch.testing.assert_close(pb[:, 0].sum(0), yr.double().sum(0), rtol=1e-4, atol=1e-3)
    # every partial row: sum and centred sum of squares of its own rpc rows
    M = yr.shape[0]
    assert n == (M + rpc - 1) // rpc
    yd = torch.nn.functional.pad(yr.double(), (0, 0, 0, n * rpc - M)).view(n, rpc, co)
    cnt = torch.clamp(M - torch.arange(n) * rpc, max=rpc).double()[:, None]
    s1 = yd.sum(1)
    mu = s1 / cnt
    valid = (torch.arange(rpc)[None, :] < cnt)[:, :, None]
    m2 = (((yd - mu[:, None, :]) ** 2) * valid).sum(1)
    torch.testing.assert_close(pb[:, 0], s1, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(pb[:, 1], m2, rtol=1e-3, atol=1e-2)


# conv3x3_halo_kernel (csrc/nsm_conv_s16_dma.inc): W in {64, 128, 256}, 64 / 128
# output channels, >= 256 tiles of 512 pixels; (96 / 32 input channels: 3 and 1
# channel chunks; the dgrads of those two have 96 / 32 outputs and take the
# im2col GEMMs)
HALO_SHAPES = [(2, 256, 256, 128, 128), (8, 128, 128, 64, 128), (64, 64, 64, 128, 64),
               (2, 256, 256, 96, 64), (2, 256, 256, 32, 64)]


@pytest.mark.parametrize("B,H,W,ci,co", HALO_SHAPES)
@pytest.mark.parametrize("fmt", ["bf16", "f16"])
def test_conv3x3_halo_fwd_and_dgrad(ops, device, B, H, W, ci, co, fmt, monkeypatch):
    """The halo-tiled direct 3x3 (opt-in: NSM_BF16_HALO, read at each dispatch)
    in both 16-bit formats: the forward (with its 256-row BN partials) and the
    input gradient, against fp32 convolutions of the same rounded operands
    (only the fp32 summation order and the output rounding differ)."""
    monkeypatch.setenv("NSM_BF16_HALO", "1")
    f16 = fmt == "f16"
    sdt = ops.F16S if f16 else BF
    rnd = (lambda t: t.half().float()) if f16 else r
    store = (lambda t: t.to(device).half().view(torch.int16)) if f16 else (lambda t: t.to(device, BF))
    load = (lambda t: t.view(torch.float16).float()) if f16 else (lambda t: t.float())
    eps = 2.0 ** -11 if f16 else 2.0 ** -8
    g = torch.Generator().manual_seed(B * 7 + H + ci + co)
    x = rnd(torch.randn(B, ci, H, W, generator=g))
    w = rnd(torch.randn(co, ci, 3, 3, generator=g) / (ci * 9) ** 0.5)
    b = torch.randn(co, generator=g)
    torch.set_num_threads(16)
    wp = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_FWD, sdt)
    y, part = ops.conv_fwd_bn(store(nhwc(x)), B, H, W, wp, b.to(device), co, 3)
    assert y.dtype == sdt
    ref = F.conv2d(x, w, b, padding=1)
    got = nchw(load(y).cpu(), B, H, W)
    tol = 2.0 * eps * ref.abs().max().item()
    assert (got - ref).abs().max().item() <= tol
    yr = load(y).cpu().double()
    pb = part.buf.view(part.nchunk, 2, co).cpu().double()
    assert part.nchunk * part.rpc == B * H * W
    yd = yr.view(part.nchunk, part.rpc, co)
    torch.testing.assert_close(pb[:, 0], yd.sum(1), rtol=1e-4, atol=1e-2)
    m2 = ((yd - yd.mean(1, keepdim=True)) ** 2).sum(1)
    torch.testing.assert_close(pb[:, 1], m2, rtol=1e-3, atol=1e-2)
    # input gradient: the 3x3 of dy with the flipped, transposed weights
    dy = rnd(torch.randn(B, co, H, W, generator=g))
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, padding=1).backward(dy)
    wd = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_DGRAD, sdt)
    dx = ops.conv_fwd(store(nhwc(dy)), B, H, W, wd, None, ci, 3)
    got = nchw(load(dx).cpu(), B, H, W)
    assert (got - xr.grad).abs().max().item() <= 2.0 * eps * xr.grad.abs().max().item()


@pytest.mark.parametrize("B,H,W,ci,co", [(2, 6, 7, 32, 64), (2, 16, 16, 128, 64)])
def test_conv1x1_prologue_bf16(ops, device, B, H, W, ci, co):
    g = torch.Generator().manual_seed(7)
    y1 = r(torch.randn(B, ci, H, W, generator=g))
    sc, sh = torch.rand(ci, generator=g) + 0.5, torch.randn(ci, generator=g)
    mask = (torch.rand(B, ci, generator=g) > 0.2).float() / 0.8
    w = r(torch.randn(co, ci, 1, 1, generator=g) / ci ** 0.5)
    a = r(F.leaky_relu(y1 * sc[None, :, None, None] + sh[None, :, None, None], 0.2)
          * mask[:, :, None, None])      # the loader rounds the activated operand to bf16
    ref = F.conv2d(a, w)
    wp = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_FWD, BF)
    y = ops.conv_fwd(nhwc(y1).to(device, BF), B, H, W, wp, None, co, 1,
                     pro=(sc.to(device), sh.to(device), mask.to(device)))
    bf_close(nchw(y.cpu(), B, H, W), ref, ulps=3.0)


@pytest.mark.parametrize("B,H,W,ci,co,k", [(2, 9, 11, 32, 64, 3), (2, 8, 8, 64, 64, 3),
                                           (2, 12, 12, 64, 128, 1),
                                           (4, 128, 128, 512, 64, 3), (2, 150, 147, 768, 64, 3),
                                           # 512x128 tiles (dx has 128 channels)
                                           (4, 256, 256, 128, 64, 3),
                                           # dx of a 32 -> 32 3x3: 128x32 LDS-DMA tiles
                                           (2, 256, 256, 32, 32, 3)])
def test_conv_dgrad_bf16(ops, device, B, H, W, ci, co, k):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, ci, H, W, generator=g, requires_grad=True)
    w = r(torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5)
    dy = r(torch.randn(B, co, H, W, generator=g))
    F.conv2d(x, w, padding=k // 2).backward(dy)
    wd = ops.pack_conv_weight(w.to(device), co, ci, ops.PACK_DGRAD, BF)
    dx = ops.conv_fwd(nhwc(dy).to(device, BF), B, H, W, wd, None, ci, k)
    bf_close(nchw(dx.cpu(), B, H, W), x.grad)


@pytest.mark.parametrize("B,H,W,ci,co,k,pro", [(2, 9, 11, 32, 64, 3, False),
                                               (2, 16, 16, 64, 32, 3, False),
                                               (1, 33, 35, 128, 128, 3, False),
                                               (2, 8, 8, 32, 64, 1, True),
                                               (2, 16, 16, 128, 512, 1, True),
                                               (4, 64, 64, 32, 32, 3, False),
                                               # LDS-DMA tiles 64x64 / 128x128 / 256x128,
                                               # split-K with pixel tails
                                               (4, 64, 64, 64, 64, 3, False),
                                               (2, 12, 10, 128, 512, 3, False),
                                               (2, 16, 16, 256, 256, 3, False),
                                               (3, 45, 43, 128, 128, 3, False),
                                               # multi-tap N tiles (Cin 64: 4 taps, 128: 3 taps,
                                               # 32: 4 taps on 32x128 tiles)
                                               (2, 37, 41, 64, 64, 3, False),
                                               (3, 37, 41, 32, 32, 3, False),
                                               (2, 256, 256, 32, 32, 3, False),
                                               # prologue-free 1x1 on the DMA tiles
                                               (2, 16, 16, 128, 256, 1, False),
                                               (2, 20, 20, 512, 1024, 1, False)])
def test_conv_wgrad_bf16(ops, device, B, H, W, ci, co, k, pro):
    g = torch.Generator().manual_seed(13)
    x = r(torch.randn(B, ci, H, W, generator=g))
    sc, sh = torch.rand(ci, generator=g) + 0.5, torch.randn(ci, generator=g)
    mask = (torch.rand(B, ci, generator=g) > 0.2).float() / 0.8
    a = (r(F.leaky_relu(x * sc[None, :, None, None] + sh[None, :, None, None], 0.2)
           * mask[:, :, None, None]) if pro else x)
    w = torch.zeros(co, ci, k, k, requires_grad=True)
    dy = r(torch.randn(B, co, H, W, generator=g))
    F.conv2d(a, w, padding=k // 2).backward(dy)
    dw = torch.empty(co, ci, k, k, device=device)
    ops.conv_wgrad(nhwc(dy).to(device, BF), nhwc(x).to(device, BF), B, H, W, k, ci, co, dw,
                   pro=(sc.to(device), sh.to(device), mask.to(device)) if pro else None)
    assert rel(dw.cpu(), w.grad) <= 2e-5


def test_elementwise_bf16(ops, device):
    """bn_act (+skip), avgpool, resize fwd/bwd, up2_resize, bn_bwd on bf16
    tensors = the fp32 kernels on the upcast tensors, rounded to bf16."""
    g = torch.Generator().manual_seed(5)
    B, H, W, C = 2, 10, 14, 64
    y = r(torch.randn(B * H * W, C, generator=g)).to(device)
    res = r(torch.randn(B * H * W, C, generator=g)).to(device)
    st = ops.BNState(C, device)
    st.scale.copy_(torch.rand(C, generator=g) + 0.5)
    st.shift.copy_(torch.randn(C, generator=g))
    st.mean.copy_(torch.randn(C, generator=g))
    st.invstd.copy_(torch.rand(C, generator=g) + 0.5)
    st.gamma = (torch.rand(C, generator=g) + 0.5).to(device)
    yb, rb = y.to(BF), res.to(BF)

    def ulp1(a, b):
        # same fp32 arithmetic, but the compiler may contract the weighted sums
        # differently per instantiation: allow one bf16 rounding step
        a, b = a.float(), b.to(BF).float()
        assert ((a - b).abs() <= 2.0 ** -7 * b.abs() + 1e-6 * b.abs().max()).all()

    torch.testing.assert_close(ops.bn_act(yb, st, res=rb).float(),
                               ops.bn_act(y, st, res=res).to(BF).float(), rtol=0, atol=0)
    torch.testing.assert_close(ops.avgpool2(yb, B, H, W).float(),
                               ops.avgpool2(y, B, H, W).to(BF).float(), rtol=0, atol=0)
    ulp1(ops.resize(yb, B, H, W, 2 * H, 2 * W), ops.resize(y, B, H, W, 2 * H, 2 * W))
    ulp1(ops.up2_resize(yb, B, H, W, 2 * H - 3, 2 * W - 1),
         ops.up2_resize(y, B, H, W, 2 * H - 3, 2 * W - 1))
    dy = r(torch.randn(B * 2 * H * 2 * W, C, generator=g)).to(device)
    ulp1(ops.resize_bwd(dy.to(BF), B, H, W, 2 * H, 2 * W), ops.resize_bwd(dy, B, H, W, 2 * H, 2 * W))
    mask = ((torch.rand(B, C, generator=g) > 0.2).float() / 0.8).to(device)
    z = [torch.zeros(C, device=device) for _ in range(6)]
    dyb = ops.bn_bwd(rb, yb, st, H * W, mask, C, z[0], z[1], z[2])
    dyf = ops.bn_bwd(res, y, st, H * W, mask, C, z[3], z[4], z[5])
    torch.testing.assert_close(dyb.float(), dyf.to(BF).float(), rtol=0, atol=0)
    torch.testing.assert_close(z[0], z[3], rtol=0, atol=0)
