"""GPU: the fp32 GEMMs of the Winograd layers on the bf16 matrix cores by the
exact three-way split (csrc/nsm_conv_split.inc) carry fp32 accuracy: against a
float64 convolution their error stays within that of the v_mfma_f32_32x32x2_f32
path on the same inputs (both modes through the C ABI, same seeded data)."""
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
    prev = O.set_f32_split(1)
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
    for mode in (0, 1):
        ops.set_f32_split(mode)
        U = ops.wino_weight(ws.to(device), co, ci, flip=False, tile=tile)
        y, V = ops.conv3x3_wino(nhwc(xs).to(device), B, H, W, U, None, co, tile=tile, keep_v=True)
        Ud = ops.wino_weight(ws.to(device), ci, co, flip=True, tile=tile)
        dx = ops.conv3x3_wino(nhwc(dys).to(device), B, H, W, Ud, None, ci, tile=tile)
        dw = torch.empty(co, ci, 3, 3, device=device)
        ops.conv3x3_wgrad_wino(nhwc(dys).to(device), V, B, H, W, ci, ci, co, dw, tile=tile)
        res[mode] = (_errs(nchw(y.cpu(), B, H, W), ref.detach()),
                     _errs(nchw(dx.cpu(), B, H, W), x.grad),
                     _errs(dw.cpu(), w.grad))
    ops.set_f32_split(1)
    for i, name in enumerate(("fwd", "dgrad", "wgrad")):
        (m0, r0), (m1, r1) = res[0][i], res[1][i]
        print(f"F({tile}) {name}: fp32-MFMA max {m0:.2e} rms {r0:.2e} | split max {m1:.2e} rms {r1:.2e}")
        # the Winograd transforms dominate both; the GEMM arithmetic must not add error
        assert r1 <= 1.25 * r0 + 1e-9, (name, r0, r1)
        assert m1 <= 1.5 * m0 + 1e-8, (name, m0, m1)
