"""GPU microbenchmark: the fp32 Winograd GEMM (split kernel) with operands split
on the fly vs pre-split in global memory (NSM_SPLIT_PRE: 1 = U, 2 = V, 3 = both;
read once per process). Checks the pre-split result against the on-the-fly one
(same planes, same products: bitwise) and prints ms per launch."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pcss-unet_amd"))
from nsm_amd import ops  # noqa: E402
from nsm_amd._lib import call, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
tile = 6
shapes = [(8, 64, 64, 1024, 1024), (8, 128, 128, 512, 512), (8, 256, 256, 128, 128)]
pre = int(os.environ.get("NSM_SPLIT_PRE", "0"))


def presplit(x, nb):  # [nb][R][K] fp32 -> [nb][3][R][K] bf16 (as a float buffer)
    x = x.view(nb, -1)
    h = x.bfloat16()
    r = x - h.float()
    m = r.bfloat16()
    l = (r - m.float()).bfloat16()
    return torch.stack([h, m, l], 1).contiguous().view(torch.float32)


torch.manual_seed(0)
for (B, H, W, ci, co) in shapes:
    T = ops.wino_tiles(B, H, W, tile)
    nb = (tile + 2) ** 2
    V = torch.randn(nb * T * ci, device=dev)
    U = torch.randn(nb * co * ci, device=dev)
    Vs, Us = presplit(V, nb), presplit(U, nb)
    Mb = torch.empty(nb * T * co, device=dev)
    flop = 2.0 * nb * T * ci * co
    ops.set_f32_split(1)
    a, b = (Vs, Us) if pre == 3 else (V, Us) if pre == 1 else (Vs, U) if pre == 2 else (V, U)
    fn = lambda: call("nsm_wino_gemm", ptr(a), ptr(b), B, H, W, ci, co, tile, ptr(Mb), stream())  # noqa
    fn()
    torch.cuda.synchronize()
    got = Mb.clone()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ref = torch.bmm(V.view(nb, T, ci).double(), U.view(nb, co, ci).double().transpose(1, 2))
    err = ((got.view(nb, T, co).double() - ref).abs().max() / ref.abs().max()).item()
    print(f"pre={pre} B{B} {H}x{W} {ci}->{co} T={T}: {ms:.3f} ms {flop / ms / 1e9:.0f} TF "
          f"maxrel {err:.2e} sum {got.double().sum().item():.6e}", flush=True)
