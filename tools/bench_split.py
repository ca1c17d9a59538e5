"""GPU microbenchmark: Winograd F(6x6) batched GEMMs (fwd/dgrad form and the
weight-gradient form) of the fp32 train step, fp32 MFMA vs the bf16 split
(NSM_SPLIT_NST picks the split kernel's LDS stages). Prints ms per launch."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pcss-unet_amd"))
from nsm_amd import ops  # noqa: E402
from nsm_amd._lib import call, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
tile = 6
shapes = [(8, 64, 64, 1024, 512), (8, 64, 64, 512, 1024), (8, 128, 128, 512, 256),
          (8, 128, 128, 256, 512), (8, 256, 256, 256, 128), (8, 256, 256, 128, 128)]
MODES = [int(m) for m in os.environ.get("MODES", "0,1").split(",")]
ONLY = os.environ.get("ONLY", "")
if os.environ.get("SHAPES"):
    shapes = [shapes[int(i)] for i in os.environ["SHAPES"].split(",")]
for (B, H, W, ci, co) in shapes:
    T = ops.wino_tiles(B, H, W, tile)
    nb = (tile + 2) ** 2
    V = torch.randn(nb * T * ci, device=dev)
    U = torch.randn(nb * co * ci, device=dev)
    Mb = torch.empty(nb * T * co, device=dev)
    dM = torch.randn(nb * T * co, device=dev)
    dw = torch.empty(co, ci, 3, 3, device=dev)
    from nsm_amd._lib import lib
    ws = torch.empty(int(lib.nsm_wino_wgrad_ws(B, H, W, ci, co, tile)), device=dev)
    flop = 2.0 * nb * T * ci * co
    out = []
    for mode in MODES:
        ops.set_f32_split(mode)
        for name, fn in (("gemm", lambda: call("nsm_wino_gemm", ptr(V), ptr(U), B, H, W, ci, co, tile,
                                                 ptr(Mb), stream())),
                         ("wgrad", lambda: call("nsm_conv3x3_wgrad_wino_dm", ptr(dM), ptr(V), B, H, W,
                                                  ci, co, ci, co, tile, ptr(dw), ptr(ws), ws.numel(),
                                                  None, None, stream()))):
            if ONLY and name != ONLY:
                continue
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            out.append(f"{name}[{mode}] {ms:.3f} ms {flop / ms / 1e9:.0f} TF")
    print(f"B{B} {H}x{W} {ci}->{co} T={T}: " + " | ".join(out), flush=True)
