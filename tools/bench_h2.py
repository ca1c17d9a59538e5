"""GPU microbenchmark + accuracy check of the pre-split (h2) Winograd GEMM
(nsm_wino_gemm_h2, csrc/nsm_conv_h2.inc) against the in-kernel f16x2 split
(nsm_wino_gemm_s) on the fp32 train step's Winograd shapes. Accuracy: two
components against a float64 GEMM, error over the output rms; the h2 operands
carry a deliberately loose bound (beta) like the producers' transform bounds.
NSM_H2_TILE forces a tile (see nsm_conv_h2.inc)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pcss-unet_amd"))
from nsm_amd import ops  # noqa: E402
from nsm_amd._lib import call, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
shapes = [(8, 64, 64, 1024, 1024), (8, 128, 128, 512, 512), (8, 256, 256, 128, 128),
          (8, 256, 256, 64, 64), (8, 32, 32, 512, 512), (8, 64, 64, 128, 128)]
if os.environ.get("SHAPES"):
    shapes = [shapes[int(i)] for i in os.environ["SHAPES"].split(",")]
REPS = int(os.environ.get("REPS", "20"))
BETA = float(os.environ.get("BETA", "100"))


def timeit(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS


for (B, H, W, ci, co) in shapes:
    t = 6 if H > 32 else 4
    T = ops.wino_tiles(B, H, W, t)
    nb = (t + 2) ** 2
    g = torch.Generator(device=dev).manual_seed(ci + co)
    cs = (2.0 ** torch.linspace(-3, 3, nb, device=dev)).view(nb, 1, 1)
    V = (torch.randn(nb, T, ci, device=dev, generator=g) * cs).reshape(-1).contiguous()
    U = (torch.randn(nb, co, ci, device=dev, generator=g) * 0.03).reshape(-1).contiguous()
    Mb = torch.empty(nb * T * co, device=dev)
    amax = ops.amax_slots(2, dev)
    av, au = ops.absmax(V, ops.amax_slot(amax, 0)), ops.absmax(U, ops.amax_slot(amax, 1))
    Vh = torch.empty(V.numel() * 2, dtype=torch.float16, device=dev)
    Uh = torch.empty(U.numel() * 2, dtype=torch.float16, device=dev)
    call("nsm_to_h2", ptr(V), nb * T, ci, ptr(av), BETA, ptr(Vh), stream())
    call("nsm_to_h2", ptr(U), nb * co, ci, ptr(au), 1.0, ptr(Uh), stream())
    flop = 2.0 * nb * T * ci * co
    res, acc = [], []
    for name, fn in (
            ("f16x2", lambda: call("nsm_wino_gemm_s", ptr(V), ptr(U), B, H, W, ci, co, t,
                                   ptr(Mb), ptr(av), ptr(au), stream())),
            ("h2", lambda: call("nsm_wino_gemm_h2", ptr(Vh), ptr(Uh), B, H, W, ci, co, t,
                                ptr(Mb), ptr(av), BETA, ptr(au), 1.0, stream()))):
        Mb.fill_(float("nan"))
        ms = timeit(fn)
        res.append(f"{name} {ms:.3f} ms {3 * flop / ms / 1e9:.0f} TF(f16)")
        errs = []
        for c in (0, nb - 1):
            v = V.view(nb, T, ci)[c].double()
            u = U.view(nb, co, ci)[c].double()
            ref = v @ u.t()
            got = Mb.view(nb, T, co)[c].double()
            rms = ref.pow(2).mean().sqrt()
            errs.append(((got - ref).pow(2).mean().sqrt() / rms).item())
            errs.append(((got - ref).abs().max() / rms).item())
        acc.append(f"{name} err rms/max c0 {errs[0]:.2e}/{errs[1]:.2e} c{nb - 1} "
                   f"{errs[2]:.2e}/{errs[3]:.2e}")
    print(f"B{B} {H}x{W} {ci}->{co} T={T} F({t}): " + " | ".join(res), flush=True)
    print("    " + " | ".join(acc), flush=True)
