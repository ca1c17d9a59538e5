"""GPU microbenchmark + accuracy check: the Winograd F(6x6) batched GEMM of
the fp32 train step on the bf16 three-way split (nsm_wino_gemm) against the
f16x2 split (nsm_wino_gemm_s with the operands' maxima from nsm_absmax).
Accuracy: two components against a float64 GEMM, error over the output rms,
also for the fp32 MFMA (NSM_F32_SPLIT=0 path via ops.set_f32_split(0))."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pcss-unet_amd"))
from nsm_amd import ops  # noqa: E402
from nsm_amd._lib import call, ptr, stream  # noqa: E402

dev = torch.device("cuda:0")
tile = 6
shapes = [(8, 64, 64, 1024, 1024), (8, 128, 128, 512, 512), (8, 256, 256, 128, 128),
          (8, 256, 256, 64, 64), (8, 32, 32, 512, 512)]
if os.environ.get("SHAPES"):
    shapes = [shapes[int(i)] for i in os.environ["SHAPES"].split(",")]
REPS = int(os.environ.get("REPS", "20"))


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
    t = tile if H > 32 else 4
    T = ops.wino_tiles(B, H, W, t)
    nb = (t + 2) ** 2
    g = torch.Generator(device=dev).manual_seed(ci + co)
    # component-dependent magnitudes, as a Winograd transform gives
    cs = (2.0 ** torch.linspace(-3, 3, nb, device=dev)).view(nb, 1, 1)
    V = (torch.randn(nb, T, ci, device=dev, generator=g) * cs).reshape(-1).contiguous()
    U = (torch.randn(nb, co, ci, device=dev, generator=g) * 0.03).reshape(-1).contiguous()
    Mb = torch.empty(nb * T * co, device=dev)
    amax = ops.amax_slots(2, dev)
    av, au = ops.absmax(V, ops.amax_slot(amax, 0)), ops.absmax(U, ops.amax_slot(amax, 1))
    flop = 2.0 * nb * T * ci * co
    res, acc = [], []
    for name, mode, fn in (
            ("f32mfma", 0, lambda: call("nsm_wino_gemm", ptr(V), ptr(U), B, H, W, ci, co, t,
                                        ptr(Mb), stream())),
            ("bf16x3", 1, lambda: call("nsm_wino_gemm", ptr(V), ptr(U), B, H, W, ci, co, t,
                                       ptr(Mb), stream())),
            ("f16x2", 2, lambda: call("nsm_wino_gemm_s", ptr(V), ptr(U), B, H, W, ci, co, t,
                                      ptr(Mb), ptr(av), ptr(au), stream()))):
        ops.set_f32_split(mode)
        ms = timeit(fn)
        res.append(f"{name} {ms:.3f} ms {6 if name == 'bf16x3' else 3 if name == 'f16x2' else 1}x"
                   f"{flop / ms / 1e9:.0f} TF")
        errs = []
        for c in (0, nb - 1):
            v = V.view(nb, T, ci)[c].double()
            u = U.view(nb, co, ci)[c].double()
            ref = v @ u.t()
            got = Mb.view(nb, T, co)[c].double()
            rms = ref.pow(2).mean().sqrt()
            errs.append(((got - ref).pow(2).mean().sqrt() / rms).item())
            errs.append(((got - ref).abs().max() / rms).item())
        acc.append(f"{name} err rms/max c0 {errs[0]:.2e}/{errs[1]:.2e} c{nb - 1} {errs[2]:.2e}/{errs[3]:.2e}")
    ops.set_f32_split(1)
    print(f"B{B} {H}x{W} {ci}->{co} T={T} F({t}): " + " | ".join(res), flush=True)
    print("    " + " | ".join(acc), flush=True)
