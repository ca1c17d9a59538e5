#!/usr/bin/env python3
"""Time weight preparation and resampling kernels at the B=8 fp32 train-step
shapes in one process (HIP events, median of 10): python tools/elem_bench_f32.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pcss-unet_amd"))
import torch  # noqa: E402

from nsm_amd import ops  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


dev = torch.device("cuda:0")
for (ci, tile) in ((1024, 6), (512, 6), (512, 4)):
    w = torch.randn(ci, ci, 3, 3, device=dev)
    nb = (tile + 2) ** 2 * ci * ci * 4
    for flip in (False, True):
        t = timeit(lambda: ops.wino_weight(w, ci, ci, flip=flip, tile=tile))
        print(f"wino_weight ci={ci} F({tile}) flip={flip}: {t*1e3:7.1f} us {nb/t/1e6:7.0f} GB/s", flush=True)
B = 8
for (C, h, w) in ((128, 128, 128), (512, 64, 64), (1024, 32, 32)):
    x = torch.randn(B * h * w, C, device=dev)
    y = ops.resize(x, B, h, w, 2 * h, 2 * w)
    by = (x.numel() + y.numel()) * 4
    t = timeit(lambda: ops.resize(x, B, h, w, 2 * h, 2 * w))
    print(f"resize_fwd C={C} {h}->{2*h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s", flush=True)
    t = timeit(lambda: ops.resize_bwd(y, B, h, w, 2 * h, 2 * w))
    print(f"resize_bwd C={C} {h}<-{2*h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s", flush=True)
    t = timeit(lambda: y.clone())
    print(f"clone of the output: {t*1e3:7.1f} us {2*y.numel()*4/t/1e6:7.0f} GB/s", flush=True)
C, h = 64, 256
x = torch.randn(B * h * h, C, device=dev)
by = 2 * x.numel() * 4
t = timeit(lambda: ops.up2_resize(x, B, h, h, h, h))
print(f"up2_resize_fwd C={C} {h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s")
t = timeit(lambda: ops.up2_resize_bwd(x, B, h, h, h, h))
print(f"up2_resize_bwd C={C} {h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s")
t = timeit(lambda: x.clone())
print(f"clone: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s")

# the resize backward with the next BN's backward reduction fused (bnred=)
for (C, h, w) in ((128, 128, 128), (512, 64, 64), (1024, 32, 32)):
    y2 = torch.randn(B * h * w, C, device=dev)
    bn = torch.nn.BatchNorm2d(C).to(dev)
    st = ops.bn_train(y2, bn, C, 0.1, 1e-5)
    dyy = torch.randn(B * 4 * h * w, C, device=dev)
    t = timeit(lambda: ops.resize_bwd(dyy, B, h, w, 2 * h, 2 * w, bnred=(y2, st)))
    by = (dyy.numel() + 2 * y2.numel()) * 4
    print(f"resize_bwd+bnred C={C} {h}<-{2*h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s", flush=True)
