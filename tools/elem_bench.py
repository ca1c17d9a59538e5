#!/usr/bin/env python3
"""Time the resampling / streaming kernels at the B=64 bf16 shapes in one process
(HIP events, median of 10): python tools/elem_bench.py"""
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
B = 64
for (C, h, w) in ((128, 128, 128), (512, 64, 64), (1024, 32, 32)):
    x = torch.randn(B * h * w, C, device=dev).to(torch.bfloat16)
    y = ops.resize(x, B, h, w, 2 * h, 2 * w)
    by = (x.numel() + y.numel()) * 2
    t = timeit(lambda: ops.resize(x, B, h, w, 2 * h, 2 * w))
    print(f"resize_fwd C={C} {h}->{2*h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s", flush=True)
    t = timeit(lambda: ops.resize_bwd(y, B, h, w, 2 * h, 2 * w))
    print(f"resize_bwd C={C} {h}<-{2*h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s", flush=True)
    t = timeit(lambda: y.clone())
    print(f"clone of the output: {t*1e3:7.1f} us {2*y.numel()*2/t/1e6:7.0f} GB/s", flush=True)
C, h = 64, 256
x = torch.randn(B * h * h, C, device=dev).to(torch.bfloat16)
by = 2 * x.numel() * 2
t = timeit(lambda: ops.up2_resize(x, B, h, h, h, h))
print(f"up2_resize_fwd C={C} {h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s")
t = timeit(lambda: ops.up2_resize_bwd(x, B, h, h, h, h))
print(f"up2_resize_bwd C={C} {h}: {t*1e3:7.1f} us {by/t/1e6:7.0f} GB/s")
