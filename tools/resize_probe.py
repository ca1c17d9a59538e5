"""Decoder x2 resize-backward timings (the step's shapes) for the current
NSM_RESIZE_STREAM / NSM_RESIZE_SEP setting: python tools/resize_probe.py"""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pcss-unet_amd")]
from nsm_amd import ops  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


dev = torch.device("cuda", 0)
for dt, B in ((torch.bfloat16, 64), (torch.float32, 8)):
    for h, C in ((128, 128), (64, 512), (32, 1024)):
        dy = torch.randn(B * 4 * h * h, C, device=dev).to(dt)
        us = timeit(lambda: ops.resize_bwd(dy, B, h, h, 2 * h, 2 * h))
        nbytes = dy.numel() * dy.element_size() * 1.25
        print(f"{str(dt):15s} B={B:3d} lo={h:4d} C={C:5d} {us:8.1f} us {nbytes / us / 1e3:6.2f} TB/s")
