"""GPU microbenchmark of the F(6x6) dual transform of the fp32 decoder's
output gradients, plain and BN-fused (nsm_wino_dual_input_bn), beside the
separate BN backward it replaces. HIP events, median of 10."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pcss-unet_amd"))
from nsm_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


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


B = 8
for (H, C) in ((64, 1024), (128, 512), (256, 128), (256, 64)):
    M = B * H * H
    y = torch.randn(M, C, device=dev)
    g = torch.randn(M, C, device=dev)
    bn = torch.nn.BatchNorm2d(C).to(dev)
    st = ops.bn_train(y, bn, C, 0.1, 1e-5)
    mask = torch.ones(B, C, device=dev)
    dg, db, dbias = (torch.empty(C, device=dev) for _ in range(3))
    d = ops.bn_bwd(g, y, st, H * H, mask, C, dg, db, dbias, defer=True)
    t0 = timeit(lambda: ops.wino_dual_input(g, B, H, H, tile=6))
    t1 = timeit(lambda: ops.wino_dual_input_bn(d, y, st, mask, B, H, H, tile=6))
    t2 = timeit(lambda: ops.bn_bwd(g, y, st, H * H, mask, C, dg, db, dbias))
    print(f"{H}x{H} C={C}: dual {t0*1e3:6.1f} us  dual_bn {t1*1e3:6.1f} us  bn_bwd(reduce+apply) {t2*1e3:6.1f} us",
          flush=True)
