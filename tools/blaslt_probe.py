"""Library GEMM rates (torch.matmul -> hipBLASLt) for the step's GEMM shapes,
as a yardstick for the hand-written kernels: python tools/blaslt_probe.py"""
import torch


def rate(fn, flops, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    return ms, flops / ms / 1e9


dev = "cuda"
for name, (b, m, n, k), dt in [
        ("wino F4 conv6/7 fwd", (36, 16384, 1024, 1024), torch.float16),
        ("wino F4 conv7 (128^2)", (36, 65536, 512, 512), torch.float16),
        ("conv8 im2col 3x3 C128", (1, 4194304, 128, 1152), torch.bfloat16),
        ("conv9 im2col 3x3 C64 (512^2)", (1, 16777216, 64, 576), torch.bfloat16),
        ("square 8192", (1, 8192, 8192, 8192), torch.bfloat16)]:
    A = torch.randn(b, m, k, device=dev, dtype=dt)
    B = torch.randn(b, k, n, device=dev, dtype=dt)
    ms, tf = rate(lambda: torch.matmul(A, B), 2.0 * b * m * n * k)
    print(f"{name:32s} {b}x{m}x{n}x{k} {str(dt):15s} {ms * 1e3:8.1f} us {tf:7.1f} TFLOP/s")
    del A, B
    torch.cuda.empty_cache()
