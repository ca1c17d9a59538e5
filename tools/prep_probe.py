"""Weight-preparation launch alone vs plain HBM write/copy streams of the same
size: python tools/prep_probe.py. Prints each job's bytes and the timings."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pcss-unet_amd")]
import nsm_amd  # noqa: E402


def timeit(fn, n=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    dev = torch.device("cuda", 0)
    m = nsm_amd.Unet(in_ch=7, dropout_rate=0.2).to(dev).train()
    x = torch.randn(8, 7, 512, 512, device=dev)
    m(x).sum().backward()
    torch.cuda.synchronize()
    sws = list(m.__dict__["_step_weights"].values())
    sw = sws[0]
    nbytes = sum(t.numel() * t.element_size() for t in sw.keep)
    wbytes = sum(p.numel() * 4 for p in m.parameters())
    amax = torch.zeros(4096, dtype=torch.int32, device=dev)
    t_prep = timeit(lambda: sw.run(amax))
    print(f"prep: {len(sw.keep)} outputs, {nbytes / 1e9:.3f} GB written, {wbytes / 1e6:.1f} MB weights, "
          f"{t_prep:.1f} us -> {nbytes / t_prep / 1e3:.2f} TB/s")
    big = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    t_fill = timeit(lambda: big.fill_(1.0))
    print(f"fill_ same bytes: {t_fill:.1f} us -> {nbytes / t_fill / 1e3:.2f} TB/s")
    src = torch.empty_like(big)
    t_copy = timeit(lambda: big.copy_(src))
    print(f"copy_ same bytes: {t_copy:.1f} us -> {2 * nbytes / t_copy / 1e3:.2f} TB/s (r+w)")
    for t in sorted(sw.keep, key=lambda t: -t.numel())[:8]:
        print(f"  {tuple(t.shape)} {t.dtype} {t.numel() * t.element_size() / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
