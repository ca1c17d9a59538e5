"""Probe: the B=8 fp32 train step eager vs replayed from one HIP graph.

    python tools/graph_step_probe.py [--dtype f32|bf16] [--batch 8] [--steps 30]

Captures forward + loss + backward + FlatAdamW tail of one step with
torch.cuda.graph (dropout seed and range check frozen / off: a timing probe,
not the product path) and times replays against eager steps, HIP events
around each loop."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pcss-unet_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import nsm_amd
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, C, H = a.batch, 7, 512
    m = nsm_amd.Unet(in_ch=C, dropout_rate=0.2).to(dev).train()
    if a.dtype == "bf16":
        m.set_compute_dtype(torch.bfloat16)
    opt = nsm_amd.FlatAdamW(m.parameters(), lr=7e-4, weight_decay=1e-3, max_grad_norm=1.0,
                            sanitize=True)
    crit = nsm_amd.CustomLoss(dev, alpha=0.9, vgg_weights=False, check_range=False)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    y = torch.randint(0, 256, (B, 1, H, H), device=dev, generator=g).float() / 255.0

    def step():
        loss = crit(m(x), y, x)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    def timed(fn, n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    eager = timed(step, a.steps)
    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=True)
    t0 = time.time()
    with torch.cuda.graph(graph):
        step()
    print(f"capture {time.time() - t0:.2f} s", flush=True)
    for _ in range(3):
        graph.replay()
    replay = timed(graph.replay, a.steps)
    eager2 = timed(step, a.steps)
    print(f"{a.dtype} B={B}: eager {eager:.3f} / {eager2:.3f} ms/step, graph replay {replay:.3f} "
          f"ms/step ({B / replay * 1e3:.1f} vs {B / min(eager, eager2) * 1e3:.1f} frames/s)",
          flush=True)


if __name__ == "__main__":
    main()
