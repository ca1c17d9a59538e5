"""Host time per eager train step (the Python + launch cost of issuing one
step, GPU running behind): python tools/host_probe.py [--dtype f32|bf16]
[--batch 8] [--dp]. Prints host ms per issued step and GPU ms per step."""
import argparse
import os
import socket
import sys
import time

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pcss-unet_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dp", action="store_true")
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.dp:
        import torch.distributed as dist
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
        s.close()
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import nsm_amd
    m = nsm_amd.Unet(in_ch=7, dropout_rate=0.2).to(dev).train()
    if a.dtype == "bf16":
        m.set_compute_dtype(torch.bfloat16)
    if a.dp:
        m.data_parallel()
    opt = nsm_amd.FlatAdamW(m.parameters(), lr=1e-3, max_grad_norm=1.0, sanitize=True)
    crit = nsm_amd.CustomLoss(dev, 0.9, vgg_weights=False)
    x = torch.randn(a.batch, 7, 512, 512, device=dev)
    y = torch.rand(a.batch, 1, 512, 512, device=dev)

    def step():
        loss = crit(m(x), y, x)
        loss.backward()
        if a.dp:
            nsm_amd.allreduce_grads(m.parameters())
        opt.step()
        opt.zero_grad()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    th = (time.perf_counter() - t0) / n * 1e3
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / n * 1e3
    side = nsm_amd.unet._wg_streams.get(dev)
    if side is not None:
        import ctypes
        m16 = (ctypes.c_uint32 * 16)()
        rc = nsm_amd._lib.lib.hipExtStreamGetCUMask(ctypes.c_void_p(side.cuda_stream), 16, m16)
        print("side stream CU mask", rc, [hex(w) for w in m16])
    print(f"{a.dtype} B={a.batch} dp={a.dp}: host {th:.2f} ms per issued step, wall {tg:.2f} ms per step")
    if a.profile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(5):
            step()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
