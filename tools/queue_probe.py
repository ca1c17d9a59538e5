"""Which hardware queue does a stream land on? Run under
`rocprofv3 --kernel-trace`: each stream gets a fill kernel of a distinct size
(Grid_Size tells them apart in the trace). --dp: a world-size-1 RCCL group and
one broadcast first; --early: the probe streams are touched before that."""
import os
import socket
import sys

import torch
import torch.distributed as dist

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def touch(tag, s):
    with torch.cuda.stream(s):
        torch.empty(1024 * (tag + 1), device=dev).fill_(1.0)


streams = []
if "--early" in sys.argv:
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    for i, s in enumerate(streams):
        touch(i + 1, s)
touch(0, torch.cuda.current_stream())
if "--dp" in sys.argv:
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]))
    so.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    t = torch.ones(4096, device=dev)
    dist.broadcast(t, 0)
    dist.all_reduce(t)
n0 = len(streams)
streams += [torch.cuda.Stream(device=dev) for _ in range(6)]
for i, s in enumerate(streams[n0:]):
    touch(n0 + i + 1, s)
touch(0, torch.cuda.current_stream())
torch.cuda.synchronize()
print("streams", [s.cuda_stream for s in streams])
if dist.is_initialized():
    dist.destroy_process_group()
