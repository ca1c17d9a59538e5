import os, sys, torch, socket
sys.path[:0] = ['/root/repo', '/root/repo/pcss-unet_amd', '/root/repo/tests']
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
import torch.distributed as dist
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
import nsm_amd
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
m = nsm_amd.Unet(in_ch=7, dropout_rate=0.2).to(dev).train().data_parallel()
opt = nsm_amd.FlatAdamW(m.parameters(), lr=1e-3, max_grad_norm=1.0, sanitize=True)
crit = nsm_amd.CustomLoss(dev, 0.9, vgg_weights=False)
x = torch.randn(B, 7, 512, 512, device=dev); y = torch.rand(B, 1, 512, 512, device=dev)
def step():
    loss = crit(m(x), y, x); loss.backward()
    nsm_amd.allreduce_grads(m.parameters()); opt.step(); opt.zero_grad()
for _ in range(3): step()
torch.cuda.synchronize()
a0 = torch.cuda.memory_stats()["num_device_alloc"]; r0 = torch.cuda.memory_reserved()
for _ in range(20): step()
torch.cuda.synchronize()
print("eager DP: new device allocs over 20 steps:", torch.cuda.memory_stats()["num_device_alloc"] - a0,
      "reserved growth MB", (torch.cuda.memory_reserved() - r0) / 2**20)
dist.destroy_process_group()
