"""CPU, world_size 2 over gloo: the data-parallel exchange of the hot path.

Each rank takes its contiguous shard (nsm_amd.data.shard_range), computes the
oracle gradients of its shard into ONE flat buffer (the layout the HIP
backward produces), and calls nsm_amd.optim.allreduce_grads. The result must
equal the sum of both shards' gradients computed in one process (DDP
semantics: per-rank BN batch statistics, summed grads, mean folded into the
optimizer's clip coefficient)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard_grads(x_np, y_np, lo, hi):
    from oracle import unet_ref as O
    from oracle.weights import make_state
    sd = O.torch_state(make_state(7, 42), requires_grad=True)
    out, _ = O.forward(sd, torch.from_numpy(x_np[lo:hi]), True, None, 0.0)
    O.custom_loss(out, torch.from_numpy(y_np[lo:hi]), 0.9).backward()
    keys = O.param_keys(7)
    return [sd[k].grad.detach().clone() for k in keys]


def _worker(rank, world, port, x_np, y_np, q, overlap=False):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pcss-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nsm_amd.data import shard_range
    from nsm_amd.optim import allreduce_grads, flat_grad
    lo, hi = shard_range(len(x_np), world, rank)
    grads = shard_grads(x_np, y_np, lo, hi)
    total = sum(g.numel() for g in grads)
    flat = torch.empty(total)
    params, off = [], 0
    for g in grads:
        p = torch.nn.Parameter(torch.zeros_like(g))
        p.grad = flat[off:off + g.numel()].view_as(g)
        p.grad.copy_(g)
        params.append(p)
        off += g.numel()
    assert flat_grad(params) is not None
    if overlap:
        # what the Unet backward does: two buckets in flight, then a wait
        from nsm_amd.optim import allreduce_async
        split = sum(g.numel() for g in grads[:len(grads) // 2])
        allreduce_async(flat, split, total)
        allreduce_async(flat, 0, split)
    allreduce_grads(params)
    if rank == 0:
        q.put([p.grad.clone().numpy() for p in params])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    from nsm_amd.data import shard_range
    for n in (1, 7, 8, 512, 1001):
        for w in (1, 2, 4, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


@pytest.mark.timeout(600)
@pytest.mark.parametrize("overlap", [False, True])
def test_dp_allreduce_matches_sum_of_shards(overlap):
    from oracle.weights import synthetic_batch
    x_np, y_np = synthetic_batch(4, 7, 32, 32)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, x_np, y_np, q, overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=500)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    sys.path[:0] = [ROOT]
    ref = [a + b for a, b in zip(shard_grads(x_np, y_np, 0, 2), shard_grads(x_np, y_np, 2, 4))]
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r.numpy(), rtol=1e-5, atol=1e-7)


def _bn_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pcss-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import nsm_amd
    m = nsm_amd.Unet(in_ch=7)
    # every rank drifts its BN buffers differently (local batch statistics)
    g = torch.Generator().manual_seed(100 + rank)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.copy_(torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) + 0.5)
                mod.num_batches_tracked.fill_(3 + rank)
    keys = [k for k in m.state_dict() if "running" in k or "num_batches" in k]
    before = {k: v.clone() for k, v in m.state_dict().items() if k in keys}
    m.broadcast_buffers(0)
    after = {k: v.clone() for k, v in m.state_dict().items() if k in keys}
    # the flat re-homing keeps the reference's state_dict contract
    sd = m.state_dict()
    assert all(sd[k].shape == before[k].shape and sd[k].dtype == before[k].dtype for k in keys)
    # a .to() / load_state_dict after re-homing still broadcasts correctly
    m.load_state_dict(sd)
    m.broadcast_buffers(0)
    q.put((rank, {k: v.numpy() for k, v in before.items()}, {k: v.numpy() for k, v in after.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bn_buffers_broadcast_from_rank0():
    """SURVEY.md §8e / DDP broadcast_buffers: after Unet.broadcast_buffers()
    every rank holds rank 0's BN running stats and num_batches_tracked."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bn_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (b, a)) for r, b, a in (q.get(timeout=250) for _ in range(world)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    keys = list(res[0][0])
    assert len(keys) == 48
    for k in keys:
        assert np.array_equal(res[1][1][k], res[0][0][k]), k   # rank 1 now has rank 0's
        assert np.array_equal(res[0][1][k], res[0][0][k]), k   # rank 0 unchanged
    assert any(not np.array_equal(res[1][0][k], res[0][0][k]) for k in keys)


def _seed_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pcss-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import nsm_amd
    ps = [torch.nn.Parameter(torch.zeros(10)), torch.nn.Parameter(torch.zeros(3))]
    opt = nsm_amd.FlatAdamW(ps, world_size=world, sanitize=True)      # no seed given
    solo = nsm_amd.FlatAdamW([torch.nn.Parameter(torch.zeros(4))], world_size=1, sanitize=True)
    q.put((rank, opt.seed, solo.seed))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_flat_adamw_repair_seed_shared_across_ranks():
    """without an explicit seed every rank drew its own, so the
    NaN-repair noise (main.py:336) differed per rank and the replicas
    diverged. Under DP the seed is rank 0's everywhere."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=250) for _ in range(world)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]
    assert res[0][1] != res[1][1]    # world_size=1 optimizers keep their own draw
