"""Probe: the eager train step (what main.py and every DP rank run) with the
weight-gradient side stream on / off, before and after a GraphedTrainStep of
the same shapes exists (bench.py's order), per step:

  * wall time (host clock, synchronised) and the HIP-event step time;
  * conv7.bwd's stage time (HIP events on the main stream);
  * torch.cuda.memory_stats() deltas across the step and across conv7.bwd
    (num_alloc_retries, num_device_alloc / free, reserved bytes);
  * with --launches: every libnsm launch inside conv7.bwd bracketed by HIP
    events on its stream, plus the host time spent in the call.

    python tools/eager_probe.py [--dtype bf16] [--batch 64] [--steps 6] [--launches]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pcss-unet_amd"))

KEYS = ("num_alloc_retries", "num_device_alloc", "num_device_free", "reserved_bytes.all.current",
        "allocated_bytes.all.current", "num_sync_all_streams")


def mstats():
    s = torch.cuda.memory_stats()
    return {k: s.get(k, 0) for k in KEYS}


def delta(a, b):
    return {k: b[k] - a[k] for k in KEYS}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--launches", action="store_true")
    ap.add_argument("--phases", default="eager_side,eager_one,graph,eager_side,eager_one")
    ap.add_argument("--out", default="gpurun_out/eager_probe.json")
    ap.add_argument("--bench", action="store_true",
                    help="run bench.train_measure's fp32 then bf16 sequence, conv7.bwd traced")
    a = ap.parse_args()
    import nsm_amd
    from nsm_amd import ops, unet
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, C, H = a.batch, 7, 512
    m = nsm_amd.Unet(in_ch=C, dropout_rate=0.2).to(dev).train()
    if a.dtype == "bf16":
        m.set_compute_dtype(torch.bfloat16)
    opt = nsm_amd.FlatAdamW(m.parameters(), lr=7e-4, weight_decay=1e-3, max_grad_norm=1.0,
                            sanitize=True)
    opt.set_epoch(0, 200)
    crit = nsm_amd.CustomLoss(dev, alpha=0.9, vgg_weights=False)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(True)
    y = torch.randint(0, 256, (B, 1, H, H), device=dev, generator=g).float() / 255.0

    rec = {"active": False, "launches": [], "mem": []}
    real_call = ops.call

    def traced_call(name, *args):
        if not (rec["active"] and a.launches) or torch.cuda.is_current_stream_capturing():
            return real_call(name, *args)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        sid = torch.cuda.current_stream().stream_id
        t0 = time.perf_counter()
        e0.record()
        r = real_call(name, *args)
        e1.record()
        rec["launches"].append((name, sid, e0, e1, time.perf_counter() - t0))
        return r

    for mod in (ops, unet):
        mod.call = traced_call
    real_bwd = unet._block_bwd

    def block_bwd(blk, *args, **kw):
        if blk is not m.conv7:
            return real_bwd(blk, *args, **kw)
        torch.cuda.current_stream()
        m0 = mstats()
        t0 = time.perf_counter()
        rec["active"] = True
        try:
            return real_bwd(blk, *args, **kw)
        finally:
            rec["active"] = False
            rec["mem"].append((time.perf_counter() - t0, delta(m0, mstats())))

    unet._block_bwd = block_bwd

    if a.bench:
        # bench.py's own sequence (fp32 B=8 headline, then the bf16 B=64
        # secondary), each a graph + eager probe steps, conv7.bwd traced
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        import bench
        report = []
        for kw in (dict(dtype="f32", batch=8, steps=20, warmup=5),
                   dict(dtype="bf16", batch=64, steps=10, warmup=3)):
            args = argparse.Namespace(in_ch=7, res=512, vgg=False, workload="train", **kw)
            torch.cuda.empty_cache()
            rec["all"] = []
            real_bwd2 = unet._block_bwd

            def bb(blk, s, G, grads, need_dx, name="", gpart=None, _r=real_bwd):
                if name != "conv7":
                    return _r(blk, s, G, grads, need_dx, name, gpart)
                m0 = mstats()
                t0 = time.perf_counter()
                rec["active"], rec["launches"] = True, []
                try:
                    return _r(blk, s, G, grads, need_dx, name, gpart)
                finally:
                    rec["active"] = False
                    rec["all"].append((time.perf_counter() - t0, delta(m0, mstats()),
                                       list(rec["launches"])))
            unet._block_bwd = bb
            res = bench.train_measure(args, 1, 0, dev)
            torch.cuda.synchronize()
            unet._block_bwd = real_bwd2
            calls = [{"host_ms": round(h * 1e3, 3), "mem": md,
                      "launches": [(n, sid, round(e0_.elapsed_time(e1_), 3), round(hh * 1e3, 3))
                                   for n, sid, e0_, e1_, hh in ls]} for h, md, ls in rec["all"]]
            r = {"cfg": kw, "value": res["value"], "ms_per_step": res["ms_per_step"],
                 "stages": res["stages"], "conv7_calls": calls}
            print(json.dumps({k: v for k, v in r.items() if k != "conv7_calls"}), flush=True)
            for c in calls:
                print(json.dumps({"host_ms": c["host_ms"], "mem": c["mem"],
                                  "launch_ms": [l[2] for l in c["launches"]],
                                  "launch_host_ms": [l[3] for l in c["launches"]]}), flush=True)
            report.append(r)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)
        return

    def step():
        out = m(x)
        loss = crit(out, y, x)
        loss.backward()
        opt.step()
        opt.zero_grad()
        x.grad = None

    report = []
    graphed = None
    for phase in a.phases.split(","):
        if phase == "graph":
            unet.WGRAD_STREAM = True
            t0 = time.perf_counter()
            graphed = nsm_amd.GraphedTrainStep(m, crit, opt, x, y, warmup=1)
            for _ in range(3):
                graphed()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(a.steps):
                graphed()
            torch.cuda.synchronize()
            r = {"phase": "graph", "capture_s": round(t1 - t0, 3),
                 "replay_ms": round((time.perf_counter() - t1) / a.steps * 1e3, 3),
                 "mem": mstats()}
            print(json.dumps(r), flush=True)
            report.append(r)
            continue
        unet.WGRAD_STREAM = phase == "eager_side"
        ops.PROBES["conv7.bwd"] = []
        rows = []
        for i in range(a.steps + 1):
            rec["launches"], rec["mem"] = [], []
            torch.cuda.synchronize()
            m0 = mstats()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            step()
            e1.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            st = ops.PROBES["conv7.bwd"][-1]
            row = {"step": i, "wall_ms": round(wall, 3), "event_ms": round(e0.elapsed_time(e1), 3),
                   "conv7_bwd_ms": round(st[0].elapsed_time(st[1]), 3),
                   "conv7_bwd_host_ms": round(rec["mem"][0][0] * 1e3, 3),
                   "conv7_mem": rec["mem"][0][1], "step_mem": delta(m0, mstats())}
            if a.launches:
                row["launches"] = [(n, sid, round(e0_.elapsed_time(e1_), 3), round(h * 1e3, 3))
                                   for n, sid, e0_, e1_, h in rec["launches"]]
            rows.append(row)
            print(json.dumps({"phase": phase, **{k: v for k, v in row.items()
                                                 if k != "launches"}}), flush=True)
        r = {"phase": phase, "graph_alive": graphed is not None, "rows": rows}
        report.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
