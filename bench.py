#!/usr/bin/env python3
"""Headline benchmark: frames/sec of the 7x512x512 -> 1x512x512 U-Net training
step (forward + CustomLoss + backward + grad all-reduce + clip + AdamW) on
MI355X, data-parallel over N GPUs (one process per GPU, RCCL over xGMI).

    python bench.py [--gpus N] [--steps K] [--warmup W]   # N > 1: spawns N ranks itself
    torchrun --nproc-per-node N bench.py --gpus N ...       # or one rank per GPU via torchrun
    python bench.py --dtype bf16 --batch 64                 # configs[2]
    python bench.py --workload infer1080 [--dtype bf16]     # configs[4]: 1080p eval fwd, hipGraph
    python bench.py --dry-run --gpus 2                      # CPU/gloo launcher check only

Workload (BASELINE.json configs[1]): batch 8 per GPU, 7x512x512 fp32
synthetic G-buffers (x ~ N(0,1), labels integers(0,256)/255), random-init
weights of the reference architecture, dropout 0.2 (train mode), inputs
resident in HBM and requiring grad like the reference's batches
(setdata.py:325-326). Weak scaling: per-GPU batch fixed as N grows.

Step = forward + 0.9*L1 + backward + RCCL grad all-reduce (N > 1, overlapped
with the backward) + the reference's whole step tail on the device
(main.py:287-423: sanitise, per-parameter clips, clip_grad_norm_, AdamW).
The step is timed eagerly, back to back, as an unchanged main.py loop runs it
(weight gradients on the side stream), and at N = 1 also replayed from one HIP
graph; both over K steps, the faster is the headline and the other is reported
beside it ("graph" or "eager"; NSM_BENCH_STEP=eager|graph fixes the headline).

Rank 0 prints ONE JSON line with the metric, a roofline object for the
dominant convolution (conv6.conv.0 forward, 3x3 1024->1024: Winograd input
transform + batched MFMA GEMM + output transform, timed as a whole with HIP
events on its launch stream during the timed steps, priced on SURVEY.md
§8(d)'s algorithmic FLOPs, with the executed-MFMA fraction beside it), a
per-stage table, and a CPU baseline (the oracle restatement on the host cores).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pcss-unet_amd"))
sys.path.insert(0, ROOT)
# Eager data-parallel ranks (N > 1 without NSM_GRAPH_DP): 8 hardware queues.
# HIP binds each stream, at its first launch, to the least used of at most
# GPU_MAX_HW_QUEUES queues (its default: 4); RCCL's and ProcessGroupNCCL's
# streams take three, and the Unet backward's weight-gradient side stream then
# shared the default stream's queue and ran serialised with it (round 6 kernel
# trace). fp32 B=8 eager DP at world size 1: 694 frames/s at 4 queues, 728-729
# at 8 (753.9 without DP); bf16 B=64 eager unchanged. Not for the captured
# step: the bf16 B=64 graph drops from 1639-1641 to 1480-1491 at 8 queues (its
# weight-gradient branch then truly runs beside the critical path, whose GEMMs
# are sized for the whole chip). Set before torch initialises HIP. --force-dp
# (the per-rank DP step at N = 1, eager in the headline) takes them too.
if ((int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--force-dp" in sys.argv)
        and os.environ.get("NSM_GRAPH_DP", "0") != "1"):
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32 MFMA = f32 vector peak (spec)
BF16_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (~2.5 PF)
HBM_PEAK_GBS = 8000.0


def conv_flops(B, H, W, cin, cout, k):
    return 2.0 * B * H * W * cin * cout * k * k


def unet_fwd_flops(in_ch, H, W):
    """sum over the 17 convs of 2*H*W*Cin*Cout*k^2 per frame."""
    R = (H // 2, W // 2)
    ch = {2: (4 * in_ch, 64), 3: (64, 128), 4: (128, 512), 5: (512, 1024),
          6: (1024, 512), 7: (512, 128), 8: (128, 64), 9: (64, 16)}
    res = {2: R, 3: (R[0] // 2, R[1] // 2), 4: (R[0] // 4, R[1] // 4), 5: (R[0] // 8, R[1] // 8),
           6: (R[0] // 4, R[1] // 4), 7: (R[0] // 2, R[1] // 2), 8: R, 9: R}
    f = 0.0
    for k, (ci, co) in ch.items():
        h, w = res[k]
        f += conv_flops(1, h, w, ci, ci, 3) + conv_flops(1, h, w, ci, co, 1)
    f += conv_flops(1, R[0], R[1], 16, 4, 1)
    return f


def vgg_fwd_flops(H, W):
    """VGG19 features[:31] on one 3xHxW image, incremental (97.1 GMAC at 512^2)."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512]
    f, c, h, w = 0.0, 3, H, W
    for v in cfg:
        if v == "M":
            h, w = h // 2, w // 2
        else:
            f += conv_flops(1, h, w, c, v, 3)
            c = v
    return f


STAGES = ["conv2", "conv3", "conv4", "conv5", "conv6", "conv7", "conv8", "conv9", "head"]


def f32_split_mode():
    """NSM_F32_SPLIT as libnsm reads it: 2 (default) the f16x2 split (3 f16
    products) for every GEMM of the train step (all operand maxima are recorded
    by their producers; only a fused BN-prologue operand, NSM_F32_ACT=0, falls
    back to the bf16 three-way split), 1 bf16 split (6 bf16 products)
    everywhere, 0 fp32 MFMA."""
    v = int(os.environ.get("NSM_F32_SPLIT", "2"))
    return min(max(v, 0), 2)


def pipe_products(bf16):
    """16-bit MFMA products per fp32 product: (Winograd GEMMs, direct GEMMs)
    and the dense peak of the pipe that runs them."""
    if bf16:
        return (1, 1), BF16_PEAK_TFLOPS
    m = f32_split_mode()
    if m == 0:
        return (1, 1), FP32_PEAK_TFLOPS
    return ((3, 3) if m == 2 else (6, 6)), BF16_PEAK_TFLOPS


def stage_work(in_ch, H, W, B, bytes_per=4, wino_min=128, tile=4, passes=3):
    """Per stage: (algorithmic FLOPs, executed fp32-product FLOPs of the
    Winograd GEMMs, of the direct GEMMs, HBM bytes) of one train step
    (passes=3: fwd + dgrad + wgrad) or one forward (passes=1).

    Algorithmic = SURVEY.md §8(d): conv FLOPs 2*H*W*Cin*Cout*k^2 per pass;
    bytes = (Cin+Cout)*H*W*s + weights*s per conv and pass. Executed counts
    what the MFMA units really do: 3x3 convs with Cin >= wino_min run Winograd
    F(m x m,3x3), m = tile ((m+2)^2 GEMMs of T = B*ceil(h/m)*ceil(w/m) rows per
    pass: 2*(m+2)^2*T*Cin*Cout instead of 18*B*h*w*Cin*Cout). conv5's
    checkpoint recompute (Unetmodel.py:118) is not executed: its activations
    are kept (the double BN running-stat update is reproduced)."""
    R = (H // 2, W // 2)
    ch = {2: (4 * in_ch, 64), 3: (64, 128), 4: (128, 512), 5: (512, 1024),
          6: (1024, 512), 7: (512, 128), 8: (128, 64), 9: (64, 16)}
    res = {2: R, 3: (R[0] // 2, R[1] // 2), 4: (R[0] // 4, R[1] // 4), 5: (R[0] // 8, R[1] // 8),
           6: (R[0] // 4, R[1] // 4), 7: (R[0] // 2, R[1] // 2), 8: R, 9: R}
    out = {}
    for k, (ci, co) in ch.items():
        h, w = res[k]
        px = B * h * w
        f = 2.0 * px * (ci * ci * 9 + ci * co)
        cp = (ci + 31) // 32 * 32
        m = tile(cp, h, w) if callable(tile) else tile
        T = B * ((h + m - 1) // m) * ((w + m - 1) // m)
        wino = cp >= wino_min
        f3 = 2.0 * (m + 2) ** 2 * T * ci * ci if wino else 18.0 * px * ci * ci
        f1 = 2.0 * px * ci * co
        by = ((ci + ci) * px + 9 * ci * ci + (ci + co) * px + ci * co) * bytes_per
        out[f"conv{k}"] = (passes * f, passes * (f3 if wino else 0.0),
                           passes * (f1 + (0.0 if wino else f3)), passes * by)
    px = B * R[0] * R[1]
    fh = 2.0 * px * 16 * 4
    out["head"] = (passes * fh, 0.0, 0.0, passes * (16 * px + 4 * px) * bytes_per)
    return out


STAGE_COLS = ["stage", "ms", "alg_tflops", "mfma_frac", "hbm_frac", "meas_gbs", "meas_hbm_frac",
              "meas_over_alg", "mfma_busy", "meas_mfma_frac"]


def stage_table(work, times_ms, pipe_mult, peak, measured=None):
    """Per-stage rows (STAGE_COLS): live time (HIP events), algorithmic
    (direct-conv) TFLOP/s, `mfma_frac` = the matrix-core work the stage issues
    on the pipe that runs it (pipe_mult = 16-bit products per fp32 product of
    its Winograd GEMMs and of its direct GEMMs: f16x2 3, bf16 split 6;
    pipe_products) / time / that pipe's dense peak, `hbm_frac` = algorithmic bytes /
    time / 8 TB/s; with a committed PMC summary (tools/stage_pmc.py) of the same
    configuration: measured HBM bytes (TCC fabric requests + WRITE_SIZE) / live
    time, their ratio to the algorithmic bytes, MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES
    per SIMD-cycle at the held clock) and the counted MFMA work (512 x
    SQ_INSTS_VALU_MFMA_MOPS_*) / live time / peak."""
    rows = []
    ms_ = (measured or {}).get("stages", {})
    for st in STAGES:
        if st not in times_ms:
            continue
        t = times_ms[st] * 1e-3
        fl, exw, exd, by = work[st]
        m = ms_.get(st, {})
        mb = m.get("hbm_bytes")
        mf = None
        if "bf16_mfma_flops" in m:
            mf = (m["bf16_mfma_flops"] / (BF16_PEAK_TFLOPS * 1e12)
                  + m.get("f32_mfma_flops", 0.0) / (FP32_PEAK_TFLOPS * 1e12)) / t
        rows.append([st, round(t * 1e3, 3), round(fl / t / 1e12, 1),
                     round((pipe_mult[0] * exw + pipe_mult[1] * exd) / t / (peak * 1e12), 3),
                     round(by / t / (HBM_PEAK_GBS * 1e9), 3),
                     round(mb / t / 1e9) if mb else None,
                     round(mb / t / (HBM_PEAK_GBS * 1e9), 3) if mb else None,
                     round(mb / by, 2) if mb else None,
                     m.get("mfma_busy"), round(mf, 3) if mf is not None else None])
    return rows


_LIB_SHA = []


def loaded_lib_sha256():
    """sha256 of the libnsm.so this process loaded (the profile stamps' key)."""
    if not _LIB_SHA:
        import hashlib
        import nsm_amd
        with open(nsm_amd.LIB_PATH, "rb") as f:
            _LIB_SHA.append(hashlib.sha256(f.read()).hexdigest())
    return _LIB_SHA[0]


def _stamped(doc, rel):
    """(doc, source) when the summary was measured on the loaded library,
    else (None, "<file> (stale: ...)") — a profile of another build never
    feeds the driver line (tools/stage_pmc.py stamp)."""
    st = (doc or {}).get("stamp") or {}
    if st.get("libnsm_sha256") != loaded_lib_sha256():
        return None, f"{rel} (stale: measured on libnsm {str(st.get('libnsm_sha256'))[:12]}, " \
                     f"loaded {loaded_lib_sha256()[:12]})"
    return doc, rel


def load_stage_pmc(tag):
    """The newest committed per-stage PMC summary of this configuration, if it
    was measured on the loaded library."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"stage_pmc_{tag}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        return _stamped(json.load(f), os.path.relpath(files[-1], ROOT))


def mean_ms(evs):
    return float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs else float("nan")


def load_traffic(name):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (tools/pmc_traffic.py: sized TCC fabric read requests +
    WRITE_SIZE)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t, src = _stamped(json.load(f), os.path.relpath(files[-1], ROOT))
    return (t.get("traffic_bytes_per_launch") if t else None), src


def cpu_baseline(in_ch, H, W, frames=8, reps=3, train=True, bf16_autocast=False):
    """The reference's CPU path timed on this box's host cores: the oracle
    restatement (same ATen ops as Unetmodel.py) on a bounded sample (`frames`
    frames, median of `reps` after one warmup). train: fwd + 0.9*L1 + bwd at
    the headline batch (B=8); else the eval forward under inference_mode, with
    bf16_autocast = infer.py's CPU mode (`torch.amp.autocast('cpu',
    dtype=torch.bfloat16)`, infer.py:63-65).
    Threads: the CPU share the GPU box grants this job (OMP_NUM_THREADS = 16
    per GPU); os.sched_getaffinity lists the whole host's cores there
    (`affinity_cores`), which other jobs' GPUs share."""
    from oracle import unet_ref as O
    from oracle.weights import make_state, synthetic_batch
    cores = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", cores))
    torch.set_num_threads(max(1, min(cores, share)))
    sd = O.torch_state(make_state(in_ch, 42), requires_grad=train)
    x_np, y_np = synthetic_batch(frames, in_ch, H, W)
    y = torch.from_numpy(y_np)

    def step():
        if train:
            x = torch.from_numpy(x_np).requires_grad_(True)
            out, _ = O.forward(sd, x, True, None, 0.0)
            O.custom_loss(out, y, 0.9).backward()
        else:
            with torch.inference_mode(), torch.amp.autocast("cpu", dtype=torch.bfloat16,
                                                            enabled=bf16_autocast):
                O.forward(sd, torch.from_numpy(x_np), False)

    step()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    what = ("train step (fwd+0.9*L1+bwd) fp32" if train else
            "eval forward, inference_mode + bf16 autocast (infer.py:63-65 CPU mode)"
            if bf16_autocast else "eval forward, inference_mode, fp32")
    return {"value": round(frames / t, 4), "unit": "frames/s", "cores": torch.get_num_threads(),
            "affinity_cores": cores, "kind": "port",
            "cores_policy": "the box's CPU share per GPU (OMP_NUM_THREADS); affinity spans the "
                            "whole shared host",
            "sample": f"{frames} frame(s) {in_ch}x{H}x{W} {what}, oracle/unet_ref.py on PyTorch "
                      f"CPU, median of {reps} after 1 warmup, {round(sum(ts), 2)} s timed"}


def dominant_roofline(B, H, W, conv_ms, gemm_ms, launches, wino_tile):
    """Roofline object of the step's dominant kernel: conv6.conv.0's forward
    Winograd batched GEMM (nsm_wino_gemm, (m+2)^2 GEMMs of T x 1024 x 1024),
    timed per launch with HIP events on its stream. Priced on the pipe that
    runs it: with the f16x2 split (default) every fp32 product is 3 f16 MFMA
    products (6 bf16 ones under the three-way bf16 split, NSM_F32_SPLIT=1), so
    achieved = 3 x 2*(m+2)^2*T*1024^2 / launch time against the dense 16-bit
    peak (frac <= 1); NSM_F32_SPLIT=0 runs the fp32 MFMA (one product each,
    fp32 peak). `whole_conv` adds the two Winograd transforms
    (input + output): its time, the same work / that time, and SURVEY.md
    §8(d)'s direct-convolution FLOPs / that time (`direct_equiv_tflops`, a
    rate, not a roofline position: Winograd issues 5x fewer products)."""
    Rh, Rw = H // 2, W // 2
    m, nb = wino_tile, (wino_tile + 2) ** 2
    h6, w6 = Rh // 4, Rw // 4                     # conv6 runs at (H/8, W/8)
    T6 = B * ((h6 + m - 1) // m) * ((w6 + m - 1) // m)
    alg_flops = conv_flops(B, h6, w6, 1024, 1024, 3)
    alg_bytes = (2 * B * h6 * w6 * 1024 + 9 * 1024 * 1024 + 1024) * 4
    ex_flops = nb * 2.0 * T6 * 1024 * 1024
    gemm_bytes = nb * (2 * T6 * 1024 + 1024 * 1024) * 4  # read V, U; write M
    mode = f32_split_mode()
    mult, peak = {0: (1, FP32_PEAK_TFLOPS), 1: (6, BF16_PEAK_TFLOPS),
                  2: (3, BF16_PEAK_TFLOPS)}[mode]
    work = mult * ex_flops
    achieved = work / (gemm_ms * 1e-3) / 1e12
    from nsm_amd.prep import H2_WINO
    f16 = ("gemm_h2p_kernel<256,256> (fp32 via the f16x2 split: the two fp16 terms of each "
           "power-of-two scaled operand written by its producer, LDS-DMA, 3 products on "
           "v_mfma_f32_16x16x32_f16; persistent, one block per CU over the 4x4x64 tiles)"
           if H2_WINO else
           "gemm_f32h_kernel (fp32 via the f16x2 split of power-of-two scaled operands, 3 "
           "products on v_mfma_f32_32x32x16_f16)")
    return {"kernel": f"conv6.conv.0.fwd Winograd F({m}x{m},3x3) batched GEMM "
                      f"({nb} x M={T6} N=1024 K=1024), B={B} at {h6}x{w6}: "
                      + {2: f16,
                         1: "gemm_f32s_kernel (fp32 via the exact 3-way bf16 split, 6 products on "
                            "v_mfma_f32_32x32x16_bf16)",
                         0: "gemm_f32_kernel (v_mfma_f32_32x32x2_f32)"}[mode],
            "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "basis": (f"matrix-core work issued per launch on the pipe that runs it ({mult} x "
                      f"{ex_flops / 1e9:.1f} GFLOP of fp32 products) / launch time / that pipe's "
                      "dense peak"),
            "avg_launch_ms": round(gemm_ms, 4), "launches": launches,
            "flops_per_launch": work, "fp32_product_flops_per_launch": ex_flops,
            "algorithmic_bytes_per_launch": gemm_bytes,
            "whole_conv": {"what": "nsm_wino_input + nsm_wino_gemm + nsm_wino_output",
                           "avg_ms": round(conv_ms, 4),
                           "pipe_frac": round(work / (conv_ms * 1e-3) / 1e12 / peak, 4),
                           "direct_equiv_tflops": round(alg_flops / (conv_ms * 1e-3) / 1e12, 1),
                           "direct_conv_flops": alg_flops, "direct_conv_bytes": alg_bytes}}


def wino_f16_roofline(B, H, W, conv_ms, gemm_ms, launches):
    """Roofline object of conv6.conv.0's forward on the bf16 path (at >= 512
    channels, nsm_amd.prep.BF16_WINO): Winograd F(4x4,3x3) on single-plane
    scaled f16 operands, 36 batched GEMMs of T x 1024 x 1024 on
    gemm_h2p_kernel's single-plane mode (ONE f16 product per fp32-accumulated
    term: the pipe work equals the Winograd products), HIP events per launch.
    whole_conv adds the input / output transforms and the direct-conv rate."""
    from nsm_amd.ops import BF16_M16
    h6, w6 = H // 8, W // 8
    T6 = B * ((h6 + 3) // 4) * ((w6 + 3) // 4)
    work = 36 * 2.0 * T6 * 1024 * 1024
    alg_flops = conv_flops(B, h6, w6, 1024, 1024, 3)
    alg_bytes = (2 * B * h6 * w6 * 1024 + 9 * 1024 * 1024) * 2
    achieved = work / (gemm_ms * 1e-3) / 1e12
    m_bytes = 2 if BF16_M16 else 4   # M written as f16 (nsm_wino_gemm_f16m) or fp32
    return {"kernel": f"conv6.conv.0.fwd bf16 path: Winograd F(4x4,3x3) batched GEMM (36 x M={T6} "
                      f"N=1024 K=1024) on single-plane scaled f16 operands, B={B} at {h6}x{w6}: "
                      "gemm_h2p_kernel<256,256,...,SP> (persistent, LDS-DMA, "
                      "v_mfma_f32_16x16x32_f16, one product per term; M written as "
                      + ("f16)" if BF16_M16 else "fp32)"),
            "bound": "mfma", "achieved": round(achieved, 2), "peak": BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
            "basis": f"f16 MFMA work per launch ({work / 1e9:.1f} GFLOP) / launch time / dense peak",
            "avg_launch_ms": round(gemm_ms, 4), "launches": launches, "flops_per_launch": work,
            # V + U read, M written
            "algorithmic_bytes_per_launch": 36 * (T6 * 1024 * 2 + 1024 * 1024 * 2 + T6 * 1024 * m_bytes),
            "whole_conv": {"what": "nsm_wino_input_f16 + nsm_wino_gemm_f16" + ("m" if BF16_M16 else "")
                                   + " + nsm_wino_output_bf16" + ("m" if BF16_M16 else ""),
                           "avg_ms": round(conv_ms, 4),
                           "pipe_frac": round(work / (conv_ms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS, 4),
                           "direct_equiv_tflops": round(alg_flops / (conv_ms * 1e-3) / 1e12, 1),
                           "direct_conv_flops": alg_flops, "direct_conv_bytes": alg_bytes}}


def vgg_roofline(B, H, W, conv_ms, gemm_ms, launches, amax):
    """Roofline object of the deepest VGG19 conv the perceptual loss runs
    (features.30, 512->512 3x3 at H/16 x W/16 on the 2B output+target images,
    customLoss.py:42-90): Winograd F(4x4,3x3), 36 batched GEMMs of T x 512 x
    512, timed per launch with HIP events. Its operands carry recorded maxima
    (amax) -> the f16x2 split (3 f16 products per fp32 product), else the
    bf16 three-way split (6)."""
    h, w = H // 16, W // 16
    T = 2 * B * ((h + 3) // 4) * ((w + 3) // 4)
    ex = 36 * 2.0 * T * 512 * 512
    mult = 3 if amax else 6
    work = mult * ex
    achieved = work / (gemm_ms * 1e-3) / 1e12
    alg = conv_flops(2 * B, h, w, 512, 512, 3)
    return {"kernel": f"vgg features.30 fwd: Winograd F(4x4,3x3) batched GEMM (36 x M={T} N=512 "
                      f"K=512), 2B={2 * B} images at {h}x{w}, fp32 via "
                      + ("the f16x2 split (3 f16 products)" if amax else
                         "the exact 3-way bf16 split (6 bf16 products)"),
            "bound": "mfma", "achieved": round(achieved, 2), "peak": BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
            "basis": f"16-bit MFMA work per launch ({mult} x {ex / 1e9:.1f} GFLOP of fp32 products) "
                     "/ launch time / dense peak",
            "avg_launch_ms": round(gemm_ms, 4), "launches": launches, "flops_per_launch": work,
            "whole_conv": {"avg_ms": round(conv_ms, 4),
                           "direct_equiv_tflops": round(alg / (conv_ms * 1e-3) / 1e12, 1)}}


def direct_roofline(B, H, W, kern_ms, launches, f16=False):
    """Roofline object of conv6.conv.0 forward as one bf16 (f16) implicit GEMM
    (M = B*(H/8)*(W/8) pixels, N = 1024, K = 9*1024)."""
    M = B * (H // 8) * (W // 8)
    k_flops = conv_flops(B, H // 8, W // 8, 1024, 1024, 3)
    k_bytes = (2 * M * 1024 + 9 * 1024 * 1024) * 2
    achieved = k_flops / (kern_ms * 1e-3) / 1e12
    fn = "nsm_conv_fwd_f16" if f16 else "nsm_conv_fwd_bf16"
    return {"kernel": f"conv6.conv.0.fwd {'f16' if f16 else 'bf16'} implicit-GEMM 3x3 ({fn}: "
                      f"M={M} N=1024 K=9216)",
            "bound": "mfma", "achieved": round(achieved, 2), "peak": BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
            "avg_launch_ms": round(kern_ms, 4), "launches": launches,
            "algorithmic_flops_per_launch": k_flops, "algorithmic_bytes_per_launch": k_bytes}


def init_dist(args):
    """One process per GPU: torchrun's env (WORLD_SIZE/RANK/LOCAL_RANK), or the
    workers bench.py spawned itself for --gpus N. RCCL (`nccl`) on the GPUs;
    gloo for --dry-run (CPU launcher check)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        return world, rank, torch.device("cpu")
    if world > 1 or (getattr(args, "force_dp", False) and not dist.is_initialized()):
        import nsm_amd
        torch.cuda.set_device(local)
        # the weight-gradient side stream on a hardware queue of its own,
        # before RCCL's streams take the free ones (nsm_amd.reserve_side_stream)
        nsm_amd.reserve_side_stream(torch.device("cuda", local))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    elif getattr(args, "force_dp", False) and not dist.is_initialized():
        # --force-dp at N=1: the data-parallel step over a world-size-1 RCCL group
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", rank=0, world_size=1,
                                device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def timed(fn, steps, world, dev):
    """Barrier + synchronize on both sides, max over ranks."""
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    _sync(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def run_dry(args):
    """--dry-run: the launcher / rendezvous / timing / JSON plumbing of the
    train bench on CPU processes over gloo, with a stand-in step (a 1 MiB
    all-reduce). No GPU is touched; the line says dry_run so it can never pass
    for a measurement."""
    world, rank, dev = init_dist(args)
    buf = torch.ones(1 << 18)

    def step():
        if world > 1:
            dist.all_reduce(buf)

    for _ in range(args.warmup):
        step()
    elapsed = timed(step, args.steps, world, dev)
    # the workloads a real run at this N measures (train: headline + secondary)
    plan = [{"config": "configs[1]", "role": "headline", "batch_per_gpu": args.batch,
             "global_batch": world * args.batch, "dtype": args.dtype}]
    if not args.no_secondary:
        plan.append({"config": "configs[3]" if world > 1 else "configs[2] (= configs[3] at N=1)",
                     "role": "secondary", "batch_per_gpu": 64, "global_batch": world * 64,
                     "dtype": "bf16"})
        if world == 1:
            plan += [{"config": "configs[4]", "role": "secondary", "batch_per_gpu": 1,
                      "dtype": d} for d in ("bf16", "f32")]
            plan.append({"config": "configs[0]", "role": "secondary", "batch_per_gpu": 1,
                         "dtype": "f32"})
    if rank == 0:
        print(json.dumps({"metric": "dry-run (launcher check, not a measurement)", "value": 0.0,
                          "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
                          "dry_run": True, "world_size": world,
                          "backend": dist.get_backend() if world > 1 else None,
                          "workloads": plan}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_train(args):
    world, rank, dev = init_dist(args)
    res = train_measure(args, world, rank, dev)
    if not args.no_secondary:
        sec = secondary_configs(args, world, rank, dev)
        if rank == 0:
            res["secondary"] = sec
    C, H, W = args.in_ch, args.res, args.res
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(C, H, W, frames=args.batch)
        if args.dtype in ("bf16", "f16"):
            res["cpu_baseline"]["sample"] += " (fp32: the reference's CPU path)"
    if rank == 0:
        emit(res, args)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def emit(res, args):
    """The ONE JSON line (compact: the driver keeps its last 2000 characters,
    so the secondary configs and the CPU baseline come last) and, with
    --detail PATH, the full record as a file."""
    if args.detail:
        with open(args.detail, "w") as f:
            json.dump(res, f, indent=1)
    out = {k: v for k, v in res.items() if k not in ("secondary", "cpu_baseline", "_full")}
    if "secondary" in res:
        out["secondary"] = res["secondary"]
    if "cpu_baseline" in res:
        out["cpu_baseline"] = res["cpu_baseline"]
    print(json.dumps(out, separators=(",", ":")), flush=True)


def _summary(r):
    """A secondary measurement as kept in the headline JSON line."""
    roof = r["roofline"]
    out = {"config": r["config"]["workload"].split(":")[0], "dtype": r["dtype"],
           "global_batch": r["config"]["global_batch"], "value": r["value"], "unit": r["unit"],
           "ms_per_step": r["ms_per_step"], "steps": r["steps"],
           "roofline": {k: roof.get(k) for k in ("achieved", "frac", "avg_launch_ms", "traffic")}}
    if "dp" in r:
        out["dp"] = r["dp"]
    for k2 in ("eager", "graph"):
        if k2 in r:
            out[k2] = {k: r[k2][k] for k in ("value", "ms_per_step", "steps")}
            out["execution"] = "graph" if k2 == "eager" else "eager"   # the headline's
    if r["config"]["workload"].startswith(("configs[2]", "configs[3]")):
        out["stages"] = r["stages"]
    if "vgg_perceptual" in r:
        out["config"] += "+vgg"
        out["vgg_perceptual"] = r["vgg_perceptual"]
    if "cpu_baseline" in r:
        out["cpu_baseline"] = r["cpu_baseline"]
    return out


def secondary_configs(args, world, rank, dev):
    """The other BASELINE.json configs measured in the same run (so the
    driver's record carries them). Every N: configs[3]'s per-GPU work (B=64
    bf16 train step per GPU: global batch 512 at N=8; at N=1 this is
    configs[2]). N=1 also: configs[4] (1080p hipGraph inference, bf16 and fp32,
    each beside the reference's CPU infer.py timing of the same mode) and
    configs[0] (1x7x256x256 eval)."""
    import argparse as _ap
    out = []
    base = dict(vars(args))
    kws = [dict(workload="train", dtype="bf16", batch=64, steps=max(10, args.steps // 5),
                warmup=3)]
    if world == 1:
        # the reference's own GPU precision mode (fp16 autocast + GradScaler,
        # main.py:175,257-259,281,368) at configs[2]'s batch
        kws += [dict(workload="train", dtype="f16", batch=64, steps=max(10, args.steps // 5),
                     warmup=3)]
    if world == 1:
        # the reference-faithful step: CustomLoss with its VGG19 perceptual
        # term (customLoss.py:137; random-init VGG weights, value unpinned)
        kws += [dict(workload="train", dtype="f32", batch=8, steps=max(5, args.steps // 10),
                     warmup=2, vgg=True)]
        kws += [dict(workload="infer1080", dtype="bf16", batch=1, steps=100, warmup=5),
                dict(workload="infer1080", dtype="f32", batch=1, steps=50, warmup=5),
                dict(workload="infer256", dtype="f32", batch=1, steps=100, warmup=5)]
    for kw in kws:
        a = _ap.Namespace(**{**base, "vgg": False, **kw})
        torch.cuda.empty_cache()
        if a.workload == "train":
            r = train_measure(a, world, rank, dev)
        else:
            r = infer_measure(a, world, rank, dev)
            if a.workload == "infer1080" and rank == 0 and not args.no_cpu_baseline:
                r["cpu_baseline"] = cpu_baseline(a.in_ch, 1080, 1920, frames=1, reps=3,
                                                 train=False, bf16_autocast=a.dtype == "bf16")
        out.append(_summary(r))
    torch.cuda.empty_cache()
    return out


def train_measure(args, world, rank, dev):
    import nsm_amd
    from nsm_amd import ops as nops
    from nsm_amd.unet import WINOGRAD_MIN_CHANNELS, wino_tile

    torch.manual_seed(1234 + rank)
    B, C, H, W = args.batch, args.in_ch, args.res, args.res
    bf16 = args.dtype in ("bf16", "f16")   # the 16-bit storage paths
    f16 = args.dtype == "f16"
    model = nsm_amd.Unet(in_ch=C, dropout_rate=0.2).to(dev).train()
    if bf16:
        model.set_compute_dtype(torch.float16 if f16 else torch.bfloat16)
    # f16: GradScaler's loss scale (main.py:175,281; its initial 2^16, held
    # fixed here), unscaled inside the tail (main.py:361-368)
    loss_scale = 65536.0 if f16 else 1.0
    # data parallel at N > 1, or at N = 1 over a world-size-1 RCCL group
    # (--force-dp: the per-rank step of configs[3] with its collectives)
    dp = world > 1 or getattr(args, "force_dp", False)
    if dp:  # identical initial weights on every rank (DDP semantics)
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p, 0)
        # decoder bucket reduces under the encoder backward; rank 0's BN buffers
        # are broadcast at each forward (DDP semantics)
        model.data_parallel()
    # the reference's whole step tail (main.py:287-423) on the device: sanitise,
    # per-parameter clips, clip_grad_norm_(1.0) (epoch 0 of 200), AdamW
    opt = nsm_amd.FlatAdamW(model.parameters(), lr=7e-4, weight_decay=1e-3, max_grad_norm=1.0,
                            world_size=world, sanitize=True, grad_scale=loss_scale)
    opt.set_epoch(0, 200)
    crit = nsm_amd.CustomLoss(dev, alpha=0.9, vgg_weights="random" if args.vgg else False)
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(B, C, H, W, device=dev, generator=g).requires_grad_(True)
    y = (torch.randint(0, 256, (B, 1, H, W), device=dev, generator=g).float() / 255.0)

    # the backward's seed gradient (the f16 loss scale, else 1), allocated once
    # as GraphedTrainStep does: loss.backward() would fill a fresh ones tensor
    # with an ATen kernel every step (and f16's loss * scale another)
    seed = torch.full((), loss_scale, dtype=torch.float32, device=dev)

    def step():
        out = model(x)
        loss = crit(out, y, x)
        loss.backward(seed)
        if dp:
            # the exposed part of the overlapped all-reduce: how long the compute
            # stream waits for RCCL after the backward (HIP events)
            with nops.stage("dp.allreduce_wait"):
                nsm_amd.allreduce_grads(model.parameters())
        opt.step()
        opt.zero_grad()
        # the reference's batch is a fresh tensor every step (setdata.py:325-326),
        # so its input gradient is written once, never accumulated into an old one
        x.grad = None
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # Two executions of the same step: eager (what an unchanged main.py loop and
    # every DP rank run, the weight gradients on the side stream) and, at N = 1,
    # the replay of one HIP graph (nsm_amd.GraphedTrainStep: dropout masks from
    # the graph-safe generator, new every replay). NSM_BENCH_STEP=auto (default)
    # times both over K steps and reports the faster as the headline, the other
    # beside it: the eager step wins where the host keeps ahead of the GPU (its
    # side-stream overlap; interleaved A/B on one box: eager 797.8 / 798.5 /
    # 798.3 frames/s vs replay 771.7 / 769.0 / 769.0), the replay where the host
    # is slow. eager / graph: that mode is the headline, the other timed over
    # min(K, 20) steps beside it. The kernel / stage timings below come from
    # eager steps of the same shapes.
    mode = os.environ.get("NSM_BENCH_STEP", "auto")
    head_graph = mode == "graph"
    graphed, dp_ms = None, None
    dp_tags = ("dp.bn_broadcast", "dp.allreduce_wait")
    side_elapsed, side_steps = None, max(3, min(args.steps, 20))
    # one process: the graph too; N > 1 ranks run eager steps only unless
    # NSM_GRAPH_DP=1 (the captured DP step, collectives inside)
    want_graph = os.environ.get("NSM_GRAPH_STEP", "1") != "0" and (
        world == 1 or os.environ.get("NSM_GRAPH_DP", "0") == "1")
    if want_graph and head_graph:
        graphed = nsm_amd.GraphedTrainStep(model, crit, opt, x, y, loss_scale=loss_scale,
                                           warmup=1)
        for _ in range(args.warmup):
            graphed()
        torch.cuda.synchronize()
        elapsed = timed(graphed, args.steps, world, dev)
        # the eager step beside it; only the DP waits carry events
        if dp:
            for t in dp_tags:
                nops.PROBES[t] = []
        side_elapsed = timed(step, side_steps, world, dev)
    else:
        # eager timed steps: only the DP waits carry HIP events
        for t in dp_tags:
            nops.PROBES[t] = []
        elapsed = timed(step, args.steps, world, dev)
        dp_ms = {t: mean_ms(nops.PROBES.pop(t, [])) for t in dp_tags}
        if want_graph:
            graphed = nsm_amd.GraphedTrainStep(model, crit, opt, x, y, loss_scale=loss_scale,
                                               warmup=1)
            for _ in range(args.warmup):
                graphed()
            torch.cuda.synchronize()
            g_steps = args.steps if mode == "auto" else side_steps
            g_elapsed = timed(graphed, g_steps, world, dev)
            if mode == "auto" and g_elapsed < elapsed:
                # the replay is the faster execution on this machine
                side_elapsed, side_steps, elapsed, head_graph = elapsed, args.steps, g_elapsed, True
            else:
                side_elapsed, side_steps = g_elapsed, g_steps
    if dp_ms is None:
        dp_ms = {t: mean_ms(nops.PROBES.pop(t, [])) for t in dp_tags}

    # attribution steps (not timed): kernel and stage times from HIP events
    # with the weight gradients on the main stream, the configuration the
    # per-stage counters are taken in (tools/stage_pmc.py, NSM_STAGE_MARKS),
    # so each stage's bytes and time describe the same kernels
    probe_tag = "conv6.conv.0.fwd"
    nops.PROBES[probe_tag] = []
    nops.PROBES[probe_tag + ".gemm"] = []
    for st in STAGES:
        nops.PROBES[st + ".fwd"] = []
        nops.PROBES[st + ".bwd"] = []
    nops.PROBES["vgg.fwd"] = []
    nops.PROBES["vgg.30"] = []
    nops.PROBES["vgg.30.gemm"] = []
    from nsm_amd import unet as nunet
    side_prev, nunet.WGRAD_STREAM = nunet.WGRAD_STREAM, False
    try:
        for _ in range(min(args.steps, 10)):
            step()
        torch.cuda.synchronize()
    finally:
        nunet.WGRAD_STREAM = side_prev
    evs = nops.PROBES.pop(probe_tag)
    kern_ms = mean_ms(evs)
    gemm_ms = mean_ms(nops.PROBES.pop(probe_tag + ".gemm"))
    vgg_evs = nops.PROBES.pop("vgg.fwd")
    vgg30 = nops.PROBES.pop("vgg.30")
    vgg30_gemm = mean_ms(nops.PROBES.pop("vgg.30.gemm"))
    times = {}
    for st in STAGES:
        fw, bw = nops.PROBES.pop(st + ".fwd"), nops.PROBES.pop(st + ".bwd")
        if fw and bw:
            times[st] = mean_ms(fw) + mean_ms(bw)
    full = (H, W, C) == (512, 512, 7)
    pipe_mult, peak = pipe_products(bf16)
    if bf16:
        from nsm_amd.prep import BF16_WINO, BF16_WINO_MIN
        wino = BF16_WINO and not f16   # f16: direct convolutions only (its parity anchor)
        work = stage_work(C, H, W, B, bytes_per=2, wino_min=BF16_WINO_MIN if wino else 1 << 30)
        roof = (wino_f16_roofline(B, H, W, kern_ms, gemm_ms, len(evs)) if wino and gemm_ms
                else direct_roofline(B, H, W, kern_ms, len(evs), f16))
        traffic, traffic_src = (load_traffic("traffic_conv6_fwd_gemm_bf16.json" if BF16_WINO
                                             else "traffic_conv6_fwd_bf16.json")
                                if B == 64 and full and not f16 else (None, None))
        tag = f"b{B}_{args.dtype}"
    else:
        work = stage_work(C, H, W, B, wino_min=WINOGRAD_MIN_CHANNELS, tile=wino_tile)
        traffic, traffic_src = (load_traffic("traffic_conv6_fwd_gemm_f32.json") if B == 8 and full
                                else (None, None))
        roof = dominant_roofline(B, H, W, kern_ms, gemm_ms, len(evs), wino_tile(1024, H // 8, W // 8))
        tag = f"b{B}_f32"
    roof.update({"traffic": traffic, "traffic_source": traffic_src})
    measured, measured_src = load_stage_pmc(tag) if full else (None, None)

    frames = world * B * args.steps
    step_flops = 3 * unet_fwd_flops(C, H, W) * B
    res = {
        "metric": "frames/sec 7x512x512 U-Net fwd+bwd (train step)",
        "value": round(frames / elapsed, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype if bf16 else "f32",
        "data": "synthetic (x~N(0,1), labels integers(0,256)/255), random-init weights",
        "config": {"workload": (f"batch={B}/GPU {C}x{H}x{W} f16 (fp16-autocast mode: direct "
                                "convolutions on f16 operands, f16 activations, fp32 accumulate, "
                                "BN stats, params, grads; loss scale 2^16 unscaled in the tail) "
                                "train step " if f16 else
                                f"configs[2]: batch={B}/GPU {C}x{H}x{W} bf16 (fp32 accumulate, "
                                "BN stats, params, grads) train step " if bf16 else
                                f"configs[1]: batch={B}/GPU {C}x{H}x{W} fp32 train step ")
                               + "(fwd + 0.9*L1" + (" + 0.1*VGG19 perceptual (random-init weights)"
                                                   if args.vgg else "")
                               + " + bwd + RCCL grad all-reduce + clip + AdamW)",
                   "global_batch": world * B, "in_ch": C, "res": [H, W],
                   "parallelism": f"dp{world}"},
        "data_parallel": bool(dp),
        "model_tflops_per_s": round(step_flops * args.steps / elapsed / 1e12 / world, 2),
        "world_size": dist.get_world_size() if dist.is_initialized() else 1,
        "backend": dist.get_backend() if dist.is_initialized() else None,
        "stage_cols": STAGE_COLS,
        "stages": stage_table(work, times, pipe_mult, peak, measured),
        "stage_pmc_source": measured_src,
        "roofline": roof,
        "step_execution": ("one hipGraph replay per step (nsm_amd.GraphedTrainStep)"
                           if head_graph and graphed is not None else
                           "eager, back to back (an unchanged main.py loop; the per-rank step "
                           "of data parallelism), weight gradients on the side stream"),
        "stage_execution": "eager attribution steps after the timed ones, weight gradients on "
                           "the main stream (NSM_WGRAD_STREAM=0: the configuration of the "
                           "stage PMC), HIP events per stage",
    }
    if side_elapsed is not None:
        side = {"value": round(world * B * side_steps / side_elapsed, 3),
                "ms_per_step": round(side_elapsed / side_steps * 1e3, 3),
                "steps": side_steps}
        side["headline_choice"] = ("NSM_BENCH_STEP=%s: %s" % (
            mode, "the faster of the two executions, each timed over K steps" if mode == "auto"
            else "fixed"))
        if head_graph:
            side["what"] = ("the same step run eagerly (an unchanged main.py loop; the per-rank "
                            "step of data parallelism), back to back, weight gradients on the "
                            "side stream")
            res["eager"] = side
        else:
            side["what"] = ("the same step replayed from one hipGraph (nsm_amd.GraphedTrainStep), "
                            "timed after the eager steps")
            res["graph"] = side
    if dp:
        res["dp"] = {"bn_broadcast_ms": round(dp_ms["dp.bn_broadcast"], 4),
                     "allreduce_wait_ms": round(dp_ms["dp.allreduce_wait"], 4),
                     "grad_bytes": 4 * sum(p.numel() for p in model.parameters()),
                     "note": "HIP-event time the compute stream spends in the rank-0 BN "
                             "buffer broadcast at each forward and waiting for the overlapped "
                             "gradient all-reduce after the backward"}
    if vgg_evs:
        vfl = 2 * B * vgg_fwd_flops(H, W)
        vms = mean_ms(vgg_evs)
        res["vgg_perceptual"] = {"ms": round(vms, 3), "direct_equiv_gflop": round(vfl / 1e9, 1),
                                 "tflops": round(vfl / (vms * 1e-3) / 1e12, 2),
                                 "share_of_step": round(vms / (elapsed / args.steps * 1e3), 3)}
        if vgg30:
            res["vgg_perceptual"]["roofline"] = vgg_roofline(
                B, H, W, mean_ms(vgg30), vgg30_gemm, len(vgg30),
                getattr(getattr(crit, "vgg_loss", None), "f16x2", False))
    return res


def run_infer(args):
    """configs[4]: 1x7x1080x1920 eval forward, hipGraph-captured (replicas only
    for N > 1: frames are independent, no collective); configs[0] at 256x256."""
    world, rank, dev = init_dist(args)
    res = infer_measure(args, world, rank, dev)
    H, W = (1080, 1920) if args.workload == "infer1080" else (256, 256)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.in_ch, H, W, frames=1, reps=3, train=False)
    if rank == 0:
        emit(res, args)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def infer_measure(args, world, rank, dev):
    import nsm_amd
    from nsm_amd import ops as nops
    from nsm_amd.unet import WINOGRAD_MIN_CHANNELS, wino_tile

    torch.manual_seed(1234 + rank)
    B, C = args.batch, args.in_ch
    H, W = (1080, 1920) if args.workload == "infer1080" else (256, 256)
    bf16 = args.dtype in ("bf16", "f16")   # the 16-bit storage paths
    f16 = args.dtype == "f16"
    model = nsm_amd.Unet(in_ch=C, dropout_rate=0.2).to(dev).eval()
    if bf16:
        model.set_compute_dtype(torch.float16 if f16 else torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(rank)
    x = torch.randn(B, C, H, W, device=dev, generator=g)
    graphed = nsm_amd.GraphedUnet(model, x)
    for _ in range(args.warmup):
        graphed.replay()
    torch.cuda.synchronize()
    elapsed = timed(graphed.replay, args.steps, world, dev)

    # kernel/stage timing from eager forwards of the same shape (HIP events
    # cannot be read back from inside a replayed graph)
    probe_tag = "conv6.conv.0.fwd"
    nops.PROBES[probe_tag] = []
    nops.PROBES[probe_tag + ".gemm"] = []
    for st in STAGES:
        nops.PROBES[st + ".fwd"] = []
    with torch.no_grad():
        for _ in range(args.steps):
            model(x)
    torch.cuda.synchronize()
    evs = nops.PROBES.pop(probe_tag)
    gevs = nops.PROBES.pop(probe_tag + ".gemm", [])
    times = {st: mean_ms(nops.PROBES.pop(st + ".fwd")) for st in STAGES}
    pipe_mult, peak = pipe_products(bf16)
    if bf16:
        from nsm_amd.prep import BF16_WINO, BF16_WINO_EVAL, BF16_WINO_MIN
        wino = BF16_WINO and BF16_WINO_EVAL and not f16   # bf16 eval: F(4x4) at >= 512 channels
        work = stage_work(C, H, W, B, bytes_per=2, wino_min=BF16_WINO_MIN if wino else 1 << 30,
                          passes=1)
        roof = (wino_f16_roofline(B, H, W, mean_ms(evs), mean_ms(gevs), len(evs)) if wino and gevs
                else direct_roofline(B, H, W, mean_ms(evs), len(evs), f16))
    else:
        work = stage_work(C, H, W, B, wino_min=WINOGRAD_MIN_CHANNELS, tile=wino_tile, passes=1)
        roof = dominant_roofline(B, H, W, mean_ms(evs), mean_ms(gevs), len(evs), wino_tile(1024, H // 8, W // 8))
    roof.update({"traffic": None, "traffic_source": None})
    frames = world * B * args.steps
    cfg = "configs[4]" if args.workload == "infer1080" else "configs[0]"
    res = {
        "metric": f"frames/sec {C}x{H}x{W} U-Net inference (eval fwd, hipGraph)",
        "value": round(frames / elapsed, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype if bf16 else "f32",
        "data": "synthetic (x~N(0,1)), random-init weights, eval-mode BN (running stats)",
        "config": {"workload": f"{cfg}: batch={B}/GPU {C}x{H}x{W} {args.dtype} eval forward, "
                               "one hipGraph replay per step",
                   "global_batch": world * B, "in_ch": C, "res": [H, W],
                   "parallelism": f"replicas{world}"},
        "model_tflops_per_s": round(unet_fwd_flops(C, H, W) * frames / elapsed / 1e12 / world, 2),
        "stage_cols": STAGE_COLS,
        "stages": stage_table(work, times, pipe_mult, peak),
        "roofline": roof,
    }
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, args):
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _dispatch(args)


def _dispatch(args):
    if args.dry_run:
        run_dry(args)
    elif args.workload == "train":
        run_train(args)
    else:
        run_infer(args)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (train 8, infer 1)")
    ap.add_argument("--in-ch", type=int, default=7)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--workload", choices=["train", "infer1080", "infer256"], default="train")
    ap.add_argument("--no-secondary", action="store_true",
                    help="train, N=1: skip the other configs measured after the headline one")
    ap.add_argument("--dtype", choices=["f32", "bf16", "f16"], default="f32",
                    help="bf16: configs[2] (use --batch 64); f16: the reference's fp16-autocast "
                         "mode (train only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--vgg", action="store_true",
                    help="train: include CustomLoss's VGG19 perceptual term (customLoss.py:7-90)")
    ap.add_argument("--detail", default=None,
                    help="also write the full record (all stage rows of every config) to this file")
    ap.add_argument("--force-dp", action="store_true",
                    help="N=1: run the data-parallel step (BN broadcast, bucketed all-reduce) "
                         "over a world-size-1 RCCL group, captured and eager")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo launcher check with a stand-in step (no GPU, not a measurement)")
    args = ap.parse_args()
    args.batch = args.batch or (8 if args.workload == "train" else 1)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no torchrun: one worker process per GPU, spawned before anything
        # touches the GPU in this process
        import torch.multiprocessing as mp
        mp.start_processes(_worker, args=(args.gpus, _free_port(), args), nprocs=args.gpus,
                           start_method="spawn")
        return
    _dispatch(args)


if __name__ == "__main__":
    main()
