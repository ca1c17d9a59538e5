"""Per-launch duration of the dominant convolution from a rocprofv3
kernel_trace.csv, to cross-check bench.py's HIP-event `roofline.avg_launch_ms`.

usage: python tools/conv6_trace.py {f32|bf16} TRACE_CSV OUT_JSON
  f32 : conv6.conv.0 fwd (+ dgrad twin) = wino_input + Winograd GEMM
        (gemm_f32_kernel grid 16x8x36 blocks) + wino_output, consecutive
        dispatches; reports each kernel's mean and the span first-start ..
        last-end (what a HIP event pair around the three launches measures)
  bf16: the LDS-DMA implicit GEMM of conv6.conv.0 (grid 4x1024 blocks of 512)
"""
import csv
import json
import statistics
import sys


def grid_blocks(r):
    return (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
            int(r["Grid_Size_Y"]) // int(r["Workgroup_Size_Y"]),
            int(r["Grid_Size_Z"]) // int(r["Workgroup_Size_Z"]))


# conv6.conv.0's Winograd GEMM at B=8, 64x64, 1024 channels: F(6x6) (the
# default there) grid 8x8x64 blocks, F(4x4) 16x8x36
CONV6_GRIDS = ((8, 8, 64), (16, 8, 36))
H2_GRIDS = ((4, 4, 64), (256, 1, 1))   # gemm_h2{,q}_kernel<256, 256>; persistent gemm_h2p_kernel
KINDS = {
    "f32": (lambda r: ((any(k in r["Kernel_Name"] for k in ("gemm_f32_kernel", "gemm_f32s_kernel",
                                                          "gemm_f32h_kernel"))
                        and r["Kernel_Name"].count("RowsKLoader<128, 256>") == 2
                        and grid_blocks(r) in CONV6_GRIDS)
                       or (any(k in r["Kernel_Name"] for k in ("gemm_h2_kernel<256, 256",
                                                               "gemm_h2q_kernel<256, 256",
                                                               "gemm_h2p_kernel<256, 256"))
                           and r["Kernel_Name"].count("H2RowsDma<256, 8") >= 2
                           and grid_blocks(r) in H2_GRIDS)), True),
    "bf16": (lambda r: "gemm_bf16_dma_kernel<256, 256" in r["Kernel_Name"]
             and "ConvActDma" in r["Kernel_Name"] and grid_blocks(r)[:2] in ((4, 1024), (1024, 4)),
             False),
    # the bf16 path's F(4x4) forward (round 4): input transform + the
    # single-plane persistent GEMM + output transform
    "bf16_wino": (lambda r: ("gemm_h2p_kernel<256, 256" in r["Kernel_Name"]
                             or "gemm_h2q_kernel<256, 256" in r["Kernel_Name"])
                  and ", true>" in r["Kernel_Name"], True),
}

kind, path, outp = sys.argv[1], sys.argv[2], sys.argv[3]
match, triple = KINDS[kind]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a run with NSM_STAGE_MARKS=1: keep conv6's forward launches only (its
# input-gradient twins have the same kernel and grid), markers dropped
marked = any("stage_mark_kernel" in r["Kernel_Name"] for r in rows)
if marked:
    keep, cur = [], 0
    for r in rows:
        if "stage_mark_kernel" in r["Kernel_Name"]:
            cur = int(r["Grid_Size_X"]) // 64 - 1
        else:
            r["_stage"] = cur
            keep.append(r)
    rows = keep
    CONV6_FWD = 9   # nsm_amd/ops.py STAGE_CODES["conv6.fwd"]
    _m = match
    match = lambda r: r["_stage"] == CONV6_FWD and _m(r)  # noqa: E731
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
spans, parts = [], [[], [], []]
for i, r in enumerate(rows):
    if not match(r):
        continue
    if triple:
        if i == 0 or i + 1 >= len(rows):
            continue
        a, c = rows[i - 1], rows[i + 1]
        spans.append((int(c["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e6)
        for k, x in enumerate((a, r, c)):
            parts[k].append(dur(x))
    else:
        spans.append(dur(r))
if not triple and len(spans) > 2 and not marked:
    # the same kernel/grid also runs conv6.conv.4's input gradient (K = 512):
    # keep the cluster above the largest gap in the sorted durations (K = 9216)
    srt = sorted(spans)
    gap = max(range(1, len(srt)), key=lambda i: srt[i] - srt[i - 1])
    spans = srt[gap:]
out = {"kind": kind, "launches": len(spans), "forward_only": marked,
       "span_ms_mean": statistics.mean(spans),
       "span_ms_median": statistics.median(spans)}
if triple:
    out.update({"wino_input_ms": statistics.mean(parts[0]), "gemm_ms": statistics.mean(parts[1]),
                "wino_output_ms": statistics.mean(parts[2]),
                "sum_of_kernels_ms": statistics.mean(parts[0]) + statistics.mean(parts[1])
                + statistics.mean(parts[2])})
json.dump(out, open(outp, "w"), indent=1)
print(json.dumps(out, indent=1))
