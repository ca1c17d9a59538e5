#!/usr/bin/env python3
"""Per-stage hardware counters of one train step, from rocprofv3 runs of
bench.py with NSM_STAGE_MARKS=1 (every encoder/decoder stage of
Unetmodel.py:104-148 bracketed by nsm_stage_mark launches whose grid encodes
the stage; see nsm_amd/ops.py STAGE_CODES).

usage: python tools/stage_pmc.py OUT_JSON TRACE_CSV PMC_CSV [PMC_CSV ...]
  TRACE_CSV : kernel_trace.csv of a marked run (kernel time per stage)
  PMC_CSV   : counter_collection.csv of marked runs, one pass each
              (FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE ...)

Per stage (fwd, bwd and both) and per step (the mean over the steps after the
first, every dispatch between a stage's start and end markers; dispatches
outside every stage go to "other": input prep, weight prep, loss, tail):
  kernel_ms      sum of kernel durations (kernel trace, not profiled)
  read_bytes     L2 -> fabric read requests by size: 32 x TCC_EA0_RDREQ_32B +
                 64 x TCC_EA0_RDREQ_64B + 128 x TCC_EA0_RDREQ_128B (requests of
                 no listed size counted at 64 B); includes Infinity-Cache hits
  fetch_bytes_x2 FETCH_SIZE x 1024 x 2, the MI355X_MICROARCH.md §HBM
                 correction (FETCH_SIZE reads half the bytes of a 16-B/lane
                 stream on gfx950) — a cross-check of read_bytes
  write_bytes    WRITE_SIZE x 1024
  hbm_bytes      read_bytes (else fetch_bytes_x2) + write_bytes
  hbm_gbs        hbm_bytes / kernel_ms
  mfma_busy      SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8):
                 the fraction of SIMD-cycles the matrix pipe was busy, at the
                 clock the chip held — over the stage's dispatches of >= 0.3 ms
                 only (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE / 8 / time reads
                 high on shorter dispatches); absent when it has none
  bf16_mfma_flops, f32_mfma_flops
                 512 x SQ_INSTS_VALU_MFMA_MOPS_{BF16+F16, F32}: the matrix-core
                 work actually issued, per pipe (16-bit: bf16 and f16 MFMAs run
                 at the same rate; the fp32 GEMMs run there by the f16x2 split,
                 3 products per fp32 product, or the bf16 split, 6)
  mfma_pipe_frac bf16 work / kernel_ms / 2516.6 TFLOP/s + f32 work / kernel_ms
                 / 157.3 TFLOP/s: the fraction of the dense peak of the pipe
                 that ran it (at the 2.4 GHz peak clock)
  eff_clock_ghz  GRBM_GUI_ACTIVE / 8 / profiled kernel time, same dispatches
The output carries `stamp` = {libnsm_sha256 of the library the runs loaded,
git_head (env GIT_HEAD, the box has no .git)}: bench.py uses the measured
columns only when the stamp's library is the one it loaded.
"""
import hashlib
import os
import collections
import csv
import json
import sys


STAGE_NAMES = ["conv2", "conv3", "conv4", "conv5", "conv6", "conv7", "conv8", "conv9", "head"]
CODES = {1 + 2 * i + j: f"{n}.{d}" for i, n in enumerate(STAGE_NAMES)
         for j, d in enumerate(("fwd", "bwd"))}
CODES.update({40: "dp.bn_broadcast", 41: "dp.allreduce_wait"})
FIRST = 1   # conv2.fwd: a new step
N_SIMD = 256 * 4
LONG_MS = 0.3   # dispatches shorter than this read a high clock (MI355X_MICROARCH.md, DVFS)
BF16_PEAK = 2516.6e12   # dense bf16 MFMA: 1024 SIMD x 1024 FLOP/clk x 2.4 GHz
F32_PEAK = 157.3e12
SUMS = ("kernel_ms", "read_bytes", "fetch_bytes_x2", "write_bytes", "hbm_bytes",
        "mfma_busy_cycles", "bf16_mfma_flops", "f32_mfma_flops", "grbm", "prof_ms")


def is_mark(name):
    return "stage_mark_kernel" in name


def attribute(disp):
    """disp: [(name, grid_threads, payload)] in dispatch order ->
    {step: {stage: [payload, ...]}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    step, cur = -1, "other"
    for name, grid, pay in disp:
        if is_mark(name):
            code = grid // 64 - 1
            if code == 0:
                cur = "other"
            else:
                cur = CODES.get(code, f"code{code}")
                if code == FIRST:
                    step += 1
            continue
        if step >= 0:
            out[step][cur].append(pay)
    return out


def mean_steps(per_step, fn):
    """Mean over steps 1..n-1 of fn(list of payloads) per stage."""
    steps = sorted(per_step)[1:] or sorted(per_step)
    acc = collections.defaultdict(float)
    for s in steps:
        for st, pays in per_step[s].items():
            acc[st] += fn(pays)
    return {k: v / len(steps) for k, v in acc.items()}, len(steps)


def load_trace(path):
    rows = list(csv.DictReader(open(path)))
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else "Start_Timestamp"
    rows.sort(key=lambda r: int(r[key]))
    return [(r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1)
             * int(r.get("Grid_Size_Z", 1) or 1),
             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in rows]


def load_pmc(path):
    """{dispatch: (name, grid, {counter: value}, duration_ms)} in dispatch order."""
    d = {}
    for r in csv.DictReader(open(path)):
        did = int(r.get("Dispatch_Id") or r["Correlation_Id"])
        ent = d.setdefault(did, [r["Kernel_Name"], int(r["Grid_Size"]), {},
                                 (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6])
        ent[2][r["Counter_Name"]] = ent[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(n, g, (c, t)) for _, (n, g, c, t) in sorted(d.items())]


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pcss-unet_amd", "nsm_amd", "libnsm.so")


def lib_sha256(path=LIB):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def stamp():
    """What a profile summary was measured on: the library's sha256 and the git
    head (env GIT_HEAD: the GPU box's copy of the tree has no .git)."""
    return {"libnsm_sha256": lib_sha256(), "git_head": os.environ.get("GIT_HEAD")}


def main():
    out_path, trace, pmcs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = collections.defaultdict(dict)
    per, nsteps = mean_steps(attribute(load_trace(trace)), lambda ps: sum(ps))
    for st, v in per.items():
        res[st]["kernel_ms"] = v
    counters = set()
    prof_ms = {}
    for p in pmcs:
        disp = load_pmc(p)
        names = {k for _, _, (c, _) in disp for k in c}
        counters |= names
        att = attribute(disp)
        for cname in names:
            m, _ = mean_steps(att, lambda ps, c=cname: sum(x[0].get(c, 0.0) for x in ps))
            for st, v in m.items():
                res[st][cname] = v
        if "GRBM_GUI_ACTIVE" in names:
            # busy cycles / clock over the dispatches of >= LONG_MS only
            for cname in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
                if cname in names:
                    m, _ = mean_steps(att, lambda ps, c=cname: sum(x[0].get(c, 0.0) for x in ps
                                                                   if x[1] >= LONG_MS))
                    for st, v in m.items():
                        res[st][cname + "_long"] = v
            m, _ = mean_steps(att, lambda ps: sum(x[1] for x in ps if x[1] >= LONG_MS))
            prof_ms.update(m)
    stages = {}
    for st, r in res.items():
        row = {"kernel_ms": r.get("kernel_ms", 0.0)}
        n32, n64, n128 = (r.get(f"TCC_EA0_RDREQ_{k}B_sum") for k in (32, 64, 128))
        if n128 is not None and n64 is not None and n32 is not None:
            rest = max(0.0, r.get("TCC_EA0_RDREQ_sum", 0.0) - n32 - n64 - n128)
            row["read_bytes"] = 32 * n32 + 64 * (n64 + rest) + 128 * n128
        if r.get("FETCH_SIZE") is not None:
            row["fetch_bytes_x2"] = r["FETCH_SIZE"] * 1024 * 2
        if r.get("WRITE_SIZE") is not None:
            row["write_bytes"] = r["WRITE_SIZE"] * 1024
        rd = row.get("read_bytes", row.get("fetch_bytes_x2"))
        if rd is not None and "write_bytes" in row:
            row["hbm_bytes"] = rd + row["write_bytes"]
        if r.get("SQ_VALU_MFMA_BUSY_CYCLES_long") and r.get("GRBM_GUI_ACTIVE_long"):
            row["mfma_busy_cycles"] = r["SQ_VALU_MFMA_BUSY_CYCLES_long"]
            row["grbm"] = r["GRBM_GUI_ACTIVE_long"]
            row["prof_ms"] = prof_ms.get(st, 0.0)
        for k, c in (("bf16_mfma_flops", "SQ_INSTS_VALU_MFMA_MOPS_BF16"),
                     ("f16_mfma_flops", "SQ_INSTS_VALU_MFMA_MOPS_F16"),
                     ("f32_mfma_flops", "SQ_INSTS_VALU_MFMA_MOPS_F32")):
            if r.get(c) is not None:
                row[k] = 512 * r[c]
        if "f16_mfma_flops" in row:   # one 16-bit pipe: bf16 and f16 MFMAs at the same rate
            row["bf16_mfma_flops"] = row.get("bf16_mfma_flops", 0.0) + row.pop("f16_mfma_flops")
        stages[st] = row
    for n in STAGE_NAMES:   # fwd + bwd per stage
        f, b = stages.get(n + ".fwd"), stages.get(n + ".bwd")
        if f and b:
            stages[n] = {k: f[k] + b[k] for k in SUMS if k in f and k in b}
    for st, row in stages.items():
        t = row["kernel_ms"] * 1e-3
        if t > 0 and "hbm_bytes" in row:
            row["hbm_gbs"] = round(row["hbm_bytes"] / t / 1e9, 1)
        if row.get("grbm"):
            row["mfma_busy"] = round(row["mfma_busy_cycles"] / (N_SIMD * row["grbm"] / 8), 4)
            if row.get("prof_ms"):
                row["eff_clock_ghz"] = round(row["grbm"] / 8 / (row["prof_ms"] * 1e-3) / 1e9, 3)
        if t > 0 and "bf16_mfma_flops" in row:
            row["mfma_pipe_frac"] = round(row["bf16_mfma_flops"] / t / BF16_PEAK
                                          + row.get("f32_mfma_flops", 0.0) / t / F32_PEAK, 4)
            row["bf16_mfma_tflops"] = round(row["bf16_mfma_flops"] / t / 1e12, 2)
        row["kernel_ms"] = round(row["kernel_ms"], 4)
    doc = {"stamp": stamp(), "source": {"trace": trace, "pmc": pmcs}, "steps_averaged": nsteps,
           "counters": sorted(counters),
           "method": __doc__.split("Per stage", 1)[1].strip(), "stages": stages}
    json.dump(doc, open(out_path, "w"), indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items()
                          if kk in ("kernel_ms", "hbm_gbs", "mfma_busy", "mfma_pipe_frac",
                                    "eff_clock_ghz")}
                      for k, v in stages.items()}, indent=0))


if __name__ == "__main__":
    main()
