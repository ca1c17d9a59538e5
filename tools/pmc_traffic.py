"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes for the dominant
convolution into a traffic JSON (HBM bytes per launch next to the
algorithmic bytes); bench.py reads it into roofline.traffic.

Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half
the bytes of a 16-B/lane coalesced stream on gfx950 -> x2 (the kernels below
load 16 B per lane: buffer_load_dwordx4 / f32x4 / buffer_load ... lds);
WRITE_SIZE (KB) is exact for 16-B/lane stores and reported as measured.

usage: python tools/pmc_traffic.py {f32|bf16} FETCH_DIR WRITE_DIR OUT_JSON
  f32 : conv6.conv.0 forward as a whole = the three consecutive dispatches
        wino_input -> Winograd batched GEMM (F(6x6,3x3): grid 8x8x64 blocks,
        F(4x4): 16x8x36; B=8) -> wino_output (the dgrad twin has the same shapes and is
        averaged in); algorithmic bytes = x + y + weights (direct conv)
  bf16: LDS-DMA implicit GEMM of conv6.conv.0 fwd (+ its dgrad twin, same
        shape), gemm_bf16_dma_kernel<256,256>, grid 4x1024 blocks of 512, B=64
"""
import csv
import json
import sys

B8_CONV6 = 8 * 64 * 64
KINDS = {
    "f32": dict(
        match=lambda n: n.count("RowsKLoader<128, 256>") == 2 and "EpiStore" in n
        and ("gemm_f32_kernel" in n or "gemm_f32s_kernel" in n),
        grid=(8 * 8 * 64 * 256, 16 * 8 * 36 * 256), triple=True,
        alg=(2 * B8_CONV6 * 1024 + 9 * 1024 * 1024 + 1024) * 4,
        desc="conv6.conv.0 fwd (+ dgrad twin), B=8: wino_input + gemm_f32_kernel<128,128,2,2,"
             "RowsKLoader<128,256>x2,EpiStore> (F(6x6): grid 8x8x64; F(4x4): 16x8x36) + "
             "wino_output"),
    "bf16": dict(
        match=lambda n: "gemm_bf16_dma_kernel<256, 256" in n and "ConvActDma" in n,
        grid=(4 * 1024 * 512,), triple=False,
        alg=(2 * 262144 * 1024 + 9 * 1024 * 1024) * 2,
        desc="gemm_bf16_dma_kernel<256,256,2,4,2,...,ConvActDma,RowsKDma,EpiStoreB> grid 4x1024 "
             "(implicit-GEMM 3x3 conv6.conv.0 fwd + dgrad, M=262144 N=1024 K=9216, B=64)"),
}


def rows(d, counter):
    out = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Counter_Name"] != counter:
            continue
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        out[did] = (r["Kernel_Name"], r["Grid_Size"], float(r["Counter_Value"]))
    return out


def per_launch(d, counter, k):
    rs = rows(d, counter)
    vals, names = [], set()
    for did, (name, grid, v) in sorted(rs.items()):
        if not (k["match"](name) and grid in {str(g) for g in k["grid"]}):
            continue
        if k["triple"]:
            if did - 1 not in rs or did + 1 not in rs:
                continue
            names.update((rs[did - 1][0][:60], rs[did + 1][0][:60]))
            v = rs[did - 1][2] + v + rs[did + 1][2]
        vals.append(v)
    return vals, sorted(names)


kind = sys.argv[1]
k = KINDS[kind]
f, nf = per_launch(sys.argv[2], "FETCH_SIZE", k)
w, nw = per_launch(sys.argv[3], "WRITE_SIZE", k)
fetch_kb = sum(f) / len(f)
write_kb = sum(w) / len(w)
out = {"kernel": k["desc"], "launches_sampled": len(f), "fetch_size_kb_raw": fetch_kb,
       "write_size_kb": write_kb, "fetch_bytes_corrected": fetch_kb * 1024 * 2,
       "write_bytes": write_kb * 1024,
       "traffic_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
       "algorithmic_bytes_per_launch": k["alg"],
       "neighbour_kernels": sorted(set(nf) | set(nw)),
       "note": "FETCH_SIZE doubled per the gfx950 calibration (16-B/lane loads); includes "
               "Infinity-Cache hits, which the counter does not exclude"}
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out, indent=1))
