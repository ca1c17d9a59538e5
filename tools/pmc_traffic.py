"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes for one dominant kernel
into a traffic JSON (HBM bytes per launch next to the algorithmic bytes).

Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half
the bytes of a 16-B/lane coalesced stream on gfx950 -> x2 (both dominant
kernels load 16 B per lane: buffer_load_dwordx4 / buffer_load ... lds);
WRITE_SIZE (KB) is exact for 16-B/lane stores; the GEMM epilogues store 4-B
(fp32) / 2-B (bf16) per lane (uncalibrated), so WRITE_SIZE is reported as
measured next to the known output size.

usage: python tools/pmc_traffic.py {f32|bf16} FETCH_DIR WRITE_DIR OUT_JSON
  f32 : Winograd F(4x4,3x3) batched GEMM of conv6.conv.0 (fwd + dgrad twin),
        gemm_f32_kernel<128,128> RowsK x RowsK, grid 16x8x36 blocks, B=8
  bf16: LDS-DMA implicit GEMM of conv6.conv.0 fwd (+ its dgrad twin, same
        shape), gemm_bf16_dma_kernel<256,256>, grid 4x1024 blocks of 512, B=64
"""
import csv
import json
import sys

KINDS = {
    "f32": dict(
        match=lambda n: n.count("RowsKLoader<128, 256>") == 2 and "EpiStore" in n
        and "gemm_f32_kernel" in n,
        grid=16 * 8 * 36 * 256,
        alg=36 * (2 * (8 * 16 * 16) * 1024 + 1024 * 1024) * 4,
        desc="gemm_f32_kernel<128,128,2,2,RowsKLoader<128,256>,RowsKLoader<128,256>,EpiStore> "
             "grid 16x8x36 (Winograd F(4x4) GEMM of conv6.conv.0 fwd + dgrad, B=8)"),
    "bf16": dict(
        match=lambda n: "gemm_bf16_dma_kernel<256, 256" in n and "ConvActDma" in n,
        grid=4 * 1024 * 512,
        alg=(2 * 262144 * 1024 + 9 * 1024 * 1024) * 2,
        desc="gemm_bf16_dma_kernel<256,256,2,4,2,...,ConvActDma,RowsKDma,EpiStoreB> grid 4x1024 "
             "(implicit-GEMM 3x3 conv6.conv.0 fwd + dgrad, M=262144 N=1024 K=9216, B=64)"),
}


def rows(d):
    return list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))


def pick(rs, counter, k):
    return [float(r["Counter_Value"]) for r in rs
            if r["Counter_Name"] == counter and k["match"](r["Kernel_Name"])
            and r["Grid_Size"] == str(k["grid"])]


kind = sys.argv[1]
k = KINDS[kind]
f = pick(rows(sys.argv[2]), "FETCH_SIZE", k)
w = pick(rows(sys.argv[3]), "WRITE_SIZE", k)
fetch_kb = sum(f) / len(f)
write_kb = sum(w) / len(w)
out = {"kernel": k["desc"], "launches_sampled": len(f), "fetch_size_kb_raw": fetch_kb,
       "write_size_kb": write_kb, "fetch_bytes_corrected": fetch_kb * 1024 * 2,
       "write_bytes": write_kb * 1024,
       "traffic_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
       "algorithmic_bytes_per_launch": k["alg"],
       "note": "FETCH_SIZE doubled per the gfx950 calibration (16-B/lane loads); includes "
               "Infinity-Cache hits, which the counter does not exclude"}
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out, indent=1))
