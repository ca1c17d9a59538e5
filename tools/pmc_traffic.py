"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes for the dominant kernel
(the Winograd F(4x4,3x3) batched GEMM of conv6.conv.0 forward and its dgrad
twin: gemm_f32_kernel<128,128> RowsK x RowsK, grid 16x8x36 of 256-thread
blocks at B=8, T = 8*16*16 tiles) into a traffic JSON.

Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads exactly half
the bytes of a 16-B/lane coalesced stream on gfx950 -> x2; WRITE_SIZE (KB) is
exact for 16-B/lane stores; our epilogue stores are 4-B/lane (uncalibrated),
so WRITE_SIZE is reported as measured and compared with the known output size.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import json
import sys


def rows(d):
    return list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))


def pick(rs, counter):
    vals = [float(r["Counter_Value"]) for r in rs
            if r["Counter_Name"] == counter
            and r["Kernel_Name"].count("RowsKLoader<128, 256>") == 2
            and "EpiStore" in r["Kernel_Name"] and r["Grid_Size"] == str(16 * 8 * 36 * 256)]
    return vals


f = pick(rows(sys.argv[1]), "FETCH_SIZE")
w = pick(rows(sys.argv[2]), "WRITE_SIZE")
fetch_kb = sum(f) / len(f)
write_kb = sum(w) / len(w)
T, NB = 8 * 16 * 16, 36
out = {"kernel": "gemm_f32_kernel<128,128,2,2,RowsKLoader<128,256>,RowsKLoader<128,256>,EpiStore> "
                  "grid 16x8x36 (Winograd F(4x4) GEMM of conv6.conv.0 fwd + dgrad, B=8)",
       "launches_sampled": len(f), "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
       "fetch_bytes_corrected": fetch_kb * 1024 * 2, "write_bytes": write_kb * 1024,
       "traffic_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
       "algorithmic_bytes_per_launch": NB * (2 * T * 1024 + 1024 * 1024) * 4,
       "note": "FETCH_SIZE doubled per the gfx950 calibration (16-B/lane loads); includes "
               "Infinity-Cache hits, which the counter does not exclude"}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
