"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes for the dominant kernel
(conv6.conv.0 3x3 forward and its dgrad twin: the 128x128 implicit-GEMM with
a 256x8 grid of 256-thread blocks) into a traffic JSON.

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
            if r["Counter_Name"] == counter and "ConvActLoader<128, 256, false>" in r["Kernel_Name"]
            and "RowsKLoader<128, 256>" in r["Kernel_Name"] and r["Grid_Size"] == "524288"]
    return vals


f = pick(rows(sys.argv[1]), "FETCH_SIZE")
w = pick(rows(sys.argv[2]), "WRITE_SIZE")
fetch_kb = sum(f) / len(f)
write_kb = sum(w) / len(w)
out = {"kernel": "gemm_f32_kernel<128,128,2,2,ConvActLoader<128,256,false>,RowsKLoader<128,256>,EpiStore> "
                  "grid 256x8 (conv6.conv.0 fwd + conv6.conv.0 dgrad, B=8)",
       "launches_sampled": len(f), "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
       "fetch_bytes_corrected": fetch_kb * 1024 * 2, "write_bytes": write_kb * 1024,
       "traffic_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
       "algorithmic_bytes_per_launch": (2 * 8 * 64 * 64 * 1024 + 9 * 1024 * 1024) * 4,
       "note": "FETCH_SIZE doubled per the gfx950 calibration (16-B/lane loads); includes "
               "Infinity-Cache hits, which the counter does not exclude"}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
