#!/bin/bash
# Regenerate the profiles committed under profiles/<round>/ on a 1-GPU MI355X box:
#   gpurun -- bash tools/run_profiles.sh r01
# 1) kernel trace + stats of the default bench (B=8, 7x512x512, fp32);
# 2) two separate PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass)
#    with kernel trace only, summarised by tools/pmc_traffic.py for the
#    dominant kernel (Winograd batched GEMM of conv6.conv.0).
set -euo pipefail
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT" "profiles/$R"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_write.log" 2>&1
f() { find "$OUT/$1" -name "$2" -print -quit; }
cp "$(f trace run_kernel_stats.csv)" "profiles/$R/kernel_stats_bench_b8_f32.csv"
mkdir -p "$OUT/fetch_csv" "$OUT/write_csv"
cp "$(f fetch run_counter_collection.csv)" "$OUT/fetch_csv/run_counter_collection.csv"
cp "$(f write run_counter_collection.csv)" "$OUT/write_csv/run_counter_collection.csv"
python3 tools/pmc_traffic.py "$OUT/fetch_csv" "$OUT/write_csv" "profiles/$R/traffic_wino_gemm_conv6.json"
cp -r "profiles/$R" "$OUT/profiles_copy"
