#!/bin/bash
# Regenerate the profiles committed under profiles/<round>/ on a 1-GPU MI355X box:
#   gpurun -- bash tools/run_profiles.sh r02
# For the default bench (B=8, 7x512x512, fp32) and configs[2] (B=64 bf16):
# 1) kernel trace + stats;
# 2) two separate PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass)
#    with kernel trace only, summarised by tools/pmc_traffic.py for the
#    dominant kernel of each (bench.py reads the JSON into roofline.traffic).
set -euo pipefail
R=${1:-r02}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT" "profiles/$R"
export TMPDIR=/tmp
f() { find "$OUT/$1" -name "$2" -print -quit; }
run() {  # tag, extra bench args...
  local tag=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$tag" -o run -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary "$@" > "$OUT/bench_trace_$tag.log" 2>&1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$tag" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary "$@" > "$OUT/bench_fetch_$tag.log" 2>&1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$tag" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary "$@" > "$OUT/bench_write_$tag.log" 2>&1
  mkdir -p "$OUT/fetch_csv_$tag" "$OUT/write_csv_$tag"
  cp "$(f fetch_$tag run_counter_collection.csv)" "$OUT/fetch_csv_$tag/run_counter_collection.csv"
  cp "$(f write_$tag run_counter_collection.csv)" "$OUT/write_csv_$tag/run_counter_collection.csv"
}
run f32
cp "$(f trace_f32 run_kernel_stats.csv)" "profiles/$R/kernel_stats_bench_b8_f32.csv"
python3 tools/conv6_trace.py f32 "$(f trace_f32 run_kernel_trace.csv)" "profiles/$R/trace_conv6_fwd_f32.json"
python3 tools/pmc_traffic.py f32 "$OUT/fetch_csv_f32" "$OUT/write_csv_f32" \
    "profiles/$R/traffic_conv6_fwd_f32.json"
run bf16 --dtype bf16 --batch 64
cp "$(f trace_bf16 run_kernel_stats.csv)" "profiles/$R/kernel_stats_bench_b64_bf16.csv"
python3 tools/conv6_trace.py bf16 "$(f trace_bf16 run_kernel_trace.csv)" "profiles/$R/trace_conv6_fwd_bf16.json"
python3 tools/pmc_traffic.py bf16 "$OUT/fetch_csv_bf16" "$OUT/write_csv_bf16" \
    "profiles/$R/traffic_conv6_fwd_bf16.json"
cp -r "profiles/$R" "$OUT/profiles_copy"
# one train step's launches in order, with per-family totals
python3 tools/step_timeline.py "$(f trace_f32 run_kernel_trace.csv)" > "profiles/$R/step_timeline_b8_f32.txt"
python3 tools/step_timeline.py "$(f trace_bf16 run_kernel_trace.csv)" > "profiles/$R/step_timeline_b64_bf16.txt"
cp profiles/$R/step_timeline_* "$OUT/profiles_copy/"
