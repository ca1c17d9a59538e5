#!/bin/bash
# Regenerate the profiles committed under profiles/<round>/ on a 1-GPU MI355X box:
#   gpurun -- bash tools/run_profiles.sh r03 [f32|bf16|both]
# For the default bench (configs[1]: B=8, 7x512x512, fp32) and configs[2]
# (B=64 bf16):
# 1) kernel trace + stats of the plain bench (step timeline, per-kernel stats,
#    conv6.conv.0 forward durations);
# 2) the same bench with NSM_STAGE_MARKS=1 (stage marker launches around every
#    encoder/decoder stage): one kernel-trace run and four PMC passes, each in
#    its own run (rocprofv3 does not split counters over passes):
#      TCC_EA0_RDREQ_{,32B_,64B_,128B_}sum | FETCH_SIZE | WRITE_SIZE |
#      SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16/_F16/_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
#    summarised per stage by tools/stage_pmc.py and, for the dominant kernel,
#    by tools/pmc_traffic.py (bench.py reads both JSONs).
set -euo pipefail
R=${1:-r03}
WHICH=${2:-both}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT" "profiles/$R"
export TMPDIR=/tmp
f() { find "$OUT/$1" -name "$2" -print -quit; }
BENCH="python3 bench.py --no-cpu-baseline --no-secondary"
pmc() {  # tag name counters... (marked run, kernel trace only besides the counters)
  local tag=$1 name=$2; shift 2
  NSM_STAGE_MARKS=1 timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/${name}_$tag" -o run -- \
      $BENCH --steps 3 --warmup 1 $ARGS > "$OUT/bench_${name}_$tag.log" 2>&1
  cp "$(f ${name}_$tag run_counter_collection.csv)" "$OUT/${name}_$tag.csv"
  rm -rf "$OUT/${name}_$tag"
}
run() {  # tag
  local tag=$1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$tag" -o run -- \
      $BENCH --steps 5 --warmup 2 $ARGS > "$OUT/bench_trace_$tag.log" 2>&1
  NSM_STAGE_MARKS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/mtrace_$tag" -o run -- \
      $BENCH --steps 5 --warmup 2 $ARGS > "$OUT/bench_mtrace_$tag.log" 2>&1
  cp "$(f mtrace_$tag run_kernel_trace.csv)" "$OUT/mtrace_$tag.csv"
  pmc $tag rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  pmc $tag fetch FETCH_SIZE
  pmc $tag write WRITE_SIZE
  pmc $tag sq SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  python3 tools/stage_pmc.py "profiles/$R/stage_pmc_$tag.json" "$OUT/mtrace_$tag.csv" \
      "$OUT/rdreq_$tag.csv" "$OUT/fetch_$tag.csv" "$OUT/write_$tag.csv" "$OUT/sq_$tag.csv" > "$OUT/stage_$tag.txt"
  python3 tools/step_timeline.py "$(f trace_$tag run_kernel_trace.csv)" > "profiles/$R/step_timeline_$tag.txt"
  cp "$(f trace_$tag run_kernel_stats.csv)" "profiles/$R/kernel_stats_bench_$tag.csv"
}
if [ "$WHICH" != bf16 ]; then
  ARGS=""
  run b8_f32
  python3 tools/conv6_trace.py f32 "$OUT/mtrace_b8_f32.csv" "profiles/$R/trace_conv6_fwd_f32.json"
  python3 tools/pmc_traffic.py f32_gemm "profiles/$R/traffic_conv6_fwd_gemm_f32.json" \
      "$OUT/rdreq_b8_f32.csv" "$OUT/fetch_b8_f32.csv" "$OUT/write_b8_f32.csv"
  python3 tools/pmc_traffic.py f32 "profiles/$R/traffic_conv6_fwd_f32.json" \
      "$OUT/rdreq_b8_f32.csv" "$OUT/fetch_b8_f32.csv" "$OUT/write_b8_f32.csv"
fi
if [ "$WHICH" != f32 ]; then
  ARGS="--dtype bf16 --batch 64"
  run b64_bf16
  python3 tools/conv6_trace.py bf16_wino "$OUT/mtrace_b64_bf16.csv" "profiles/$R/trace_conv6_fwd_bf16.json"
  python3 tools/pmc_traffic.py bf16_wino "profiles/$R/traffic_conv6_fwd_bf16.json" \
      "$OUT/rdreq_b64_bf16.csv" "$OUT/fetch_b64_bf16.csv" "$OUT/write_b64_bf16.csv"
  python3 tools/pmc_traffic.py bf16_wino_gemm "profiles/$R/traffic_conv6_fwd_gemm_bf16.json" \
      "$OUT/rdreq_b64_bf16.csv" "$OUT/fetch_b64_bf16.csv" "$OUT/write_b64_bf16.csv"
fi
mkdir -p "$OUT/profiles_copy"
cp -r profiles/$R/* "$OUT/profiles_copy/"
