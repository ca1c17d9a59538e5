# fabric-side read traffic and L2 hit rate of the h2 Winograd GEMM microbench
set -euo pipefail
OUT=gpurun_out/pmc_h2
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name counters...
  local n=$1; shift
  SHAPES=${SHAPES:-0} REPS=10 timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv \
    -d "$OUT/raw_$n" -o run -- python3 tools/bench_h2.py > "$OUT/bench_$n.log" 2>&1
  cp "$(find "$OUT/raw_$n" -name run_counter_collection.csv -print -quit)" "$OUT/counters_$n.csv"
  rm -rf "$OUT/raw_$n"
}
pass c TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass d TCC_HIT_sum TCC_MISS_sum
pass e WRITE_SIZE
python3 tools/pmc_summary.py "$OUT"/counters_[cde].csv | grep -A12 "gemm_h2\|gemm_f32h" > "$OUT/summary_b.txt"
