# PMC passes over the h2 Winograd GEMM microbench (tools/bench_h2.py, conv6 / conv7 shapes)
set -euo pipefail
OUT=gpurun_out/pmc_h2
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name counters...
  local n=$1; shift
  SHAPES=${SHAPES:-0,1} REPS=10 timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv \
    -d "$OUT/raw_$n" -o run -- python3 tools/bench_h2.py > "$OUT/bench_$n.log" 2>&1
  cp "$(find "$OUT/raw_$n" -name run_counter_collection.csv -print -quit)" "$OUT/counters_$n.csv"
  rm -rf "$OUT/raw_$n"
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
pass b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS \
  SQ_ACTIVE_INST_MISC SQ_INSTS_SALU
python3 tools/pmc_summary.py "$OUT"/counters_*.csv > "$OUT/summary.txt"
