# Three PMC passes over a short fp32 bench run (per-kernel SQ breakdown, HBM fetch, HBM write)
set -euo pipefail
OUT=gpurun_out/pmc_step
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary ${CFG:-}"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/r1" -o run -- $B > "$OUT/b1.log" 2>&1
cp "$(find "$OUT/r1" -name run_counter_collection.csv -print -quit)" "$OUT/sq.csv"; rm -rf "$OUT/r1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/r2" -o run -- $B > "$OUT/b2.log" 2>&1
cp "$(find "$OUT/r2" -name run_counter_collection.csv -print -quit)" "$OUT/fetch.csv"; rm -rf "$OUT/r2"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/r3" -o run -- $B > "$OUT/b3.log" 2>&1
cp "$(find "$OUT/r3" -name run_counter_collection.csv -print -quit)" "$OUT/write.csv"; rm -rf "$OUT/r3"
