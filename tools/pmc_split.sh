# PMC pass over the split-GEMM microbench (mode 1, GEMM form, conv6/conv7 shapes)
set -euo pipefail
OUT=gpurun_out/pmc_split
mkdir -p "$OUT"
export TMPDIR=/tmp
MODES=1 ONLY=gemm SHAPES=0,2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/raw" -o run -- python3 tools/bench_split.py > "$OUT/bench.log" 2>&1
cp "$(find "$OUT/raw" -name run_counter_collection.csv -print -quit)" "$OUT/counters.csv"
rm -rf "$OUT/raw"
MODES=1 ONLY=gemm SHAPES=0,2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU \
  --output-format csv -d "$OUT/raw2" -o run -- python3 tools/bench_split.py > "$OUT/bench2.log" 2>&1
cp "$(find "$OUT/raw2" -name run_counter_collection.csv -print -quit)" "$OUT/counters2.csv"
rm -rf "$OUT/raw2"
