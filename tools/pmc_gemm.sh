#!/bin/bash
# One PMC pass over a short bench run (bf16 B=64 by default; CFG="" for the
# fp32 B=8 headline config): SQ cycle breakdown + MFMA busy + clock of every
# dispatch.
#   gpurun -- bash tools/pmc_gemm.sh TAG [extra bench args]
set -euo pipefail
TAG=${1:-pmc}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/raw" -o run -- python3 bench.py ${CFG---dtype bf16 --batch 64} --steps 2 \
  --warmup 1 --no-cpu-baseline --no-secondary "$@" > "$OUT/bench.log" 2>&1
cp "$(find "$OUT/raw" -name run_counter_collection.csv -print -quit)" "$OUT/counters.csv"
rm -rf "$OUT/raw"
