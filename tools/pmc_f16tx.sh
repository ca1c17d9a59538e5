# VALU / wait counters of the bf16 B=64 step's F(4x4) transforms (one pass)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/pmct; mkdir -p $O; rm -rf $O/raw
PAT=${PAT:-wino_}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR \
  --kernel-include-regex "$PAT" --output-format csv -d $O/raw -o run -- \
  python3 bench.py --dtype bf16 --batch 64 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/bench.log 2>&1
python3 tools/pmc_disp.py "$(find $O/raw -name run_counter_collection.csv -print -quit)" "$PAT" 30 > $O/disp.txt
rm -rf $O/raw
echo ok
