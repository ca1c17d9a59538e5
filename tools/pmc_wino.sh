# PMC of the fp32 B=8 step's Winograd transform kernels (two passes; per
# dispatch: tools/pmc_disp.py). CFG: bench flags, PAT: kernel regex.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcw; mkdir -p $O
PAT=${PAT:-wino_}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM FETCH_SIZE"
P2="WRITE_SIZE TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf $O/raw$i
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$PAT" --output-format csv -d $O/raw$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline ${CFG:-} > $O/bench$i.log 2>&1
  python3 tools/pmc_disp.py "$(find $O/raw$i -name run_counter_collection.csv -print -quit)" "$PAT" 40 > $O/disp$i.txt
  rm -rf $O/raw$i
done
echo ok
