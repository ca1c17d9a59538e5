# LDS / MFMA counters of the bf16 B=64 step's direct-conv GEMMs (two passes;
# per dispatch: tools/pmc_disp.py)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcg; mkdir -p $O
PAT=${PAT:-gemm_bf16_dma_kernel}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_WAIT_ANY"
P2="SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE TA_TA_BUSY_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1)); rm -rf $O/raw$i
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$PAT" --output-format csv -d $O/raw$i -o run -- \
    python3 bench.py --dtype bf16 --batch 64 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/bench$i.log 2>&1
  python3 tools/pmc_disp.py "$(find $O/raw$i -name run_counter_collection.csv -print -quit)" "$PAT" 60 > $O/disp$i.txt
  rm -rf $O/raw$i
done
echo ok
