# SQ counters of the bf16 B=64 step's direct-conv GEMMs (gemm_bf16_dma_kernel)
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc8; mkdir -p $O; rm -rf $O/raw
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "gemm_bf16_dma_kernel|gemm_h2p_kernel" --output-format csv -d $O/raw -o run -- \
  python3 bench.py --dtype bf16 --batch 64 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/bench.log 2>&1
python3 tools/pmc_disp.py "$(find $O/raw -name run_counter_collection.csv -print -quit)" "gemm" 40 > $O/disp.txt
rm -rf $O/raw
