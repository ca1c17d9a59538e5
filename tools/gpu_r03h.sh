# round 3: whole -m gpu suite, then the f16x2 GEMM's SQ counters
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_g.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_g.log; [ $rc -le 1 ] || exit $rc
mkdir -p gpurun_out/r03g
SHAPES=0,1 REPS=50 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r03g/sq16 -o run -- python3 tools/bench_split16.py > gpurun_out/r03g/sq16.log 2>&1 || exit $?
cp $(find gpurun_out/r03g/sq16 -name run_counter_collection.csv) gpurun_out/r03g/sq16.csv; rm -rf gpurun_out/r03g/sq16
