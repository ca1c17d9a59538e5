# The captured-DP and graph-step tests first, then the whole -m gpu suite,
# then the --force-dp bench line (world-size-1 RCCL group, captured vs eager)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_graph_step.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/t_dpgraph.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_dpgraph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/t_r06.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_r06.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dtype bf16 --batch 64 --steps 20 --no-secondary --no-cpu-baseline --force-dp > gpurun_out/b_forcedp.log 2>&1
