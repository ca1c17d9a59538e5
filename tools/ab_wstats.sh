# GPU: Winograd output-transform BN statistics: op tests, fp32 model parity,
# A/B of NSM_WINO_STATS 0 / 1 on the fp32 train step.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bn_stats or winograd or bn_train" -q --timeout 200 --timeout-method thread > gpurun_out/t_ws_ops.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_ws_ops.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_dp.py -q --timeout 300 --timeout-method thread > gpurun_out/t_ws_model.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_ws_model.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
 for m in 0 1; do
  NSM_WINO_STATS=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_ws_${m}_$i.log 2>&1 || exit 1
 done
done
