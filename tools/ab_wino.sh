# GPU: Winograd F(6x6) op tests, model parity with every Winograd layer on F(6x6),
# then a tile 4 / 6 A/B of the fp32 bench (stage table per run).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "winograd" -q --timeout 200 --timeout-method thread > gpurun_out/t_wino_ops.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_wino_ops.log; [ $rc -le 1 ] || exit $rc
NSM_WINO_TILE=6 timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py -k "not bf16 and not configs2" -q -rA --timeout 300 --timeout-method thread > gpurun_out/t_wino6_model.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_wino6_model.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
 for t in 4 6; do
  NSM_WINO_TILE=$t timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_wino_${t}_$i.log 2>&1 || exit 1
 done
done
