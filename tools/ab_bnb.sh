# GPU: the epilogue BN-backward (nsm_conv1x1_dgrad_bnbwd) op tests, the model
# parity suites, then an A/B of NSM_BNB 0 / 1 / 2 on both train configs.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "dgrad_bn_bwd or bn_act" -q --timeout 200 --timeout-method thread > gpurun_out/t_bnb_ops.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_bnb_ops.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_bf16.py tests/test_gpu_dp.py -q --timeout 300 --timeout-method thread > gpurun_out/t_bnb_model.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_bnb_model.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
 for m in 0 1 2; do
  NSM_BNB=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_bnb_f32_${m}_$i.log 2>&1 || exit 1
  NSM_BNB=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_bnb_bf16_${m}_$i.log 2>&1 || exit 1
 done
done
