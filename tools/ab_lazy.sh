# GPU: bn_act_pool + lazy decoder outputs: op/model tests + A/B on both train configs
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_configs.py tests/test_gpu_bf16.py -q -k "lazy or pool or train or configs or bf16" --timeout 300 --timeout-method thread > gpurun_out/t_lz.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_lz.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
 for m in 0 1; do
  NSM_ACT_POOL=$m NSM_LAZY_DECODER=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_lz_f32_${m}_$i.log 2>&1 || exit 1
  NSM_ACT_POOL=$m NSM_LAZY_DECODER=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_lz_bf16_${m}_$i.log 2>&1 || exit 1
 done
done
