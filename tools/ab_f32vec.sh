# GPU: fp32 LDS-staged 16-B store epilogue (NSM_F32_EPI_VEC): op/model tests + A/B
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread > gpurun_out/t_fv.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_fv.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
 for m in 0 1; do
  NSM_F32_EPI_VEC=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_fv_${m}_$i.log 2>&1 || exit 1
 done
done
