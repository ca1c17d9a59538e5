# GPU: every fp32 GEMM on the split kernel: op/model/config tests, then step A/B
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > gpurun_out/t_split.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_split.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for m in 0 1; do
  NSM_F32_SPLIT=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_sp_${m}_$i.log 2>&1 || exit 1
done
done
