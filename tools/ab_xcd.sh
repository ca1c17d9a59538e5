# GPU: XCD remap of the split GEMM: op/model tests, microbench, step A/B
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_ops.py tests/test_gpu_model.py -q -x --timeout 300 --timeout-method thread > gpurun_out/t_xcd.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_xcd.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1; do
  NSM_SPLIT_XCD=$x MODES=1 timeout -k 10 120 python tools/bench_split.py > gpurun_out/bs_x$x.log 2>&1 || exit 1
done
for i in 1 2; do
for x in 0 1; do
  NSM_SPLIT_XCD=$x timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_x_${x}_$i.log 2>&1 || exit 1
done
done
