# GPU: split GEMM microbench (NST 1 / 2), split op tests, then step A/B
set -o pipefail
for n in 1 2; do
  NSM_SPLIT_NST=$n timeout -k 10 120 python tools/bench_split.py > gpurun_out/bs_nst$n.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_ops.py -q -x -k "split or wino" --timeout 300 --timeout-method thread > gpurun_out/t_split.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_split.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  NSM_F32_SPLIT=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_sp_${m}_1.log 2>&1 || exit 1
done
