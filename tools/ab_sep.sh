# separable resampling kernels vs the 2-D gather forms (NSM_RESIZE_SEP), bf16 B=64 shapes + full bench
set -o pipefail
O=gpurun_out/absep; mkdir -p $O
for v in 0 1; do
  NSM_RESIZE_SEP=$v timeout -k 10 120 python tools/elem_bench.py > $O/eb_$v.log 2>&1 || exit 1
done
for v in 0 1; do
  NSM_RESIZE_SEP=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/b_$v.log 2>&1 || exit 1
done
