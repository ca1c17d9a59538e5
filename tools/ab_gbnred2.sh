# GPU: A/B of NSM_GRAD_BNRED 0 / 1 (resize + pooling producers) on both train configs.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q -k "train" --timeout 200 --timeout-method thread > gpurun_out/t_gb_model.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_gb_model.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
 for m in 0 1; do
  NSM_GRAD_BNRED=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_gb_f32_${m}_$i.log 2>&1 || exit 1
  NSM_GRAD_BNRED=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_gb_bf16_${m}_$i.log 2>&1 || exit 1
 done
done
