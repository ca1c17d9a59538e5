# GPU A/B: batched weight preparation (one launch) vs per-layer packing, fp32 and bf16 steps + 1080p bf16.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q --timeout 200 --timeout-method thread -x > gpurun_out/t_prep.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_prep.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
 for m in 0 1; do
  NSM_PREP_BATCH=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_prep_f32_${m}_$i.log 2>&1 || exit 1
  NSM_PREP_BATCH=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_prep_bf16_${m}_$i.log 2>&1 || exit 1
  NSM_PREP_BATCH=$m timeout -k 10 120 python bench.py --workload infer1080 --dtype bf16 --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/ab_prep_inf_${m}_$i.log 2>&1 || exit 1
 done
done
