# GPU: A/B of NSM_BNB 0 / 2 (per-layer policy) on both train configs.
set -o pipefail
for i in 1 2; do
 for m in 0 2; do
  NSM_BNB=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_bnb_f32_${m}_$i.log 2>&1 || exit 1
  NSM_BNB=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_bnb_bf16_${m}_$i.log 2>&1 || exit 1
 done
done
