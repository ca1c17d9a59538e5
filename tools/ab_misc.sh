# GPU A/B: Winograd for the 64-channel layers (NSM_WINO_MIN=64) in fp32; 16x16x32 MFMA on the
# deep 256x256 bf16 tiles only (NSM_BF16_MF16=2).
set -o pipefail
NSM_WINO_MIN=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "configs1 or configs0" -q --timeout 250 --timeout-method thread > gpurun_out/t_misc.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_misc.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
 for m in 128 64; do
  NSM_WINO_MIN=$m timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/ab_wmin_${m}_$i.log 2>&1 || exit 1
 done
 for m in 0 2; do
  NSM_BF16_MF16=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_mf2_${m}_$i.log 2>&1 || exit 1
 done
done
