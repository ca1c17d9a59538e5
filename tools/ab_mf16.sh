set -o pipefail
export NSM_BF16_MF16=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_configs.py -k "bf16 or configs2" -q --timeout 200 --timeout-method thread > gpurun_out/t_mf16.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_mf16.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
 for m in 0 1; do
  NSM_BF16_MF16=$m timeout -k 10 120 python bench.py --dtype bf16 --batch 64 --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/ab_mf16_${m}_$i.log 2>&1 || exit 1
 done
done
