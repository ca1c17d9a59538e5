# the bf16 spread parity test under arithmetic switches (ARMS, diagnosis)
set -o pipefail
for arm in ${ARMS:-"- NSM_BF16_WINO=0"}; do
  envs=$(echo "$arm" | tr ',' ' '); [ "$arm" = "-" ] && envs="NSM_AB_BASE=1"
  echo "== $arm" >> gpurun_out/diag_spread.log
  env $envs timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "small_res and spread" -x -q -s --timeout 280 --timeout-method thread 2>&1 | grep -E "configs\[2\]|worst|passed|failed" >> gpurun_out/diag_spread.log
done
true
