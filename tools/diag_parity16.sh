# Which F(4x4) f16 component drives the bf16 spread-parity ratio: the spread
# case of test_configs2_b64_bf16_small_res_vs_oracle under env variants,
# each printing its worst per-parameter ratios (parity_margins.json lines).
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_configs.py::test_configs2_b64_bf16_small_res_vs_oracle[spread]"
for v in ${DIAG_VARIANTS:-"X=1" "NSM_BF16_M16=0" "NSM_BF16_WINO=0"}; do
  env $v timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -q -s --timeout 250 --timeout-method thread > gpurun_out/diag16.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  grep -E "worst grad ratios|median grad|configs\[2\]" gpurun_out/diag16.log | cut -c1-700
  [ $rc -le 1 ] || exit $rc
done
