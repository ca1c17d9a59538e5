# policy knobs re-checked under the split GEMM: default vs NSM_BNB=1 / NSM_F32_ACT=0 / NSM_WINO_STATS=0
set -o pipefail
O=gpurun_out/knobs; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for E in "NSM_DUMMY=0" "NSM_BNB=1" "NSM_F32_ACT=0" "NSM_WINO_STATS=0"; do
    env $E timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-secondary --no-cpu-baseline > $O/b.log 2>&1 || exit 1
    echo "$E $(grep -o '"value": [0-9.]*' $O/b.log)" >> $O/res.log
  done
done
