# BN partial merges: separate first-level merge kernels (default thresholds) vs the block-per-channel finalize reading every row
set -o pipefail
O=gpurun_out/merge; rm -rf $O; mkdir -p $O
for v in a b a b a b; do
  if [ $v = a ]; then E="NSM_MERGE_ABOVE=1024 NSM_SUM_ROWS_ABOVE=512"; else E="NSM_MERGE_ABOVE=8192 NSM_SUM_ROWS_ABOVE=8192"; fi
  env $E timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-secondary --no-cpu-baseline > $O/b.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' $O/b.log)" >> $O/res.log
done
NSM_MERGE_ABOVE=8192 NSM_SUM_ROWS_ABOVE=8192 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "bn or model or configs" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit 1
