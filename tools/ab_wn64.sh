# 256x64 tiles for the 64-channel Winograd GEMMs (NSM_WINO_N64_BM256)
set -o pipefail
O=gpurun_out/wn64; rm -rf $O; mkdir -p $O
NSM_WINO_N64_BM256=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "wino or model or configs or split" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit 1
for v in 0 1 0 1 0 1; do
  NSM_WINO_N64_BM256=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-secondary --no-cpu-baseline > $O/b.log 2>&1 || exit 1
  echo "$v $(grep -o '"value": [0-9.]*' $O/b.log)" >> $O/res.log
done
for v in 0 1; do
  NSM_WINO_N64_BM256=$v bash tools/prof_step.sh || exit 1
  grep -E "<(128|256), 64, (2, 2|4, 1)" gpurun_out/prof_step/timeline.txt | cut -c1-110 > $O/tl_$v.txt
done
