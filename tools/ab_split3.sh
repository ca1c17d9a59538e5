set -o pipefail
for t in 128 256 257; do
  NSM_SPLIT_TILE=$t MODES=1 ONLY=gemm timeout -k 10 120 python tools/bench_split.py > gpurun_out/bs_t$t.log 2>&1 || exit 1
done
