# A/B: 256-tile weight-gradient split target (1024 blocks vs one round of 256)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in 1024 256 1024 256; do
  NSM_H2_WG256_BLOCKS=$T timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/q_b_$T.log 2>&1 || exit 1
  echo "WG256=$T $(grep -o '"value":[0-9.]*' gpurun_out/q_b_$T.log | head -1)"
done
