# A/B: conv2.0 weight gradient on multi-tap 32x128 tiles (default) vs per-tap
# 32x32 tiles, after the split-count rounding fix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in 1 0 1 0; do
  NSM_WGRAD_MULTITAP=$T timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/s_b_$T.log 2>&1 || exit 1
  echo "MULTITAP=$T $(grep -o '"value":[0-9.]*' gpurun_out/s_b_$T.log | head -1)"
done
