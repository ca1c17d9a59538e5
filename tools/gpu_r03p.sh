# persistent h2 GEMM: accuracy tests, GEMM timing A/B, short step bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q -k h2 --timeout 120 --timeout-method thread > gpurun_out/p_t.log 2>&1 && tail -3 gpurun_out/p_t.log &&
for P in 1 0 1 0; do
  NSM_H2_PERSIST=$P SHAPES=0,1 REPS=30 timeout -k 10 120 python tools/bench_h2.py > gpurun_out/p_h2_$P.log 2>&1 && echo "PERSIST=$P" && cat gpurun_out/p_h2_$P.log || exit 1
done &&
for P in 1 0 1 0; do
  NSM_H2_PERSIST=$P timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/p_b_$P.log 2>&1 || exit 1
  echo "bench PERSIST=$P" && grep -o '"value": [0-9.]*' gpurun_out/p_b_$P.log | head -1
done
