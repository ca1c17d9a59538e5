# after the direct-wgrad split rounding and the shared prep slot: the tests
# that cover them, then a short bench with a kernel trace of the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r_t.log 2>&1; rc=$?
tail -3 gpurun_out/r_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r_tr -o run -- python3 bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline > gpurun_out/r_tr.log 2>&1 || exit 1
python3 tools/step_timeline.py "$(find gpurun_out/r_tr -name run_kernel_trace.csv | head -1)" > gpurun_out/r_timeline.txt || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r_b$i.log 2>&1 || exit 1
  echo "bench $(grep -o '"value":[0-9.]*' gpurun_out/r_b$i.log | head -1)"
done
