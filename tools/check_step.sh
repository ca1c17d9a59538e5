# quick GPU check after a change: selected tests ($K), two benches, the step timeline
set -o pipefail
O=gpurun_out/chk; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q ${K:+-k "$K"} --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-secondary --no-cpu-baseline >> $O/bench.log 2>&1 || exit $?
done
bash tools/prof_step.sh && cp gpurun_out/prof_step/timeline.txt $O/
