# Winograd transform changes: op tests, bench, per-step kernel timeline
set -o pipefail
O=gpurun_out/wino; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wino" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-secondary --no-cpu-baseline >> $O/bench.log 2>&1 || exit $?
bash tools/prof_step.sh && cp gpurun_out/prof_step/timeline.txt $O/
