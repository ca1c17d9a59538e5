# GPU check of round 6: the out-of-bounds audit first (its own time limit, so
# a fault ends the call there), then the named tests (TESTS, default the whole
# -m gpu suite), then the default bench line (BENCH=0 skips it). Each step
# under its own time limit, && chained; logs under gpurun_out/.
set -o pipefail
T=${TESTS:-"tests"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_guard.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_guard.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/t_r06.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_r06.log; [ $rc -eq 0 ] || exit $rc
[ "${BENCH:-1}" = "0" ] && exit 0
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/b_r06.log 2>&1
