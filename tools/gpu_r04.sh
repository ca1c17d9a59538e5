# GPU: the named test files (TESTS, default the h2 1x1 ops + the B=8 parity),
# then a short bench (STEPS). Each step under its own time limit, && chained.
set -o pipefail
T=${TESTS:-"tests/test_gpu_h2d.py tests/test_gpu_configs.py"}
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r04.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_r04.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/b_r04.log 2>&1
