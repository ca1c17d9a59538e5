# Check of git HEAD on one box (through gpurun) when the library is unchanged
# since the last profiles: the out-of-bounds audit, the whole -m gpu suite and
# the default bench line (which reads the stamped profiles/r05 files). Each step
# under its own time limit, && chained; logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/h_guard.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/h_bench.log 2>&1
