# Round-5 final check on one box (through gpurun): the out-of-bounds audit, the
# whole -m gpu suite, the profiles under profiles/r05 (stamped with GIT_HEAD and
# the library hash) and the default bench line, which reads them. Each step
# under its own time limit, && chained; logs under gpurun_out/.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/f_guard.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/f_tests.log 2>&1 &&
timeout -k 10 400 bash tools/run_profiles.sh r05 both > gpurun_out/f_prof.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/f_bench.log 2>&1
