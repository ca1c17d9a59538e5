# Round-6 final GPU check on one box: the out-of-bounds audit, the whole
# -m gpu suite, the stamped profiles (tools/run_profiles.sh r06), the default
# bench line (reading the profiles just written) and smoke(). Each step under
# its own time limit; the first failure ends the call.
set -uo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_guard.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --durations=15 --timeout 240 --timeout-method thread > gpurun_out/t_r06.log 2>&1 || exit 1
timeout -k 10 600 bash tools/run_profiles.sh r06 > gpurun_out/prof_r06.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/b_final3.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
echo FINAL_OK
