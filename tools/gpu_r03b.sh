# round 3: the f16x2 split microbenchmark, the new / changed GPU tests, then the bf16 profiles
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_split16.py > gpurun_out/split16.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_tail.py tests/test_gpu_dp.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_b.log 2>&1 || exit $?
timeout -k 10 900 bash tools/run_profiles.sh r03 bf16 > gpurun_out/prof_b.log 2>&1
