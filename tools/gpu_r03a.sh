# round 3: the default bench (headline + secondary + CPU baselines), then the f32 profiles
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail gpurun_out/bench_detail_a.json > gpurun_out/b_a.log 2>&1 || exit $?
timeout -k 10 900 bash tools/run_profiles.sh r03 f32 > gpurun_out/prof_a.log 2>&1
