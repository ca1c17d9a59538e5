# round 3: the whole -m gpu suite on the f16x2 default, then the default bench
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_c.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_c.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail gpurun_out/bench_detail_c.json > gpurun_out/b_c.log 2>&1
