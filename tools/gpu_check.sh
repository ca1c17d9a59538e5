# GPU: the whole -m gpu suite, then the default bench (headline + secondary configs).
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_all.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/b_all.log 2>&1
