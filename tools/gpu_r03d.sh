# round 3: gpu suite on f16x2 + slot-spread maxima, then A/B of NSM_F32_SPLIT 1 vs 2 on the headline step
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_d.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_d.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for m in 1 2; do
    NSM_F32_SPLIT=$m timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline --detail gpurun_out/bd_d_${m}_$i.json > gpurun_out/b_d_${m}_$i.log 2>&1 || exit $?
  done
done
