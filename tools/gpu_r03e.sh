# round 3: gpu suite with the direct 1x1 GEMMs on f16x2 too, then A/B of NSM_F32_SPLIT 1 vs 2
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_e.log 2>&1
rc=$?; echo RC=$rc >> gpurun_out/t_e.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for m in 1 2; do
    NSM_F32_SPLIT=$m timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline --detail gpurun_out/bd_e_${m}_$i.json > gpurun_out/b_e_${m}_$i.log 2>&1 || exit $?
  done
done
