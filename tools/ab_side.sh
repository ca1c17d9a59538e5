# Interleaved A/B of the weight-gradient side stream (NSM_WGRAD_STREAM 1 / 0):
# graph-replay and eager step rates, fp32 B=8 and bf16 B=64, three rounds
set -o pipefail
mkdir -p gpurun_out/side
for r in 1 2 3; do
  for v in 1 0; do
    NSM_WGRAD_STREAM=$v timeout -k 10 200 python bench.py --steps 50 --no-secondary --no-cpu-baseline > gpurun_out/side/f32_${v}_$r.log 2>&1 || exit 1
    NSM_WGRAD_STREAM=$v timeout -k 10 200 python bench.py --dtype bf16 --batch 64 --steps 20 --no-secondary --no-cpu-baseline > gpurun_out/side/bf16_${v}_$r.log 2>&1 || exit 1
    for c in f32 bf16; do
      python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], 'side', sys.argv[3], 'graph', d['value'], 'eager', d['eager']['value'])
" gpurun_out/side/${c}_${v}_$r.log $c $v
    done
  done
done
