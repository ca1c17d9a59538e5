set -o pipefail
mkdir -p gpurun_out
for v in 8 1000 1 8; do
  NSM_WGRAD_HOLD_GB=$v timeout -k 10 200 python bench.py --dtype bf16 --batch 64 --steps 20 --no-secondary --no-cpu-baseline > gpurun_out/ab1_$v.log 2>&1 || exit 1
  python - gpurun_out/ab1_$v.log $v <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print('hold',sys.argv[2],'graph',d['value'],'eager',d.get('eager'),'conv7',[r[1] for r in d['stages']])
PY
done
NSM_WGRAD_STREAM=0 timeout -k 10 200 python bench.py --dtype bf16 --batch 64 --steps 20 --no-secondary --no-cpu-baseline > gpurun_out/ab1_ns.log 2>&1 && grep -o '"value":[0-9.]*\|"eager":{[^}]*}' gpurun_out/ab1_ns.log
