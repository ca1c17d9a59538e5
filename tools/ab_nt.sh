# A/B of non-temporal streaming stores (libnsm_nt.so, -DNSM_ST8_NT=1) and the
# row-blocked resize forward, bf16 B=64 and fp32 B=8, interleaved
set -o pipefail
mkdir -p gpurun_out/nt
for r in 1 2; do
  for arm in "X=1" "NSM_LIB=pcss-unet_amd/nsm_amd/libnsm_nt.so" "NSM_LIB=pcss-unet_amd/nsm_amd/libnsm_nt.so NSM_RESIZE_FWD_ROWS=2"; do
    env $arm timeout -k 10 200 python bench.py --dtype bf16 --batch 64 --steps 20 --no-secondary --no-cpu-baseline > gpurun_out/nt/b.log 2>&1 || exit 1
    env $arm timeout -k 10 200 python bench.py --steps 50 --no-secondary --no-cpu-baseline > gpurun_out/nt/f.log 2>&1 || exit 1
    python3 - "$arm" <<'PY'
import json,sys
def g(f):
    for l in open(f):
        if l.startswith('{'): return json.loads(l)
b=g('gpurun_out/nt/b.log'); f=g('gpurun_out/nt/f.log')
print(sys.argv[1][:60].ljust(60), 'bf16', b['value'], b['eager']['value'], 'f32', f['value'], f['eager']['value'])
print('   bf16 stages', [r[1] for r in b['stages']])
PY
  done
done
