# kernel trace of the 1080p inference bench (bf16 and fp32), for the per-kernel view
set -euo pipefail
export TMPDIR=/tmp
for d in bf16 f32; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_inf_$d -o run -- python3 bench.py --workload infer1080 --dtype $d --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_inf_$d.log 2>&1
done
