# the last eager 1080p forward's launches (bf16 and fp32), one rocprofv3 kernel trace each
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pinf
for d in bf16 f32; do
  rm -rf gpurun_out/pinf/raw_$d
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pinf/raw_$d -o run -- python3 bench.py --workload infer1080 --dtype $d --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pinf/$d.log 2>&1
  T=$(find gpurun_out/pinf/raw_$d -name run_kernel_trace.csv -print -quit)
  N=$(python3 -c "import csv; print(len(list(csv.DictReader(open('$T')))))")
  python3 tools/ktrace.py "$T" $((N - ${NK:-80})) ${NK:-80} > gpurun_out/pinf/last_$d.txt
  rm -rf gpurun_out/pinf/raw_$d
  grep -o '"value":[0-9.]*' gpurun_out/pinf/$d.log | head -1
done
