# kernel trace of a short fp32 (default) or bf16 (CFG) bench run -> per-step timeline
set -euo pipefail
OUT=gpurun_out/prof_step
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/raw" -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-secondary ${CFG:-} > "$OUT/bench.log" 2>&1
python3 tools/step_timeline.py "$(find "$OUT/raw" -name run_kernel_trace.csv -print -quit)" > "$OUT/timeline.txt"
rm -rf "$OUT/raw"
