# kernel traces for round-5 work: the 1080p bf16 eval (one graph replay's
# launches, the last N) and the bf16 B=64 train step timeline
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/prof5; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/inf -o run -- \
    python3 bench.py --workload infer1080 --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline > $O/inf.log 2>&1
T=$(find $O/inf -name run_kernel_trace.csv -print -quit)
N=$(python3 -c "import csv,sys; r=list(csv.DictReader(open('$T'))); print(len(r))")
python3 tools/ktrace.py "$T" $((N - ${NK:-110})) ${NK:-110} > $O/inf_last.txt
cp "$(find $O/inf -name run_kernel_stats.csv -print -quit)" $O/inf_stats.csv
rm -rf $O/inf
CFG="--dtype bf16 --batch 64" bash tools/prof_step.sh
cp gpurun_out/prof_step/timeline.txt $O/step_b64_bf16.txt
