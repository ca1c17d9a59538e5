# kernel trace of the VGG-inclusive fp32 step (bench.py --vgg): per-kernel
# stats and the step timeline under gpurun_out/vggprof/
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/vggprof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- \
    python3 bench.py --vgg --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/b.log 2>&1
cp "$(find $O/t -name run_kernel_stats.csv -print -quit)" $O/stats.csv
python3 tools/step_timeline.py "$(find $O/t -name run_kernel_trace.csv -print -quit)" > $O/timeline.txt
rm -rf $O/t
