# Kernel-trace A/B: for each "ENV=VAL ..." variant in VARIANTS (separated by
# ';'), a short bench run under rocprofv3 --kernel-trace; prints the last
# (serialised attribution) step's kernels matching PAT with their durations,
# and the step's kernel total. CFG: bench flags (default fp32 B=8).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/abt; mkdir -p $O
IFS=';' read -ra VS <<< "${VARIANTS:-X=1}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  rm -rf $O/raw$i
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/raw$i -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-secondary ${CFG:-} > $O/bench$i.log 2>&1 || { echo "variant $v failed"; tail -5 $O/bench$i.log; exit 1; }
  python3 tools/step_timeline.py "$(find $O/raw$i -name run_kernel_trace.csv -print -quit)" > $O/tl$i.txt
  rm -rf $O/raw$i
  echo "== $v  $(grep -o '"value":[0-9.]*' $O/bench$i.log | head -1)  $(grep '^kernels' $O/tl$i.txt)"
  grep -nE "${PAT:-gemm}" $O/tl$i.txt | head -${NL:-40} | cut -c1-140
done
