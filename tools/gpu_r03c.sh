# round 3: the f16x2 split microbenchmark
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_split16.py > gpurun_out/split16.log 2>&1
