set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for m in 0 2; do
NSM_BNB=$m timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/prof_bnb$m -o run -- python3 bench.py --dtype bf16 --batch 64 --steps 3 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/prof_bnb$m.log 2>&1 || exit 1
NSM_BNB=$m timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/prof_bnbf$m -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/prof_bnbf$m.log 2>&1 || exit 1
done
