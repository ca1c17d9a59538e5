# A/B of environment knobs on one box (run through gpurun):
#   ARMS="NSM_F32_SPLIT=1 NSM_F32_SPLIT=2" [REPS=2] [ARGS="--dtype bf16 --batch 64"] bash tools/ab.sh
# Each arm is a comma-separated list of VAR=value (an empty arm: "-"); the arms
# alternate within each repetition so clock drift hits them alike. Prints and
# appends "arm value ms_per_step" to gpurun_out/ab/res.log.
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
REPS=${REPS:-2}
for rep in $(seq 1 "$REPS"); do
  for arm in $ARMS; do
    envs=$(echo "$arm" | tr ',' ' '); [ "$arm" = "-" ] && envs="NSM_AB_BASE=1"
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-secondary \
        --no-cpu-baseline $ARGS > $O/b.log 2>&1 || exit $?
    line="$arm $(python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
    echo "$line" | tee -a $O/res.log
  done
done
