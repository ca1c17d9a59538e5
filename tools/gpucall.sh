# Local helper (runs HERE, not on the box): one gpurun call, re-issued only
# when gpurun reports that nothing ran (no slot / no box / transient lease
# loss: exit 3 or status=transient). Any other outcome ends it.
#   bash tools/gpucall.sh TIMEOUT 'command' OUTFILE
T=$1; CMD=$2; OUT=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q 'status=transient' "$OUT"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
