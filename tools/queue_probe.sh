# Hardware queue of each probe stream (tools/queue_probe.py) under variants.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/qp; mkdir -p $O
for f in "" "--dp" "--dp --early"; do
  rm -rf $O/raw
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/raw -o run -- python3 tools/queue_probe.py $f > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
  echo "== $f"
  python3 - "$(find $O/raw -name run_kernel_trace.csv -print -quit)" <<'PY'
import csv, sys
import collections
other = collections.Counter()
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"])):
    if "vectorized_elementwise" in r["Kernel_Name"]:
        print(f'  q{r["Queue_Id"]} s{r["Stream_Id"]} grid {r["Grid_Size_X"]:>8} (touch {int(r["Grid_Size_X"]) // 256 - 1})')
    else:
        other[(r["Queue_Id"], r["Stream_Id"])] += 1
print("  other kernels by (queue, stream):", dict(other))
PY
done
rm -rf $O/raw
