# Queue and stream of the main-chain and weight-gradient kernels in the eager
# DP step vs the plain eager step (bench.py --force-dp at world size 1), and
# how much of the side stream's kernel time overlaps the main stream's.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/dpq; mkdir -p $O
for f in "" "--force-dp"; do
  rm -rf $O/raw
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/raw -o run -- python3 bench.py --steps 5 --warmup 3 --no-secondary --no-cpu-baseline $f > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
  echo "== ${f:-plain}"
  python3 - "$(find $O/raw -name run_kernel_trace.csv -print -quit)" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
by = collections.Counter()
for r in rows:
    n = r["Kernel_Name"]
    if "wino_wgrad_out" in n or "wgrad_reduce" in n:
        by[("side", r["Queue_Id"], r["Stream_Id"])] += 1
    elif "wino_output6" in n or "bn_finalize_train" in n:
        by[("main", r["Queue_Id"], r["Stream_Id"])] += 1
print("  (role, queue, stream): count", dict(by))
# overlap in the middle third of the trace (timed steps): side-stream kernels
# = stream ids seen on wgrad kernels
side = {k[2] for k in by if k[0] == "side"}
main = {k[2] for k in by if k[0] == "main"}
iv = {"side": [], "main": []}
n = len(rows)
for r in rows[n // 3: 2 * n // 3]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if r["Stream_Id"] in side and r["Stream_Id"] not in main:
        iv["side"].append((s, e))
    elif r["Stream_Id"] in main:
        iv["main"].append((s, e))
tot = sum(e - s for s, e in iv["side"])
ov = 0
j = 0
m = sorted(iv["main"])
for s, e in sorted(iv["side"]):
    for ms, me in m:
        if me <= s or ms >= e:
            continue
        ov += min(e, me) - max(s, ms)
print(f"  side kernel time {tot/1e3:.0f} us, overlapped with main {ov/1e3:.0f} us")
PY
done
rm -rf $O/raw
