#!/usr/bin/env python3
"""Per-dispatch PMC values of a rocprofv3 counter_collection CSV (one pass):
python tools/pmc_disp.py CSV [name-regex] [last-N]: for the last N dispatches
matching the regex (default all), the grid, the duration and every counter,
with the wave-cycle shares of the SQ_WAIT_* / SQ_ACTIVE_* counters."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
last = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
disp = collections.OrderedDict()
for r in rows:
    if pat and not pat.search(r["Kernel_Name"]):
        continue
    key = r.get("Dispatch_Id") or r.get("Correlation_Id")
    d = disp.setdefault(key, {"name": re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""),
                              "grid": (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")),
                              "c": {}})
    d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if "Start_Timestamp" in r and r.get("End_Timestamp"):
        d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for key, d in list(disp.items())[-last:]:
    c = d["c"]
    print(f"{d.get('us', 0):9.1f} us grid={d['grid']} {d['name'][:110]}")
    w = c.get("SQ_WAVE_CYCLES")
    for k in sorted(c):
        share = f"  ({c[k] / w:.3f} of wave cycles)" if w and k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"    {k:30s} {c[k]:.4g}{share}")
