#!/usr/bin/env python3
"""List the launches of one step from a rocprofv3 kernel_trace.csv in order:
    python tools/ktrace.py trace.csv [first_dispatch] [count] [name-filter]
Prints duration (us), grid, block, name."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else 400
filt = sys.argv[4] if len(sys.argv) > 4 else ""
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if filt in r["Kernel_Name"]][first:first + count]
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("nsm::", "")[:90]
    g = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    print(f"{d:9.1f} {str(g):22s} wg={r['Workgroup_Size_X']:>4} v={r['VGPR_Count']}/{r['Accum_VGPR_Count']} {n}")
