#!/usr/bin/env python3
"""One train step's launches from a rocprofv3 kernel_trace.csv (steps end at
the AdamW kernel): duration, grid (blocks), short name; then totals per kernel
family. usage: python tools/step_timeline.py TRACE_CSV|RESULTS_DB [step_index_from_end=1]
(RESULTS_DB: the rocpd sqlite file rocprofv3 writes without --output-format csv)"""
import collections
import os
import csv
import re
import sys

def load(path):
    if not path.endswith(".db"):
        return list(csv.DictReader(open(path)))
    import sqlite3
    c = sqlite3.connect(path)
    q = ("select s.display_name, d.start, d.end, d.grid_size_x, d.grid_size_y, d.grid_size_z, "
         "d.workgroup_size_x, d.workgroup_size_y, d.workgroup_size_z from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    keys = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y",
            "Grid_Size_Z", "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z"]
    return [dict(zip(keys, r)) for r in c.execute(q)]


rows = load(sys.argv[1])
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ends = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
a, b = ends[-1 - k] + 1, ends[-k] + 1
fam = collections.Counter()
tot = 0.0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("nsm::", "")
    g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]) //
         int(r["Workgroup_Size_Y"]), int(r["Grid_Size_Z"]) // int(r["Workgroup_Size_Z"]))
    print(f"{d:8.1f} {str(g):18s} {n[:int(os.environ.get('STL_NAMELEN', 110))]}")
    fam[re.sub(r"<.*", "", n)] += d
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"\nkernels {tot:.0f} us, span {span:.0f} us, launches {b - a}")
for n, d in fam.most_common():
    print(f"{d:9.1f} us {100 * d / tot:5.1f}%  {n}")
