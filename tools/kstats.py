#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv (top kernels by total time).

    python tools/kstats.py gpurun_out/x/run_kernel_stats.csv [N]
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.replace("nsm::", "")
    return name[:170]


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:n]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e6:9.2f} ms {100 * t / tot:6.2f}% n={int(r['Calls']):>5} "
              f"avg={float(r['AverageNs']) / 1e3:9.1f}us {short(r['Name'])}")
    print(f"total {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} launches")


if __name__ == "__main__":
    main()
