#!/usr/bin/env python3
"""One-line summaries of bench.py JSON logs: python tools/bsum.py log [log ...]"""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print(f, "NO JSON")
        continue
    d = json.loads(lines[-1])
    r = d["roofline"]
    st = " ".join(f"{s['stage']}={s['ms']}" for s in d.get("stages", []))
    print(f"{f}: {d['value']} {d['unit']} {d['ms_per_step']} ms/step | dom {r['achieved']} "
          f"{r['unit']} frac {r['frac']} | {st}")
