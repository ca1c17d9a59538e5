"""Mean PMC counter values per kernel family over rocprofv3 counter_collection
CSVs (one or more passes): usage python tools/pmc_summary.py CSV... ;
derived: MFMA busy per SIMD-cycle, effective clock (GRBM_GUI_ACTIVE / 8 XCDs /
kernel time), wait / issue shares of wave cycles."""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        fam = re.sub(r"^nsm::", "", name)[:120]
        acc[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "Start_Timestamp" in r:
            dur[fam].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for fam, cs in acc.items():
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    print(fam)
    for k in sorted(m):
        print(f"   {k:28s} {m[k]:.4g}")
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        # SQ_BUSY_CYCLES: per SE quad-cycles summed; MFMA busy counts cycles per SIMD
        pass
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in m:
                print(f"   share {k:22s} {m[k] / w:.3f}")
    if fam in dur and dur[fam] and "GRBM_GUI_ACTIVE" in m:
        t = sum(dur[fam]) / len(dur[fam])
        print(f"   kernel_us {t:.1f}  eff_clock_GHz {m['GRBM_GUI_ACTIVE'] / 8 / (t * 1e3):.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            simd_cycles = m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4
            print(f"   mfma_busy_per_simd_cycle {m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.3f}")
