"""tools/stage_pmc.py: dispatches between stage markers are attributed to
their stage, per step, and the counter arithmetic (request sizes, MFMA MOPS,
busy fraction) is as documented. Synthetic rocprofv3 CSVs, no GPU."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mark(code):
    return ("void nsm::stage_mark_kernel(int)", (code + 1) * 64)


def _step():
    # other: prep; conv2.fwd: one GEMM; conv2.bwd: one kernel; head.fwd; other: tail
    return [("prep_weights_kernel", 256), _mark(1), ("gemm_a", 1024), _mark(0), _mark(2),
            ("bwd_b", 512), _mark(0), _mark(17), ("head_c", 64), _mark(0), ("tail_adamw", 64)]


def _write(tmp, steps=3):
    disp = [d for _ in range(steps) for d in _step()]
    tr = tmp / "trace.csv"
    with open(tr, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z",
                    "Start_Timestamp", "End_Timestamp"])
        t = 0
        for i, (n, g) in enumerate(disp):
            dur = {"gemm_a": 2000, "bwd_b": 1000, "head_c": 500}.get(n, 100)
            w.writerow([i + 1, n, g, 1, 1, t, t + dur])
            t += dur + 10
    vals = {"gemm_a": {"TCC_EA0_RDREQ_sum": 100, "TCC_EA0_RDREQ_32B_sum": 10,
                       "TCC_EA0_RDREQ_64B_sum": 20, "TCC_EA0_RDREQ_128B_sum": 60,
                       "WRITE_SIZE": 2.0, "SQ_VALU_MFMA_BUSY_CYCLES": 1024 * 100,
                       "GRBM_GUI_ACTIVE": 8 * 200, "SQ_INSTS_VALU_MFMA_MOPS_BF16": 1000,
                       "SQ_INSTS_VALU_MFMA_MOPS_F32": 0},
            # a short dispatch (< 0.3 ms): its busy fraction is not reported
            "bwd_b": {"WRITE_SIZE": 1.0, "SQ_VALU_MFMA_BUSY_CYCLES": 1024 * 50,
                      "GRBM_GUI_ACTIVE": 8 * 100}}
    dur_ns = {"gemm_a": 400000}
    pm = tmp / "pmc.csv"
    with open(pm, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Correlation_Id", "Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name",
                    "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        for i, (n, g) in enumerate(disp):
            for c, v in vals.get(n, {"WRITE_SIZE": 1.0, "GRBM_GUI_ACTIVE": 8}).items():
                w.writerow([i + 1, i + 1, g, n, c, v, 0, dur_ns.get(n, 4000)])
    return tr, pm


def test_stage_attribution_and_counters(tmp_path):
    tr, pm = _write(tmp_path)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stage_pmc.py"), str(out),
                    str(tr), str(pm)], check=True, capture_output=True)
    d = json.load(open(out))
    st = d["stages"]
    assert d["steps_averaged"] == 2
    assert st["conv2.fwd"]["kernel_ms"] == 0.002
    assert st["conv2.bwd"]["kernel_ms"] == 0.001
    assert st["head.fwd"]["kernel_ms"] == 0.0005
    # other = tail of the step + prep of the next one
    assert abs(st["other"]["kernel_ms"] - 0.0002) < 1e-9
    # 10 + 10 unsized requests at 32/64 B, 20 at 64 B, 60 at 128 B
    assert st["conv2.fwd"]["read_bytes"] == 32 * 10 + 64 * (20 + 10) + 128 * 60
    assert st["conv2.fwd"]["write_bytes"] == 2048
    assert st["conv2.fwd"]["mfma_busy"] == 0.5
    assert abs(st["conv2.fwd"]["eff_clock_ghz"] - 200 / 0.4e-3 / 1e9) <= 1e-3  # rounded to MHz
    assert "mfma_busy" not in st["conv2.bwd"]       # 0.004 ms dispatch: no clock / busy
    assert len(d["stamp"]["libnsm_sha256"]) == 64
    assert st["conv2.fwd"]["bf16_mfma_flops"] == 512 * 1000
    # fwd + bwd rolled up
    assert st["conv2"]["kernel_ms"] == 0.003
    assert st["conv2"]["write_bytes"] == 2048 + 1024
