"""Calibration of rocprofv3's HBM byte counters on known byte counts
(MI355X_MICROARCH.md §HBM calibrates only 16-B/lane
global loads and stores).

  python tools/pmc_calib.py run
      the launches, under rocprofv3 --pmc (one counter set per run):
      nsm_pmc_calib kinds 0..6 (include/nsm.h: global / LDS-DMA 16-B reads;
      global 16-B / LDS-staged buffer 16-B (the persistent h2 GEMM's fp32
      epilogue) / buffer 8-B (its f16-M epilogue) / 4-B / 8-B stores), each
      1 GiB, 3 launches each; then conv6.conv.0's forward Winograd GEMM
      (nsm_wino_gemm_h2, F(6x6), B=8: 64 x M=968 N=1024 K=2048 f16, V + U
      read = 522 MB, M written = 254 MB) run ALONE, 3 launches. Every launch
      is followed by a 64 MiB read-only probe (kind 0) whose write counter
      shows the dirty lines the launch before left in L2 (written back later).
  python tools/pmc_calib.py summarize OUT_JSON CSV [CSV ...]
      per pattern: the true bytes, the counted ones and their ratio -> the
      per-pattern correction that tools/pmc_traffic.py / tools/stage_pmc.py
      apply.
"""
import json
import os
import sys

GIB = 1 << 30
PROBE = 64 << 20
KINDS = {0: ("read", "global_load_dwordx4"), 1: ("read", "buffer_load ... lds (LDS-DMA 16 B/lane)"),
         2: ("write", "global_store_dwordx4"),
         3: ("write", "LDS-staged raw_buffer_store_b128 (h2p fp32 epilogue)"),
         4: ("write", "raw_buffer_store_b64 (h2p f16-M epilogue)"),
         5: ("write", "global_store_dword (4 B/lane)"), 6: ("write", "global_store_dwordx2 (8 B/lane)")}
REPS = 3
# conv6.conv.0 fwd at B=8: F(6x6) over 64x64 -> T = 8 * 11 * 11 tiles
T6, C6, NB6 = 968, 1024, 64
GEMM_READ = NB6 * (T6 * 2 * C6 + C6 * 2 * C6) * 2
GEMM_WRITE = NB6 * T6 * C6 * 4


def run():
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pcss-unet_amd"))
    from nsm_amd import ops
    from nsm_amd._lib import call, ptr, stream
    dev = torch.device("cuda:0")
    src = torch.randint(0, 1 << 30, (GIB // 4,), dtype=torch.int32, device=dev)
    dst = torch.empty(GIB // 4, dtype=torch.int32, device=dev)
    psrc = torch.randint(0, 1 << 30, (PROBE // 4,), dtype=torch.int32, device=dev)
    pdst = torch.empty(2048, dtype=torch.int32, device=dev)
    st = stream()

    def probe():
        call("nsm_pmc_calib", 0, ptr(psrc), ptr(pdst), PROBE, st)
        torch.cuda.synchronize()

    probe()
    for k in KINDS:
        for _ in range(REPS):
            call("nsm_pmc_calib", k, ptr(src), ptr(dst), GIB, st)
            torch.cuda.synchronize()
            probe()
    # the dominant GEMM alone on h2 operands written by nsm_to_h2
    g = torch.Generator(device=dev).manual_seed(6)
    V = torch.randn(NB6 * T6 * C6, device=dev, generator=g)
    U = torch.randn(NB6 * C6 * C6, device=dev, generator=g) * 0.03
    am = ops.amax_slots(2, dev)
    av, au = ops.absmax(V, ops.amax_slot(am, 0)), ops.absmax(U, ops.amax_slot(am, 1))
    Vh = torch.empty(V.numel() * 2, dtype=torch.float16, device=dev)
    Uh = torch.empty(U.numel() * 2, dtype=torch.float16, device=dev)
    call("nsm_to_h2", ptr(V), NB6 * T6, C6, ptr(av), 1.0, ptr(Vh), st)
    call("nsm_to_h2", ptr(U), NB6 * C6, C6, ptr(au), 1.0, ptr(Uh), st)
    del V, U
    Mb = torch.empty(NB6 * T6 * C6, device=dev)
    torch.cuda.synchronize()
    probe()
    for _ in range(REPS):
        call("nsm_wino_gemm_h2", ptr(Vh), ptr(Uh), 8, 64, 64, C6, C6, 6, ptr(Mb), ptr(av), 1.0,
             ptr(au), 1.0, st)
        torch.cuda.synchronize()
        probe()
    print("pmc_calib: launches done", flush=True)


def summarize(out_path, csvs):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from stage_pmc import load_pmc, stamp
    seq = [("probe", None)]
    for k in KINDS:
        for _ in range(REPS):
            seq += [(f"kind{k}", k), ("probe", None)]
    seq += [("to_h2", None), ("to_h2", None), ("probe", None)]
    for _ in range(REPS):
        seq += [("gemm", None), ("probe", None)]
    acc = {}
    for p in csvs:
        disp = [d for d in load_pmc(p) if "pmc_calib_kernel" in d[0] or "gemm_h2" in d[0]
                or "to_h2_kernel" in d[0]]
        # the absmax launches before the GEMM are not in seq: keep calib / to_h2 / GEMM only
        if len(disp) != len(seq):
            raise SystemExit(f"{p}: {len(disp)} dispatches, expected {len(seq)}")
        for i, (name, _, (cnt, _)) in enumerate(disp):
            for c, v in cnt.items():
                acc.setdefault((i, c), []).append(v)
    counters = sorted({c for (_, c) in acc})

    def val(i, c):
        v = acc.get((i, c))
        return sum(v) / len(v) if v else None

    def bytes_of(i):
        out = {}
        rd = val(i, "TCC_EA0_RDREQ_128B_sum")
        if rd is not None:
            r32, r64, tot = val(i, "TCC_EA0_RDREQ_32B_sum"), val(i, "TCC_EA0_RDREQ_64B_sum"), \
                val(i, "TCC_EA0_RDREQ_sum")
            rest = max(0.0, tot - r32 - r64 - rd)
            out["read_req_bytes"] = 32 * r32 + 64 * (r64 + rest) + 128 * rd
        if val(i, "FETCH_SIZE") is not None:
            out["fetch_size_x2"] = val(i, "FETCH_SIZE") * 1024 * 2
        if val(i, "WRITE_SIZE") is not None:
            out["write_size"] = val(i, "WRITE_SIZE") * 1024
        if val(i, "TCC_EA0_WRREQ_64B_sum") is not None:
            w64, wt = val(i, "TCC_EA0_WRREQ_64B_sum"), val(i, "TCC_EA0_WRREQ_sum")
            out["write_req_bytes"] = 64 * w64 + 32 * max(0.0, wt - w64)
        return out

    res = {"what": __doc__.split("\n\n")[0], "counters": counters, "patterns": {}}
    for k, (rw, desc) in KINDS.items():
        idx = [i for i, (n, kk) in enumerate(seq) if kk == k]
        rows = [bytes_of(i) for i in idx]
        follow = [bytes_of(i + 1) for i in idx]
        avg = {f: sum(r[f] for r in rows) / len(rows) for f in rows[0]}
        fol = {f: sum(r[f] for r in follow) / len(follow) for f in follow[0]}
        true = GIB
        ent = {"access": desc, "direction": rw, "true_bytes": true, "counted": avg,
               "probe_after": fol}
        if rw == "read":
            for f in ("read_req_bytes", "fetch_size_x2"):
                if f in avg:
                    ent[f"{f}_over_true"] = round(avg[f] / true, 4)
        else:
            for f in ("write_size", "write_req_bytes"):
                if f in avg:
                    # the launch's own count + what the next launch wrote back for it
                    ent[f"{f}_over_true"] = round(avg[f] / true, 4)
                    ent[f"{f}_with_writeback_over_true"] = round((avg[f] + fol.get(f, 0.0)) / true, 4)
        res["patterns"][f"kind{k}"] = ent
    gi = [i for i, (n, _) in enumerate(seq) if n == "gemm"]
    rows = [bytes_of(i) for i in gi]
    follow = [bytes_of(i + 1) for i in gi]
    avg = {f: sum(r[f] for r in rows) / len(rows) for f in rows[0]}
    fol = {f: sum(r[f] for r in follow) / len(follow) for f in follow[0]}
    g = {"kernel": "nsm_wino_gemm_h2 alone: conv6.conv.0 fwd F(6x6) B=8 (64 x 968 x 1024 x 2048 f16)",
         "true_read_bytes": GEMM_READ, "true_write_bytes": GEMM_WRITE, "counted": avg,
         "probe_after": fol}
    if "read_req_bytes" in avg:
        g["read_req_over_true"] = round(avg["read_req_bytes"] / GEMM_READ, 4)
    if "write_size" in avg:
        g["write_size_over_true"] = round(avg["write_size"] / GEMM_WRITE, 4)
        g["write_size_with_writeback_over_true"] = round(
            (avg["write_size"] + fol.get("write_size", 0.0)) / GEMM_WRITE, 4)
    res["gemm_alone"] = g
    res["stamp"] = stamp()
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2], sys.argv[3:])
