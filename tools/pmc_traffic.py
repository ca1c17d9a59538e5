"""HBM traffic per launch of the dominant convolution kernel, from rocprofv3
PMC passes of a bench.py run with NSM_STAGE_MARKS=1 (the stage markers tell
conv6's forward launches from its input-gradient twins of the same shape);
bench.py reads the JSON into roofline.traffic.

usage: python tools/pmc_traffic.py KIND OUT_JSON PMC_CSV [PMC_CSV ...]
  f32_gemm : conv6.conv.0 fwd Winograd batched GEMM alone (B=8, F(6x6):
             gemm_f32s_kernel<128,128,2,2,RowsKLoader x2,EpiStore> grid 8x8x64)
  f32      : conv6.conv.0 fwd as a whole = wino_input + that GEMM + wino_output
  bf16     : conv6.conv.0 fwd LDS-DMA implicit GEMM, gemm_bf16_dma_kernel<256,256,..,
             ConvActDma,..> grid 4x1024 blocks (B=64)
Bytes per launch: reads = 32/64/128 x TCC_EA0_RDREQ_{32B,64B,128B}_sum (the
L2's fabric read requests by size; Infinity-Cache hits included), cross-
checked against FETCH_SIZE x 2 (MI355X_MICROARCH.md §HBM); writes =
WRITE_SIZE (exact for 16-B/lane stores).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stage_pmc import CODES, is_mark, load_pmc  # noqa: E402

B8_CONV6 = 8 * 64 * 64
F32_GEMM = lambda n: ((n.count("RowsKLoader<128, 256>") == 2 and "EpiStore" in n  # noqa: E731
                       and any(k in n for k in ("gemm_f32_kernel", "gemm_f32s_kernel", "gemm_f32h_kernel")))
                      or (any(k in n for k in ("gemm_h2_kernel<256, 256", "gemm_h2q_kernel<256, 256",
                                               "gemm_h2p_kernel<256, 256"))
                          and n.count("H2RowsDma<256, 8") >= 2
                          # not conv6's 1x1 forward GEMM (EpiStoreH): its 128x2 blocks of
                          # 512 threads equal the persistent grid's 256 x 512 in the PMC
                          # CSV's thread count, which round 4's summary averaged in
                          # (profiles/r05/pmc_calibration.json)
                          and "EpiStoreH" not in n and "EpiBnBwd" not in n))
# blocks x threads of conv6.conv.0's forward GEMM: the register-path kernels'
# 8x8x64 blocks of 256 threads, the h2 kernels' 4x4x64 blocks of 512, or the
# persistent h2 kernel's one block of 512 per CU (256 CUs)
F32_GRIDS = (8 * 8 * 64 * 256, 4 * 4 * 64 * 512, 256 * 512)
KINDS = {
    "f32_gemm": dict(match=F32_GEMM, grid=F32_GRIDS, triple=False,
                     alg=64 * (2 * 968 * 1024 + 1024 * 1024) * 4,
                     desc="conv6.conv.0 fwd Winograd F(6x6) batched GEMM, B=8 (64 x M=968 N=1024 "
                          "K=1024): gemm_h2p_kernel<256,256,2,4,H2RowsDma x2> (persistent, one block "
                          "per CU over the 4x4x64 tiles; gemm_h2q/h2_kernel grid 4x4x64 without it) "
                          "on the pre-split f16x2 operands (NSM_H2=1), or the register-path split kernel "
                          "grid 8x8x64; algorithmic bytes = V + U read + M written (fp32 bytes; "
                          "an h2 operand has the same)"),
    "f32": dict(match=F32_GEMM, grid=F32_GRIDS, triple=True,
                alg=(2 * B8_CONV6 * 1024 + 9 * 1024 * 1024 + 1024) * 4,
                desc="conv6.conv.0 fwd as a whole, B=8: wino_input + the GEMM above + "
                     "wino_output; algorithmic bytes = x + y + weights (direct conv)"),
    "bf16": dict(match=lambda n: "gemm_bf16_dma_kernel<256, 256" in n and "ConvActDma" in n,
                 grid=(4 * 1024 * 512,), triple=False,
                 alg=(2 * 262144 * 1024 + 9 * 1024 * 1024) * 2,
                 desc="conv6.conv.0 fwd bf16 LDS-DMA implicit GEMM, B=64: gemm_bf16_dma_kernel"
                      "<256,256,...,ConvActDma,RowsKDma,EpiStoreB> grid 4x1024 (M=262144 N=1024 "
                      "K=9216)"),
    # round 4: the bf16 path's conv6 forward is Winograd F(4x4) on f16 operands
    # (input transform + the single-plane persistent GEMM + output transform)
    "bf16_wino": dict(match=lambda n: ("gemm_h2p_kernel<256, 256" in n or "gemm_h2q_kernel<256, 256" in n)
                      and ", true>" in n,
                      grid=(256 * 512, 64 * 4 * 36 * 512), triple=True,
                      alg=(2 * 262144 * 1024 + 9 * 1024 * 1024) * 2,
                      desc="conv6.conv.0 fwd as a whole on the bf16 path, B=64: wino_input_f16 + "
                           "gemm_h2p_kernel<256,256,...,SP> + wino_output_kernel<4,...,bf16>; "
                           "algorithmic bytes = x + y + weights of the direct conv (bf16)"),
    "bf16_wino_gemm": dict(match=lambda n: ("gemm_h2p_kernel<256, 256" in n
                                            or "gemm_h2q_kernel<256, 256" in n)
                           and ", true>" in n,
                           grid=(256 * 512, 64 * 4 * 36 * 512), triple=False,
                           alg=36 * (16384 * 1024 * 2 + 1024 * 1024 * 2 + 16384 * 1024 * 2),
                           desc="conv6.conv.0 fwd's F(4x4) batched GEMM alone on the bf16 path, B=64 "
                                "(36 x M=16384 N=1024 K=1024, single-plane f16 V, U; f16 M, "
                                "nsm_wino_gemm_f16m): "
                                "algorithmic bytes = V + U read + M written"),
}
FWD = [c for c, n in CODES.items() if n == "conv6.fwd"][0]


def launches(path, k):
    """Counter dicts of the matching launches inside conv6.fwd (summed with the
    two neighbours for a triple), markers skipped."""
    disp = load_pmc(path)
    seq, cur = [], None
    for name, grid, (cnt, _) in disp:
        if is_mark(name):
            code = grid // 64 - 1
            cur = code if code else None
            continue
        seq.append((name, grid, cnt, cur))
    out, names = [], set()
    for i, (name, grid, cnt, cur) in enumerate(seq):
        if cur != FWD or not k["match"](name) or grid not in k["grid"]:
            continue
        if k["triple"]:
            tot = dict(cnt)
            for j in (i - 1, i + 1):
                names.add(seq[j][0][:60])
                for c, v in seq[j][2].items():
                    tot[c] = tot.get(c, 0.0) + v
            cnt = tot
        out.append(cnt)
    return out, names


def main():
    kind, outp, paths = sys.argv[1], sys.argv[2], sys.argv[3:]
    k = KINDS[kind]
    acc, n_by, names = {}, {}, set()
    for p in paths:
        ls, nm = launches(p, k)
        names |= nm
        for cnt in ls:
            for c, v in cnt.items():
                acc[c] = acc.get(c, 0.0) + v
                n_by[c] = n_by.get(c, 0) + 1
    avg = {c: acc[c] / n_by[c] for c in acc}
    out = {"kernel": k["desc"], "launches_sampled": max(n_by.values()) if n_by else 0,
           "counters_per_launch": avg, "algorithmic_bytes_per_launch": k["alg"],
           "neighbour_kernels": sorted(names)}
    if "TCC_EA0_RDREQ_128B_sum" in avg:
        rest = max(0.0, avg.get("TCC_EA0_RDREQ_sum", 0.0) - avg["TCC_EA0_RDREQ_32B_sum"]
                   - avg["TCC_EA0_RDREQ_64B_sum"] - avg["TCC_EA0_RDREQ_128B_sum"])
        out["read_bytes"] = (32 * avg["TCC_EA0_RDREQ_32B_sum"] + 64 * (avg["TCC_EA0_RDREQ_64B_sum"]
                             + rest) + 128 * avg["TCC_EA0_RDREQ_128B_sum"])
    if "FETCH_SIZE" in avg:
        out["fetch_bytes_x2"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        out["write_bytes"] = avg["WRITE_SIZE"] * 1024
    rd = out.get("read_bytes", out.get("fetch_bytes_x2"))
    if rd is not None and "write_bytes" in out:
        out["traffic_bytes_per_launch"] = rd + out["write_bytes"]
        out["traffic_over_algorithmic"] = round(out["traffic_bytes_per_launch"] / k["alg"], 3)
    out["note"] = ("reads from the sized fabric read requests (FETCH_SIZE x 2 beside them as the "
                   "guide's cross-check); Infinity-Cache hits are counted, not excluded")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from stage_pmc import stamp
    out["stamp"] = stamp()
    json.dump(out, open(outp, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
