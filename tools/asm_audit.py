#!/usr/bin/env python3
"""Audit the gfx950 assembly of libnsm kernels: per kernel (name filter), the
MFMA / LDS-DMA / ds_read counts, scratch use, register counts and the vmcnt
waits hipcc emitted (a vmcnt(0) inside a DMA-pipelined K loop drains it).

    python tools/asm_audit.py [name-substring] [source.hip]
Builds with -save-temps into /tmp/nsm_asm (nothing written in the repo).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pcss-unet_amd", "csrc")


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else "dma"
    src = sys.argv[2] if len(sys.argv) > 2 else "nsm_conv.hip"
    out = "/tmp/nsm_asm"
    os.makedirs(out, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-Wno-unused-function", "-Wno-unused-variable", "-munsafe-fp-atomics", "-c",
                    os.path.join(CSRC, src), "-o", os.path.join(out, "x.o"), "-save-temps"],
                   cwd=out, check=True, stderr=subprocess.DEVNULL)
    base = os.path.splitext(src)[0]
    s = open(os.path.join(out, f"{base}-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    for m in re.finditer(r"^(_Z\S+):[ \t]*(?:;.*)?$", s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        body = s[m.end():s.find(".Lfunc_end", m.end())]
        md = s[s.find(".name:           " + name):]
        md = md[:md.find("\n  - ")] if "\n  - " in md else md[:4000]

        def meta(k):
            r = re.search(r"\." + k + r":\s+(\d+)", md)
            return r.group(1) if r else "?"
        waits = re.findall(r"s_waitcnt[^\n]*vmcnt\(\d+\)", body)
        ndma = len(re.findall(r"buffer_load_dwordx4[^\n]*lds", body))
        nds = len(re.findall(r"ds_read", body))
        print(f"{name[:110]}\n  lines={body.count(chr(10))} mfma={body.count('v_mfma')} "
              f"dma={ndma} ds_read={nds} scratch={body.count('scratch_')} "
              f"vgpr={meta('vgpr_count')} agpr={meta('agpr_count')} sgpr={meta('sgpr_count')} "
              f"lds={meta('group_segment_fixed_size')} spill={meta('vgpr_spill_count')}\n"
              f"  vmcnt waits: {waits[:16]}")


if __name__ == "__main__":
    main()
