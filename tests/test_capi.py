"""CPU: the C-ABI library loads and exports every entry point include/nsm.h
declares; host-side helpers (fast division, tile/workspace planning)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nsm.h")
LIB = os.path.join(ROOT, "pcss-unet_amd", "nsm_amd", "libnsm.so")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nsm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    syms = declared_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    import nsm_amd._lib as L
    assert sorted(L.symbols()) == declared_symbols()
    assert L.lib.nsm_version() == 1


def test_error_path_without_gpu_work():
    """Argument validation fails before any launch, with a readable message."""
    import nsm_amd._lib as L
    rc = L.lib.nsm_conv_fwd(None, 0, 1, 1, 1, 32, None, None, 32, 3, None, 32, None, None, None,
                            0.2, None)
    assert rc == 1
    assert "null" in L.last_error()


def test_wgrad_workspace_plan():
    import nsm_amd._lib as L
    # conv6 3x3 at B=8, 64x64: M=1024, N=9216
    n = L.lib.nsm_conv_wgrad_ws(8, 64, 64, 1024, 1024, 3)
    assert n % (1024 * 9216) == 0 and n >= 1024 * 9216
    assert L.lib.nsm_reduce_chunks(524288, 32) >= 1


def fastdiv(n, d):
    """Python replica of nsm::make_fastdiv / fdiv (nsm_common.h)."""
    if d <= 1:
        return n
    l = (d - 1).bit_length()
    p = 31 + l
    mul = ((1 << p) + d - 1) // d
    return ((n * mul) >> 32) >> (p - 32)


def test_fastdiv_exact():
    rng = np.random.default_rng(0)
    for d in list(range(1, 300)) + [540, 960, 1080, 1920, 65536, 262144, 1 << 20]:
        ns = list(range(0, 2000)) + [int(v) for v in rng.integers(0, 2**31, 2000)] + [2**31 - 1]
        for n in ns:
            assert fastdiv(n, d) == n // d, (n, d)


def test_tail_plan_blocks_never_straddle_parameters():
    """nsm_tail_plan (host): blocks of nsm_tail_chunk() elements, one parameter
    each, covering the flat buffer in order."""
    import nsm_amd._lib as L
    sizes = [1728, 16, 512, 37, 9000, 4, 1, 9, 9437184]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    seg_off = (ctypes.c_int64 * len(offs))(*offs.tolist())
    nseg = len(sizes)
    nblk = L.lib.nsm_tail_plan(seg_off, nseg, None, None, None, None, 0)
    ch = L.lib.nsm_tail_chunk()
    assert nblk == sum(-(-s // ch) for s in sizes)
    bs, lo, hi = (ctypes.c_int * nblk)(), (ctypes.c_int64 * nblk)(), (ctypes.c_int64 * nblk)()
    sb = (ctypes.c_int * (nseg + 1))()
    assert L.lib.nsm_tail_plan(seg_off, nseg, bs, lo, hi, sb, nblk) == nblk
    assert lo[0] == 0 and hi[nblk - 1] == offs[-1]
    for b in range(nblk):
        s = bs[b]
        assert offs[s] <= lo[b] < hi[b] <= offs[s + 1] and hi[b] - lo[b] <= ch
        if b:
            assert lo[b] == hi[b - 1]
    assert [sb[s] for s in range(nseg + 1)] == [0] + list(np.cumsum([-(-s // ch) for s in sizes]))
    assert L.lib.nsm_tail_ws_bytes(nseg, nblk) > 0
