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
