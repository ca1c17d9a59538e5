#!/usr/bin/env python3
"""Exact Cook-Toom matrices for Winograd F(m x m, 3x3) (Lavin & Gray 2016 construction).

Finite interpolation points p_0..p_{n-2} plus the point at infinity, n = m + 2:
  A^T[i][j] = p_j^i,                     A^T[i][n-1] = [i == m-1]
  G[j][k]   = p_j^k / prod_{l!=j}(p_j-p_l),  G[n-1][k] = [k == 2]
  B^T[j]    = coefficients (x^0..x^{n-1}) of prod_{l!=j}(x - p_l);  B^T[n-1] = of prod_l (x - p_l)
F(2x2): points (0, 1, -1); F(4x4): points (0, 1, -1, 1/2, -2), which in fp32 gives
~3x less error than the textbook (0, +-1, +-2) set (measured: tools/wino_coeffs.py --check);
F(6x6): points (0, +-1, +-2, +-1/2): 8.8e-6 rms vs 2.9e-6 (F4) and 4.0e-7 (direct) on a
512-channel fp32 layer with O(1) outputs (the lowest of the 7-point sets tried).
Prints the C++ tables used in pcss-unet_amd/csrc/nsm_conv.hip (WinoMats<m>).
"""
import sys
from fractions import Fraction as Fr

import numpy as np

POINTS = {2: [Fr(0), Fr(1), Fr(-1)], 4: [Fr(0), Fr(1), Fr(-1), Fr(1, 2), Fr(-2)],
          6: [Fr(0), Fr(1), Fr(-1), Fr(2), Fr(-2), Fr(1, 2), Fr(-1, 2)]}


def polymul(a, b):
    out = [Fr(0)] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            out[i + j] += x * y
    return out


def mats(m):
    p = POINTS[m]
    n = m + 2
    AT = [[p[j] ** i if j < n - 1 else Fr(int(i == m - 1)) for j in range(n)] for i in range(m)]
    G = []
    for j in range(n - 1):
        N = Fr(1)
        for q in p:
            if q != p[j]:
                N *= p[j] - q
        G.append([p[j] ** k / N for k in range(3)])
    G.append([Fr(0), Fr(0), Fr(1)])
    BT = []
    for j in range(n):
        poly = [Fr(1)]
        for l, q in enumerate(p):
            if l != j:
                poly = polymul(poly, [-q, Fr(1)])
        poly = poly + [Fr(0)] * (n - len(poly))
        BT.append(poly)
    return AT, G, BT


def check(m):
    """float64 exactness of the 2-D algorithm against direct correlation."""
    AT, G, BT = (np.array(M, dtype=np.float64) for M in mats(m))
    rng = np.random.default_rng(0)
    d = rng.standard_normal((m + 2, m + 2))
    g = rng.standard_normal((3, 3))
    y = AT @ ((G @ g @ G.T) * (BT @ d @ BT.T)) @ AT.T
    ref = np.array([[np.sum(d[i:i + 3, j:j + 3] * g) for j in range(m)] for i in range(m)])
    return np.abs(y - ref).max()


def cxx(name, M):
    rows = ",\n      ".join("{" + ", ".join(f"{float(v)!r}f" for v in r) + "}" for r in M)
    return f"  static constexpr float {name}[{len(M)}][{len(M[0])}] = {{\n      {rows}}};"


if __name__ == "__main__":
    for m in (2, 4, 6):
        assert check(m) < 1e-12, m
        AT, G, BT = mats(m)
        print(f"// F({m}x{m},3x3), points {[str(v) for v in POINTS[m]]} + inf")
        print(cxx("AT", AT))
        print(cxx("G", G))
        print(cxx("BT", BT))
    if "--check" in sys.argv:
        print("exactness ok")
