#!/usr/bin/env python3
"""float64 simulation of the bf16 path's F(4x4) Winograd 3x3 with f16 operands
and f16 M (csrc nsm_wino_gemm_f16m / nsm_wino_output_bf16m): the error against
the exact convolution of the same bf16 input, with M rounded under the static
bound (C * bound_V * bound_U, as the kernel's 2^-(15 + ceil log2 K)) and under
its exact maximum, beside fp32 M and the direct conv's bf16 output rounding.
DESIGN.md "bf16: Winograd M in f16". CPU only, ~10 s."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wino_coeffs import mats  # noqa: E402


def bf(x):
    """round to bf16 (nearest even), as float64"""
    x = np.asarray(x, np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).astype(np.float64)


def f16s(x, bound):
    """f16 under the power-of-two scale 2^(15 - ceil log2 bound)"""
    s = 2.0 ** (15 - int(np.ceil(np.log2(bound))))
    return (x * s).astype(np.float16).astype(np.float64) / s


def main(C=256, K=256, H=16, W=16, B=2, seed=0):
    AT, G, BT = (np.array(M, dtype=np.float64) for M in mats(4))
    rng = np.random.default_rng(seed)
    x = bf(np.maximum(rng.standard_normal((B, C, H, W)), 0))
    w = bf(rng.standard_normal((K, C, 3, 3)) * np.sqrt(2 / (9 * C)))
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)))
    ref = np.zeros((B, K, H, W))
    for dy in range(3):
        for dx in range(3):
            ref += np.einsum('bchw,kc->bkhw', xp[:, :, dy:dy + H, dx:dx + W], w[:, :, dy, dx])
    T = H // 4
    d = np.zeros((B, C, T, T, 6, 6))
    for ty in range(T):
        for tx in range(T):
            d[:, :, ty, tx] = xp[:, :, 4 * ty:4 * ty + 6, 4 * tx:4 * tx + 6]
    V = np.einsum('ij,bcyxjk,lk->bcyxil', BT, d, BT)
    U = np.einsum('ij,kcjl,ml->kcim', G, w, G)
    bV = np.abs(x).max() * np.abs(BT).sum(1).max() ** 2
    bU = np.abs(w).max() * np.abs(G).sum(1).max() ** 2
    M = np.einsum('bcyxij,kcij->bkyxij', f16s(V, bV), f16s(U, bU))

    def out(Mq):
        y = np.einsum('ai,bkyxij,cj->bkyxac', AT, Mq, AT)
        return y.transpose(0, 1, 2, 4, 3, 5).reshape(B, K, H, W)

    def err(y):
        e = bf(y) - ref
        return np.sqrt((e ** 2).mean()), np.abs(e).max()

    print(f"direct (bf16 output rounding only): rms {err(ref)[0]:.3e} max {err(ref)[1]:.3e}")
    print(f"F(4x4), f16 V/U, fp32 M:            rms {err(out(M.astype(np.float32)))[0]:.3e} "
          f"max {err(out(M.astype(np.float32)))[1]:.3e}")
    for name, bound in (("static bound C*bV*bU", C * bV * bU), ("exact max|M|", np.abs(M).max())):
        r, m = err(out(f16s(M, bound)))
        print(f"F(4x4), f16 M, {name:22s} rms {r:.3e} max {m:.3e} "
              f"(slack 2^{np.log2(bound / np.abs(M).max()):.1f})")


if __name__ == "__main__":
    main()
