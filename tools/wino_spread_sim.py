#!/usr/bin/env python3
"""float64 simulation behind DESIGN.md "bf16 parity under spread scales": the
per-output-channel relative error of one 3x3 convolution under channel scales
2^U(-12, 0) (input channels and output channels, as tests/test_gpu_configs.py's
spread case), for
  * the reference's bf16 autocast: bf16 input and weights, fp32 sums, bf16 out;
  * this repo's bf16 path: F(4x4) Winograd, V / U in f16 under one power-of-two
    scale per tensor, M in f16 under one exponent per 64 x 64 tile, bf16 out;
  * the same with one U exponent per output channel;
  * the same with fp32 M.
Errors are against the exact float64 convolution of the unrounded operands.
CPU only: python tools/wino_spread_sim.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from wino_coeffs import mats  # noqa: E402
from wino_m16_sim import bf  # noqa: E402


def f16_pow2(x, amax):
    """f16 under the scale 2^(15 - ceil log2 amax) (amax broadcastable)"""
    s = 2.0 ** (15 - np.ceil(np.log2(np.maximum(amax, 1e-300))))
    return (x * s).astype(np.float16).astype(np.float64) / s


def conv_direct(xp, w, H, W):
    out = np.zeros((xp.shape[0], w.shape[0], H, W))
    for dy in range(3):
        for dx in range(3):
            out += np.einsum('bchw,kc->bkhw', xp[:, :, dy:dy + H, dx:dx + W], w[:, :, dy, dx])
    return out


def main(C=128, K=128, H=32, W=32, B=2, seed=0):
    AT, G, BT = (np.array(M, dtype=np.float64) for M in mats(4))
    rng = np.random.default_rng(seed)
    cin = 2.0 ** rng.uniform(-12, 0, C)
    cout = 2.0 ** rng.uniform(-12, 0, K)
    x = np.maximum(rng.standard_normal((B, C, H, W)), 0) * cin[None, :, None, None]
    w = rng.standard_normal((K, C, 3, 3)) * np.sqrt(2 / (9 * C)) * cout[:, None, None, None]
    pad = ((0, 0), (0, 0), (1, 1), (1, 1))
    exact = conv_direct(np.pad(x, pad), w, H, W)
    # the reference's autocast
    ref = bf(conv_direct(np.pad(bf(x), pad), bf(w), H, W))
    # this repo: activations stored bf16, Winograd on f16 operands
    xb = bf(x)
    xp = np.pad(xb, pad)
    T = H // 4
    d = np.zeros((B, C, T, T, 6, 6))
    for ty in range(T):
        for tx in range(T):
            d[:, :, ty, tx] = xp[:, :, 4 * ty:4 * ty + 6, 4 * tx:4 * tx + 6]
    V = np.einsum('ij,bcyxjk,lk->bcyxil', BT, d, BT)
    U = np.einsum('ij,kcjl,ml->kcim', G, w, G)
    Vq = f16_pow2(V, np.abs(V).max())
    variants = {"U one scale": f16_pow2(U, np.abs(U).max()),
                "U per output channel": f16_pow2(U, np.abs(U).reshape(K, -1).max(1)[:, None, None, None])}

    def out(Mq):
        y = np.einsum('ai,bkyxij,cj->bkyxac', AT, Mq, AT)
        return bf(y.transpose(0, 1, 2, 4, 3, 5).reshape(B, K, H, W))

    def m16(M):  # one exponent per 64 tiles x 64 output channels of each component
        Mr = M.transpose(0, 2, 3, 1, 4, 5).reshape(B * T * T, K, 6, 6)
        q = np.empty_like(Mr)
        for r in range(0, Mr.shape[0], 64):
            for k in range(0, K, 64):
                blk = Mr[r:r + 64, k:k + 64]
                q[r:r + 64, k:k + 64] = f16_pow2(blk, np.abs(blk).max(axis=(0, 1)))
        return q.reshape(B, T, T, K, 6, 6).transpose(0, 3, 1, 2, 4, 5)

    def per_channel(y):
        e = np.sqrt(((y - exact) ** 2).mean(axis=(0, 2, 3)))
        return e / np.sqrt((exact ** 2).mean(axis=(0, 2, 3)))

    r_ref = per_channel(ref)
    print(f"reference bf16 autocast: median per-channel rel error {np.median(r_ref):.3e}")
    for name, Uq in variants.items():
        M = np.einsum('bcyxij,kcij->bkyxij', Vq, Uq)
        for mname, Mq in (("f16 M (tile exponent)", m16(M)), ("fp32 M", M.astype(np.float32))):
            r = per_channel(out(Mq)) / r_ref
            print(f"F(4x4) {name:22s} {mname:22s}: error / reference per channel: "
                  f"median {np.median(r):.3f} max {r.max():.3f}")


if __name__ == "__main__":
    main()
