"""Shared helpers for parity tests (test infrastructure)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# tolerances (grounded in measured CPU-backend noise floors)
OUT_ABS = 1e-4        # fp32 output max-abs
LOSS_REL = 1e-5       # fp32 loss
GRAD_REL_L2 = 2e-2    # per-tensor gradient rel-L2
PRE_BN_BIAS_ABS = 1e-6  # conv biases feeding train-mode BN: grad is 0 analytically
RUN_TOL = 1e-4        # running stats


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


def proj_vector(idx, n):
    return np.random.default_rng([7, idx]).standard_normal(n).astype(np.float32)


def is_pre_bn_bias(key):
    return key.endswith(".0.bias") or key.endswith(".4.bias")


def check_grads(named_grads, fx, report=None):
    """Compare a list of (key, grad ndarray) in named_parameters order with a
    fixture's grad summary. Returns list of failures."""
    fails = []
    for idx, (k, g) in enumerate(named_grads):
        g = np.asarray(g, np.float64).ravel()
        if "g/" + k in fx:
            r = fx["g/" + k].astype(np.float64)
            if is_pre_bn_bias(k):
                err = np.abs(g - r).max()
                ok = err <= PRE_BN_BIAS_ABS
            else:
                err = np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)
                ok = err <= GRAD_REL_L2
        else:
            l2r = float(fx[f"g/{k}/l2"])
            l2 = np.sqrt((g * g).sum())
            pj = (g * proj_vector(idx, g.size)).sum()
            e1 = abs(l2 - l2r) / l2r
            e2 = abs(pj - float(fx[f"g/{k}/proj"])) / l2r
            head = fx[f"g/{k}/head"].astype(np.float64)
            e3 = np.linalg.norm(g[:64] - head) / max(np.linalg.norm(head), 1e-30)
            err = max(e1, e2)
            ok = e1 <= GRAD_REL_L2 and e2 <= 2 * GRAD_REL_L2 and e3 <= 5 * GRAD_REL_L2
        if report is not None:
            report.append((k, float(err)))
        if not ok:
            fails.append((k, float(err)))
    return fails
