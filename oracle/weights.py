"""TEST INFRASTRUCTURE ONLY — deterministic parameter recipe shared by the
golden-fixture generator, the oracle and the parity tests.

The reference ships no checkpoint, so parity runs on synthetic weights made
by a documented numpy PCG64 recipe:

  * conv weight / bias  ~ U(-1/sqrt(fan_in), +1/sqrt(fan_in))
  * BN gamma ~ U(0.75, 1.25), BN beta ~ U(-0.1, 0.1)   (non-trivial affine)
  * BN running_mean = 0, running_var = 1, num_batches_tracked = 0

drawn in state_dict key order from `numpy.random.default_rng(seed)`.
Key order and shapes follow the reference's `Unet.__init__`
(`/root/reference/Unetmodel.py:36-63`, DoubleConv at `:17-33`).
"""
from collections import OrderedDict

import numpy as np

# (in, out) channels of conv2..conv9 for in_ch=4; conv2 generalises to 4*in_ch.
# Unetmodel.py:39,42,45,48,52,55,58,61
BLOCK_CHANNELS = {2: (16, 64), 3: (64, 128), 4: (128, 512), 5: (512, 1024),
                  6: (1024, 512), 7: (512, 128), 8: (128, 64), 9: (64, 16)}


def block_channels(in_ch=4):
    ch = dict(BLOCK_CHANNELS)
    ch[2] = (4 * in_ch, 64)
    return ch


def state_dict_spec(in_ch=4):
    """Ordered (key, shape, dtype) list identical to the reference state_dict."""
    spec = []
    for k, (ci, co) in block_channels(in_ch).items():
        p = f"conv{k}.conv."
        spec += [(p + "0.weight", (ci, ci, 3, 3), "f4"), (p + "0.bias", (ci,), "f4")]
        for n in ("weight", "bias", "running_mean", "running_var"):
            spec.append((p + "1." + n, (ci,), "f4"))
        spec.append((p + "1.num_batches_tracked", (), "i8"))
        spec += [(p + "4.weight", (co, ci, 1, 1), "f4"), (p + "4.bias", (co,), "f4")]
        for n in ("weight", "bias", "running_mean", "running_var"):
            spec.append((p + "5." + n, (co,), "f4"))
        spec.append((p + "5.num_batches_tracked", (), "i8"))
    spec += [("conv10.weight", (4, 16, 1, 1), "f4"), ("conv10.bias", (4,), "f4")]
    return spec


def make_state(in_ch=4, seed=42):
    """numpy state_dict (OrderedDict) from the recipe above."""
    rng = np.random.default_rng(seed)
    sd = OrderedDict()
    fan_in = None
    for key, shape, dt in state_dict_spec(in_ch):
        leaf = key.rsplit(".", 1)[1]
        is_bn = (".1." in key or ".5." in key)
        if dt == "i8":
            sd[key] = np.zeros(shape, np.int64)
        elif not is_bn and leaf == "weight":
            fan_in = int(np.prod(shape[1:]))
            b = 1.0 / np.sqrt(fan_in)
            sd[key] = rng.uniform(-b, b, shape).astype(np.float32)
        elif not is_bn and leaf == "bias":
            b = 1.0 / np.sqrt(fan_in)
            sd[key] = rng.uniform(-b, b, shape).astype(np.float32)
        elif leaf == "weight":
            sd[key] = rng.uniform(0.75, 1.25, shape).astype(np.float32)
        elif leaf == "bias":
            sd[key] = rng.uniform(-0.1, 0.1, shape).astype(np.float32)
        elif leaf == "running_mean":
            sd[key] = np.zeros(shape, np.float32)
        elif leaf == "running_var":
            sd[key] = np.ones(shape, np.float32)
        else:
            raise KeyError(key)
    return sd


def synthetic_batch(batch, in_ch, h, w, seed_x=0, seed_y=1):
    """Synthetic G-buffer batch per SURVEY.md §8(d): x ~ N(0,1) (the
    post-normalisation distribution of setdata.py:316), labels =
    integers(0,256)/255 (PNG ground truth quantisation, prepare_dataset.py:47)."""
    x = np.random.default_rng(seed_x).standard_normal((batch, in_ch, h, w)).astype(np.float32)
    y = (np.random.default_rng(seed_y).integers(0, 256, (batch, 1, h - h % 2, w - w % 2)) / 255.0).astype(np.float32)
    return x, y
