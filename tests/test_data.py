"""CPU: the .npy frame loader mirror against the reference's
MmapLiverDataset output (fixture made by running setdata.py), and the
native .npy header parser of the frame loader."""
import json
import os

import numpy as np
import pytest
import torch

from util import load


def _write(tmp_path, fx, stats="json"):
    np.save(tmp_path / "train_inputs.npy", fx["inputs"])
    np.save(tmp_path / "train_labels.npy", fx["labels"])
    st = {"means": fx["means"].tolist(), "stds": fx["stds"].tolist()}
    if stats == "npy":   # what calculate_dataset_stats.py writes besides the json
        np.save(tmp_path / "train_stats.npy", st, allow_pickle=True)
    else:
        (tmp_path / "train_stats.json").write_text(json.dumps(st))


def test_mmap_dataset_matches_reference_bitwise(tmp_path):
    from nsm_amd.data import MmapLiverDataset
    fx = load("mmap_norm")
    _write(tmp_path, fx, "json")
    ds = MmapLiverDataset(str(tmp_path), "train")
    xs, ys = zip(*[ds[i] for i in range(len(ds))])
    assert all(x.requires_grad for x in xs)
    assert np.array_equal(torch.stack(xs).detach().numpy(), fx["x"])
    assert np.array_equal(torch.stack(ys).numpy(), fx["y"])
    assert ys[0].dtype == torch.float32


def test_pickled_stats_are_refused(tmp_path):
    """train_stats.npy is a pickle: never loaded; the json twin is required."""
    from nsm_amd.data import MmapLiverDataset
    fx = load("mmap_norm")
    _write(tmp_path, fx, "npy")
    with pytest.raises(FileNotFoundError, match="train_stats.json"):
        MmapLiverDataset(str(tmp_path), "train")


def test_sharded_frames_cover_dataset(tmp_path):
    from nsm_amd.data import MmapLiverDataset, ShardedFrames
    fx = load("mmap_norm")
    _write(tmp_path, fx)
    ds = MmapLiverDataset(str(tmp_path), "train")
    seen = []
    for r in range(2):
        for x, y in ShardedFrames(ds, 1, world=2, rank=r, drop_last=False):
            seen.append(x.detach())
    assert len(seen) == 3
    assert np.array_equal(torch.cat(seen).numpy(), fx["x"])


@pytest.mark.parametrize("dtype,shape", [(np.float32, (3, 7, 8, 10)), (np.float64, (3, 1, 8, 10)),
                                         (np.float32, (5,))])
def test_native_npy_header(tmp_path, dtype, shape):
    """nsm_npy_info (the frame loader's parser) on files numpy writes."""
    import ctypes
    from nsm_amd._lib import lib
    path = os.path.join(tmp_path, "a.npy")
    a = np.arange(int(np.prod(shape)), dtype=dtype).reshape(shape)
    np.save(path, a)
    sh = (ctypes.c_int64 * 8)()
    nd, dt, off = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    rc = lib.nsm_npy_info(path.encode(), sh, 8, ctypes.byref(nd), ctypes.byref(dt), ctypes.byref(off))
    assert rc == 0
    assert tuple(sh[:nd.value]) == shape
    assert dt.value == (0 if dtype == np.float32 else 1)
    raw = open(path, "rb").read()
    assert np.array_equal(np.frombuffer(raw[off.value:], dtype=dtype).reshape(shape), a)
    np.save(path, a.astype(np.int32))
    assert lib.nsm_npy_info(path.encode(), sh, 8, ctypes.byref(nd), ctypes.byref(dt), None) != 0
