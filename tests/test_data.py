"""CPU: the .npy frame loader mirror against the reference's
MmapLiverDataset output (fixture made by running setdata.py)."""
import json

import numpy as np
import torch

from util import load


def _write(tmp_path, fx, stats="npy"):
    np.save(tmp_path / "train_inputs.npy", fx["inputs"])
    np.save(tmp_path / "train_labels.npy", fx["labels"])
    st = {"means": fx["means"].tolist(), "stds": fx["stds"].tolist()}
    if stats == "npy":
        np.save(tmp_path / "train_stats.npy", st)
    else:
        (tmp_path / "train_stats.json").write_text(json.dumps(st))


def test_mmap_dataset_matches_reference_bitwise(tmp_path):
    from nsm_amd.data import MmapLiverDataset
    fx = load("mmap_norm")
    for stats in ("npy", "json"):
        _write(tmp_path, fx, stats)
        ds = MmapLiverDataset(str(tmp_path), "train")
        xs, ys = zip(*[ds[i] for i in range(len(ds))])
        assert all(x.requires_grad for x in xs)
        assert np.array_equal(torch.stack(xs).detach().numpy(), fx["x"])
        assert np.array_equal(torch.stack(ys).numpy(), fx["y"])
        assert ys[0].dtype == torch.float32


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
