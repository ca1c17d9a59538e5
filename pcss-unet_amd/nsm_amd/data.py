"""Input side of the hot path: the reference's `.npy` frame format and the
data-parallel sharding of it.

* `MmapLiverDataset` mirrors `setdata.MmapLiverDataset` (setdata.py:207-331):
  `{split}_inputs.npy` f32 [N,C,H,W] and `{split}_labels.npy` (f64 from
  prepare_dataset.py:47,71-72) memory-mapped; items are
  `((x - mean_c) / (std_c + 1e-8)) as f32 [C,H,W]` (requires_grad, like
  setdata.py:325-326) and `label as f32 [1,H,W]`. Stats come from
  `train_stats.json` (calculate_dataset_stats.py:93-95) or the pickled
  `train_stats.npy` the reference writes. Unlike the reference (hard-coded 4
  channels, setdata.py:271,316) any channel count works (7-ch G-buffers).
* `shard_range` / `ShardedFrames`: plain data parallelism — rank r owns the
  contiguous frame slice [r*N/W, (r+1)*N/W) (the reference iterates in order,
  shuffle=False, main.py:850) and serves batches already resident on its GPU.
"""
import json
import os

import numpy as np
import torch


def load_stats(stats_dir, channels=None):
    js = os.path.join(stats_dir, "train_stats.json")
    npy = os.path.join(stats_dir, "train_stats.npy")
    st = None
    if os.path.exists(js):
        with open(js) as f:
            st = json.load(f)
    elif os.path.exists(npy):
        # the reference's own stats file is a pickled dict (calculate_dataset_stats.py:88-92)
        st = np.load(npy, allow_pickle=True).item()
    if not st or "means" not in st or "stds" not in st:
        return None
    if channels is not None and len(st["means"]) != channels:
        return None
    return (torch.tensor(st["means"], dtype=torch.float32),
            torch.tensor(st["stds"], dtype=torch.float32))


class MmapLiverDataset(torch.utils.data.Dataset):
    EPS = 1e-8

    def __init__(self, data_dir, split="train", stats_dir=None, transform=None,
                 target_transform=None, apply_normalization=True):
        stats_dir = stats_dir or data_dir
        self.inputs_path = os.path.join(data_dir, f"{split}_inputs.npy")
        self.labels_path = os.path.join(data_dir, f"{split}_labels.npy")
        for p in (self.inputs_path, self.labels_path):
            if not os.path.exists(p):
                raise FileNotFoundError(p)
        self.split = split
        self.inputs = np.load(self.inputs_path, mmap_mode="r")
        self.labels = np.load(self.labels_path, mmap_mode="r")
        if self.inputs.shape[0] != self.labels.shape[0]:
            raise ValueError("inputs/labels count mismatch")
        self.transform, self.target_transform = transform, target_transform
        self.apply_normalization = apply_normalization
        C = self.inputs.shape[1]
        self.means = torch.zeros(C)
        self.stds = torch.ones(C)
        if apply_normalization:
            st = load_stats(stats_dir, C)
            if st is not None:
                self.means, self.stds = st

    def __len__(self):
        return len(self.inputs)

    def __getitem__(self, index):
        x = torch.from_numpy(self.inputs[index].astype(np.float32))
        y = torch.from_numpy(self.labels[index].astype(np.float32))
        if self.apply_normalization:
            C = x.shape[0]
            x = (x - self.means.view(C, 1, 1)) / (self.stds.view(C, 1, 1) + self.EPS)
        if self.transform is not None:
            x = self.transform(x)
        if self.target_transform is not None:
            y = self.target_transform(y)
        x = x.detach().clone().requires_grad_(True)
        return x, y


def shard_range(n, world, rank):
    """Contiguous slice of n frames owned by `rank` (balanced to +-1 frame)."""
    lo = rank * n // world
    hi = (rank + 1) * n // world
    return lo, hi


class ShardedFrames:
    """Per-rank batch iterator over a dataset's contiguous shard; batches are
    moved to `device` with a non-blocking copy from pinned memory."""

    def __init__(self, dataset, batch_size, world=1, rank=0, device=None, drop_last=True):
        self.ds, self.bs, self.device, self.drop_last = dataset, batch_size, device, drop_last
        self.lo, self.hi = shard_range(len(dataset), world, rank)

    def __len__(self):
        n = self.hi - self.lo
        return n // self.bs if self.drop_last else -(-n // self.bs)

    def __iter__(self):
        for b in range(len(self)):
            idx = range(self.lo + b * self.bs, min(self.hi, self.lo + (b + 1) * self.bs))
            xs, ys = zip(*(self.ds[i] for i in idx))
            x = torch.stack([t.detach() for t in xs])
            y = torch.stack(ys)
            if self.device is not None and self.device.type == "cuda":
                x = x.pin_memory().to(self.device, non_blocking=True)
                y = y.pin_memory().to(self.device, non_blocking=True)
            yield x.requires_grad_(True), y
