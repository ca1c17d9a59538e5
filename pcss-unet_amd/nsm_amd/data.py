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
* `FrameLoader`: the same frames through the native loader (libnsm
  nsm_loader_*: mmap + host threads staging upcoming batches in pinned
  memory + async H2D on the compute stream), normalised on the GPU
  (nsm_normalize_frames) — the production input path.
"""
import json
import os

import numpy as np
import torch


def load_stats(stats_dir, channels=None):
    js = os.path.join(stats_dir, "train_stats.json")
    st = None
    if os.path.exists(js):
        with open(js) as f:
            st = json.load(f)
    elif os.path.exists(os.path.join(stats_dir, "train_stats.npy")):
        raise FileNotFoundError(
            f"{js} not found: only the pickled train_stats.npy is present, and pickles are not "
            "loaded; calculate_dataset_stats.py writes train_stats.json with the same content")
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


class FrameLoader:
    """Batches (x [b,C,H,W] normalised f32 requiring grad, y [b,1,H,W] f32) of
    this rank's shard, resident on `device`, in the reference's order; loops
    over epochs. len() = batches per epoch."""

    def __init__(self, data_dir, split="train", batch=8, device="cuda", world=1, rank=0,
                 stats_dir=None, apply_normalization=True, slots=3, threads=4):
        from ._lib import NsmError, call, last_error, lib
        self._lib, self._call = lib, call
        self.device = torch.device(device)
        xin = os.path.join(data_dir, f"{split}_inputs.npy")
        yin = os.path.join(data_dir, f"{split}_labels.npy")
        h = lib.nsm_loader_create(xin.encode(), yin.encode(), batch, rank, world, slots, threads)
        if not h:
            raise NsmError(f"nsm_loader_create failed: {last_error()}")
        self._h = h
        import ctypes
        c, hh, ww = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        call("nsm_loader_frame_dims", h, ctypes.byref(c), ctypes.byref(hh), ctypes.byref(ww))
        self.C, self.H, self.W = c.value, hh.value, ww.value
        self.batch = batch
        self.nbatches = int(lib.nsm_loader_batches(h))
        self.norm = None
        if apply_normalization:
            st = load_stats(stats_dir or data_dir, self.C)
            if st is not None:
                self.norm = (st[0].to(self.device), st[1].to(self.device))

    def __len__(self):
        return self.nbatches

    def next(self):
        from ._lib import NsmError, last_error, ptr, stream
        x = torch.empty(self.batch, self.C, self.H, self.W, dtype=torch.float32, device=self.device)
        y = torch.empty(self.batch, 1, self.H, self.W, dtype=torch.float32, device=self.device)
        n = self._lib.nsm_loader_next(self._h, ptr(x), ptr(y), stream())
        if n < 0:
            raise NsmError(f"nsm_loader_next failed: {last_error()}")
        x, y = x[:n], y[:n]
        if self.norm is not None:
            self._call("nsm_normalize_frames", ptr(x), n, self.C, self.H * self.W, ptr(self.norm[0]),
                       ptr(self.norm[1]), MmapLiverDataset.EPS, stream())
        return x.requires_grad_(True), y

    def __iter__(self):
        for _ in range(self.nbatches):
            yield self.next()

    def close(self):
        if getattr(self, "_h", None):
            # the staged copies ran on the current stream: let them land first
            torch.cuda.current_stream(self.device).synchronize()
            self._lib.nsm_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
