"""Train-step tail on libnsm kernels over ONE flat parameter buffer, and the
data-parallel gradient all-reduce.

Reference step tail (main.py:281-423, optimizer/scheduler main.py:952-969):

    backward -> [sanitise: NaN/Inf census, skip if >20 % of a tensor is bad,
    else repair NaN->mean+noise, Inf->+-10*max (:287-354)] -> per-parameter
    pre-unscale clip to 1000*scale (:361-365) -> unscale_ -> per-parameter
    NaN/Inf skip, norm > 1e5 skip, norm > 1e3 rescale to 1e3 (:368-402) ->
    clip_grad_norm_(max_norm) with max_norm = 1.0, or max(0.1, 1-epoch/E)
    after half the epochs (:357-358,405) -> skip if a clipped norm > 10
    (:408-418) -> AdamW step (:421) ; LambdaLR warmup + cosine (:959-969).

`FlatAdamW(..., sanitize=True)` runs all of that on the device as a fixed
sequence of five kernels (include/nsm.h `nsm_grad_tail` + `nsm_adamw_tail`):
every decision the reference takes on the host becomes a device flag that the
next kernel reads, the AdamW step count lives on the device (a skipped step
does not advance it, exactly like a `continue` before `optimizer.step()`), and
nothing synchronises with the host. `sanitize=False` is the plain
clip_grad_norm_ + AdamW tail.

`FlatAdamW` re-homes the parameters into a single contiguous fp32 buffer
(views keep the module's parameter objects, so state_dict / LambdaLR /
named_parameters are unchanged). The Unet backward writes all 66 gradients
into one flat buffer too, so the DP exchange is one all-reduce of 60 MiB.
`state_dict()` / `load_state_dict()` use torch.optim.AdamW's format, so
main.py's `optimizer_state_dict` checkpoints interchange.
"""
import math
import os

import torch
import torch.distributed as dist

from ._lib import call, lib, ptr, stream


def flat_grad(params):
    """The flat tensor backing all .grad views (in parameter order), or None."""
    gs = [p.grad for p in params]
    if any(g is None for g in gs):
        return None
    base = gs[0]
    st = base.untyped_storage()
    off = base.storage_offset()
    for g in gs:
        if g.untyped_storage().data_ptr() != st.data_ptr() or g.storage_offset() != off \
                or not g.is_contiguous():
            return None
        off += g.numel()
    total = off - base.storage_offset()
    return torch.empty(0, dtype=base.dtype, device=base.device).set_(
        st, base.storage_offset(), (total,), (1,))


# Gradient all-reduces already in flight for a flat gradient buffer, issued by
# the Unet backward as soon as a contiguous bucket of it is final:
# {storage ptr: (flat tensor kept alive, [async work handles])}. Only one
# step's buffer is ever outstanding.
_PENDING = {}


def allreduce_async(flat, lo, hi, group=None):
    """Start the (sum) all-reduce of flat[lo:hi] on RCCL's stream, ordered after
    the work already queued on the current stream; allreduce_grads() waits."""
    key = flat.untyped_storage().data_ptr()
    ent = _PENDING.get(key)
    if ent is None or ent[0] is not flat:
        _PENDING.clear()
        ent = _PENDING[key] = (flat, [])
    ent[1].append(dist.all_reduce(flat[lo:hi], group=group, async_op=True))
    spans = getattr(flat, "_nsm_spans", None)
    if spans is None:
        spans = flat._nsm_spans = []
    spans.append((lo, hi))


def allreduce_grads(params, group=None):
    """Sum grads over ranks (RCCL over xGMI); averaging is folded into the
    optimizer (inv_world). If the backward already put the buckets of this flat
    buffer in flight (Unet.overlap_grad_allreduce), this only makes the current
    stream wait for them."""
    params = list(params)
    g = flat_grad(params)
    if g is not None:
        ent = _PENDING.pop(g.untyped_storage().data_ptr(), None)
        if ent is not None:
            flat, works = ent
            covered = sum(w_hi - w_lo for w_lo, w_hi in getattr(flat, "_nsm_spans", []))
            for w in works:
                w.wait()
            if covered == g.numel():
                return
            raise RuntimeError("pending gradient buckets do not cover the flat buffer")
    if g is None:
        for p in params:
            if p.grad is not None:
                dist.all_reduce(p.grad, group=group)
    else:
        dist.all_reduce(g, group=group)


# ---- schedules of main.py ---------------------------------------------------
def lr_lambda(warmup_epochs=5, num_epochs=200):
    """main.py:959-967 `get_lr_lambda`: linear warmup from 0 (epoch 0 -> lr 0),
    then cosine to a floor of 1 % — pass to torch.optim.lr_scheduler.LambdaLR."""
    def f(epoch):
        if epoch < warmup_epochs:
            return float(epoch) / float(max(1, warmup_epochs))
        decay = 0.5 * (1.0 + math.cos(math.pi * (epoch - warmup_epochs)
                                      / (num_epochs - warmup_epochs)))
        return max(0.01, decay)
    return f


def make_lambda_lr(optimizer, warmup_epochs=5, num_epochs=200):
    """The reference's scheduler (main.py:969) on any optimizer (FlatAdamW included)."""
    return torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda=lr_lambda(warmup_epochs,
                                                                            num_epochs))


def max_norm_for(epoch, num_epochs):
    """main.py:357-358: clip_grad_norm_ threshold of an epoch."""
    r = epoch / num_epochs
    return 1.0 if r < 0.5 else max(0.1, 1.0 - r)


FLAG_NAMES = ("skip", "repaired", "severe", "nonfinite", "huge", "postclip", "n_rescaled",
              "n_zeroed")


def _bump(params):
    """The parameters were rewritten in place by HIP kernels, invisibly to
    autograd's version counters: bump them, so caches keyed on the versions
    (infer.GraphedUnet's frozen weight layouts) see the change."""
    with torch.no_grad():
        for p in params:
            torch.autograd.graph.increment_version(p)


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=7e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-3,
                 max_grad_norm=None, world_size=1, sanitize=False, grad_scale=1.0, seed=None):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdamW supports one param group")
        dev = params[0].device
        total = sum(p.numel() for p in params)
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        off = 0
        offs = [0]
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
                off += n
                offs.append(off)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.max_grad_norm = max_grad_norm
        self.world_size = world_size
        self.inv_world = 1.0 / world_size
        self.sanitize = sanitize
        self.grad_scale = float(grad_scale)
        self.step_count = 0          # host count (sanitize=False: no step is ever skipped)
        nb = lib.nsm_loss_blocks(total)
        self._partial = torch.empty(nb, dtype=torch.float32, device=dev)
        self._sumsq = torch.empty((), dtype=torch.float32, device=dev)
        self._coef = torch.empty((), dtype=torch.float32, device=dev)
        # device state of the reference tail: [AdamW steps taken, tail calls]
        self._step_dev = torch.zeros(2, dtype=torch.int32, device=dev)
        self.flags = torch.zeros(8, dtype=torch.int32, device=dev)
        self.stat = torch.zeros(4, dtype=torch.float32, device=dev)
        if sanitize:
            self._plan(offs, dev)
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little") >> 1
            # data parallel: every rank must draw the same repair noise, or the
            # replicas diverge at the first NaN repair (all ranks hold the same
            # averaged gradient) -> rank 0's seed everywhere
            if world_size > 1 and dist.is_available() and dist.is_initialized():
                bdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
                t = torch.tensor([seed], dtype=torch.int64, device=bdev)
                dist.broadcast(t, 0)
                seed = int(t.item())
        self.seed = seed

    def _plan(self, offs, dev):
        import ctypes
        nseg = len(offs) - 1
        seg_off = (ctypes.c_int64 * (nseg + 1))(*offs)
        nblk = lib.nsm_tail_plan(seg_off, nseg, None, None, None, None, 0)
        blk_seg = (ctypes.c_int * nblk)()
        blk_lo = (ctypes.c_int64 * nblk)()
        blk_hi = (ctypes.c_int64 * nblk)()
        seg_blk = (ctypes.c_int * (nseg + 1))()
        if lib.nsm_tail_plan(seg_off, nseg, blk_seg, blk_lo, blk_hi, seg_blk, nblk) != nblk:
            raise RuntimeError("nsm_tail_plan failed")
        t = lambda a, dt: torch.tensor(list(a), dtype=dt).to(dev)  # noqa: E731
        self._nseg, self._nblk = nseg, nblk
        self._seg_off = t(seg_off, torch.int64)
        self._seg_blk = t(seg_blk, torch.int32)
        self._blk_seg = t(blk_seg, torch.int32)
        self._blk_lo = t(blk_lo, torch.int64)
        self._blk_hi = t(blk_hi, torch.int64)
        nbytes = int(lib.nsm_tail_ws_bytes(nseg, nblk))
        self._ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self._seg_coef = torch.zeros(4 * nseg, dtype=torch.float32, device=dev)

    # main.py:357-358
    def set_epoch(self, epoch, num_epochs):
        """Apply the reference's max_norm schedule for `epoch` of `num_epochs`."""
        self.max_grad_norm = max_norm_for(epoch, num_epochs)

    @torch.no_grad()
    def step(self, closure=None, noise=None):
        """One tail step. `noise` (flat like the gradient, sanitize=True only)
        supplies the randn values of the NaN repair (main.py:336) for parity
        tests; otherwise a counter-based device generator draws them."""
        params = self.param_groups[0]["params"]
        g = flat_grad(params)
        if g is None:
            g = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                           for p in params])
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        n = self.flat.numel()
        st = stream()
        if self.sanitize:
            mx = float(self.max_grad_norm) if self.max_grad_norm is not None else float("inf")
            call("nsm_grad_tail", ptr(g), self._nseg, ptr(self._seg_off), ptr(self._seg_blk),
                 ptr(self._blk_seg), ptr(self._blk_lo), ptr(self._blk_hi), self._nblk,
                 self.inv_world, self.grad_scale, mx, ptr(noise), self.seed, ptr(self._ws),
                 self._ws.numel(), ptr(self._seg_coef), ptr(self.stat), ptr(self.flags),
                 ptr(self._step_dev), st)
            call("nsm_adamw_tail", ptr(self.flat), ptr(g), ptr(self.exp_avg), ptr(self.exp_avg_sq),
                 ptr(self._blk_seg), ptr(self._blk_lo), ptr(self._blk_hi), self._nblk,
                 ptr(self._seg_coef), ptr(self.flags), ptr(self._step_dev), float(grp["lr"]),
                 float(b1), float(b2), float(grp["eps"]), float(grp["weight_decay"]), st)
            _bump(params)
            return None
        self.step_count += 1
        coef = None
        if self.max_grad_norm is not None or self.inv_world != 1.0:
            call("nsm_sumsq", ptr(g), n, ptr(self._partial), ptr(self._sumsq), st)
            mx = float(self.max_grad_norm) if self.max_grad_norm is not None else float("inf")
            call("nsm_clip_coef", ptr(self._sumsq), self.inv_world, mx, ptr(self._coef), st)
            coef = self._coef
        call("nsm_adamw_step", ptr(self.flat), ptr(g), ptr(self.exp_avg), ptr(self.exp_avg_sq), n,
             float(grp["lr"]), float(b1), float(b2), float(grp["eps"]), float(grp["weight_decay"]),
             self.step_count, ptr(coef), st)
        _bump(params)
        return None

    def zero_grad(self, set_to_none=True):
        for p in self.param_groups[0]["params"]:
            p.grad = None

    # ---- inspection (these synchronise; not for the hot loop) ----------------
    def steps_taken(self):
        return int(self._step_dev[0].item()) if self.sanitize else self.step_count

    def last_flags(self):
        """{name: value} of the last sanitised step's decisions (host sync)."""
        f = self.flags.tolist()
        d = dict(zip(FLAG_NAMES, f))
        s = self.stat.tolist()
        d.update(total_norm=s[0], clip_coef=s[1], max_norm=s[2], max_clipped_norm=s[3])
        return d

    # ---- torch.optim.AdamW-compatible checkpoint format ----------------------
    def _torch_group_defaults(self):
        ref = torch.optim.AdamW([torch.zeros(1)])
        d = dict(ref.defaults)
        d.update({k: v for k, v in self.param_groups[0].items() if k != "params"})
        return d

    def state_dict(self):
        params = self.param_groups[0]["params"]
        step = float(self.steps_taken())
        state, off = {}, 0
        for i, p in enumerate(params):
            n = p.numel()
            if step > 0:
                state[i] = {"step": torch.tensor(step),
                            "exp_avg": self.exp_avg[off:off + n].view_as(p).clone(),
                            "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p).clone()}
            off += n
        grp = self._torch_group_defaults()
        grp["params"] = list(range(len(params)))
        return {"state": state, "param_groups": [grp]}

    def load_state_dict(self, sd):
        params = self.param_groups[0]["params"]
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(params):
            raise ValueError("state_dict does not match FlatAdamW's single parameter group")
        grp = groups[0]
        for k in ("lr", "betas", "eps", "weight_decay"):
            if k in grp:
                self.param_groups[0][k] = grp[k]
        for k in ("initial_lr",):
            if k in grp:
                self.param_groups[0][k] = grp[k]
        steps = set()
        off = 0
        with torch.no_grad():
            for i, p in enumerate(params):
                n = p.numel()
                st = sd["state"].get(i, sd["state"].get(grp["params"][i]))
                if st is not None:
                    self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                    self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                    steps.add(int(float(st["step"])))
                else:
                    self.exp_avg[off:off + n].zero_()
                    self.exp_avg_sq[off:off + n].zero_()
                    steps.add(0)
                off += n
        if len(steps) != 1:
            raise ValueError(f"FlatAdamW keeps one step count; checkpoint has {sorted(steps)}")
        s = steps.pop()
        self.step_count = s
        self._step_dev[0] = s
