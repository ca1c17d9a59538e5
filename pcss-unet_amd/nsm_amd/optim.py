"""Train-step tail on libnsm kernels: global-norm clip + AdamW over ONE flat
parameter buffer (main.py:405 clip_grad_norm_, main.py:421 AdamW step,
main.py:952-953 `optim.AdamW(lr, weight_decay=1e-3)`), and the data-parallel
gradient all-reduce.

`FlatAdamW` re-homes the parameters into a single contiguous fp32 buffer
(views keep the module's parameter objects, so state_dict / LambdaLR /
named_parameters are unchanged). The Unet backward writes all 66 gradients
into one flat buffer too, so clip + update is three kernel launches and the
DP exchange is one all-reduce of 60 MiB, with no host synchronisation.
"""
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
    optimizer's clip coefficient (inv_world). If the backward already put the
    buckets of this flat buffer in flight (Unet.overlap_grad_allreduce), this
    only makes the current stream wait for them."""
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


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=7e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-3,
                 max_grad_norm=None, world_size=1):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdamW supports one param group")
        dev = params[0].device
        total = sum(p.numel() for p in params)
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
                off += n
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.max_grad_norm = max_grad_norm
        self.inv_world = 1.0 / world_size
        self.step_count = 0
        nb = lib.nsm_loss_blocks(total)
        self._partial = torch.empty(nb, dtype=torch.float32, device=dev)
        self._sumsq = torch.empty((), dtype=torch.float32, device=dev)
        self._coef = torch.empty((), dtype=torch.float32, device=dev)

    @torch.no_grad()
    def step(self, closure=None):
        params = self.param_groups[0]["params"]
        g = flat_grad(params)
        if g is None:
            g = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                           for p in params])
        grp = self.param_groups[0]
        self.step_count += 1
        n = self.flat.numel()
        coef = None
        if self.max_grad_norm is not None or self.inv_world != 1.0:
            call("nsm_sumsq", ptr(g), n, ptr(self._partial), ptr(self._sumsq), stream())
            mx = float(self.max_grad_norm) if self.max_grad_norm is not None else float("inf")
            call("nsm_clip_coef", ptr(self._sumsq), self.inv_world, mx, ptr(self._coef), stream())
            coef = self._coef
        b1, b2 = grp["betas"]
        call("nsm_adamw_step", ptr(self.flat), ptr(g), ptr(self.exp_avg), ptr(self.exp_avg_sq), n,
             float(grp["lr"]), float(b1), float(b2), float(grp["eps"]), float(grp["weight_decay"]),
             self.step_count, ptr(coef), stream())
        return None

    def zero_grad(self, set_to_none=True):
        for p in self.param_groups[0]["params"]:
            p.grad = None
