"""One whole training step replayed from a HIP graph.

The reference's step (main.py:255-423: forward under autocast, the loss,
`scaler.scale(loss).backward()`, the NaN/Inf census and repair, the
per-parameter clips, clip_grad_norm_, AdamW) is ~200 kernel launches on this
path; `GraphedTrainStep` captures forward + loss + backward + the FlatAdamW
device tail once and replays them as one graph, so the launches no longer pay
the host's per-launch cost nor the gaps between dispatches.

What the graph holds fixed, and how the step stays the reference's:
  * inputs: `step.x` / `step.y` are static buffers — copy each batch into them
    (`step(x, y)` does it);
  * Dropout2d masks: drawn from torch's graph-safe CUDA generator inside the
    graph (unet._masks_for -> nsm_dropout_masks_dev), new masks every replay;
  * the CustomLoss range assert: its sticky device flag only, allocated
    before the capture (`loss_fn.prepare_capture`); `loss_fn.check_range_now()`
    reads it, or the step itself every `range_check_every` replays;
  * version counters: each replay bumps those of the parameters and buffers
    (the kernels rewrote them), so infer.GraphedUnet refreshes its layouts;
  * hyper-parameters passed as kernel arguments (lr, betas, eps, weight decay,
    max_norm, the loss scale): the step re-captures when one of them changes
    (an epoch's LambdaLR / max_norm schedule costs one capture);
  * parameter / buffer addresses: FlatAdamW's flat storage keeps them; a
    re-allocation raises.
The constructor runs `warmup` eager steps on (x, y) to settle the caches,
then restores parameters, AdamW moments, the tail's counters and the BN
buffers, so building the step changes no training state. Under data
parallelism (`Unet.data_parallel`) the collectives are captured with the
rest: the rank-0 BN buffer broadcast at the forward, the two gradient buckets'
all-reduce the backward issues, and the wait for them before the tail; every
rank must build and replay its step in lockstep, as with eager collectives."""
import torch

from ._lib import require_gpu
from .optim import _bump, allreduce_grads


class GraphedTrainStep:
    def __init__(self, model, loss_fn, optimizer, x, y, loss_scale=1.0, warmup=3,
                 range_check_every=0):
        require_gpu(x, "GraphedTrainStep input")
        # data parallel (Unet.data_parallel): the rank-0 BN broadcast, the
        # bucketed gradient all-reduce the backward issues and the wait for it
        # are captured too (RCCL kernels recorded into the graph)
        self.dp = model._grad_allreduce is not None
        if not getattr(optimizer, "sanitize", False):
            # the plain FlatAdamW step passes its step count (AdamW's bias
            # correction) as a kernel argument, which a graph would freeze; the
            # reference's tail (sanitize=True) counts on the device
            raise ValueError("GraphedTrainStep: needs nsm_amd.FlatAdamW(..., sanitize=True), "
                             "whose device tail keeps the AdamW step count on the device")
        self.model, self.loss_fn, self.opt = model, loss_fn, optimizer
        self.loss_scale = float(loss_scale)
        self.x = x.detach().clone().requires_grad_(x.requires_grad)
        self.y = y.detach().clone()
        self.warmup = warmup
        # every N-th replay raises the reference's `assert 0 <= output <= 1`
        # (customLoss.py:131) from the sticky device flag (a host sync); 0:
        # only when the caller runs loss_fn.check_range_now()
        self.range_check_every = int(range_check_every)
        self.replays = 0
        self.graph = None
        self._capture()

    def _hyper(self):
        g = self.opt.param_groups[0]
        return (float(g["lr"]), tuple(g["betas"]), float(g["eps"]), float(g["weight_decay"]),
                self.opt.max_grad_norm, self.opt.grad_scale, self.loss_scale)

    def _addresses(self):
        return [t.data_ptr() for t in list(self.model.parameters()) + list(self.model.buffers())]

    def _body(self):
        out = self.model(self.x)
        loss = self.loss_fn(out, self.y, self.x)
        # d(loss_scale * loss)/d loss seeded from a buffer filled before the
        # capture: the same gradient as (loss * s).backward(), without the
        # seed's fill (and the scale's multiply) launched by ATen in the graph
        loss.backward(self._seed)
        if self.dp:
            allreduce_grads(self.model.parameters(), self.model._grad_allreduce[0])
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.x.grad = None
        return loss.detach()

    def _state(self):
        """Everything a step writes besides its scratch: parameters and AdamW
        moments (FlatAdamW's flat buffers), the tail's device counters and
        flags, the BN running statistics and counts."""
        o = self.opt
        ts = [o.flat, o.exp_avg, o.exp_avg_sq, o._step_dev, o.flags, o.stat]
        return ts + [b for b in self.model.buffers()]

    def _capture(self, warmup=None):
        warmup = self.warmup if warmup is None else warmup
        self._seed = torch.full((), self.loss_scale, dtype=torch.float32, device=self.x.device)
        side = torch.cuda.Stream(device=self.x.device)
        side.wait_stream(torch.cuda.current_stream())
        saved = [t.detach().clone() for t in self._state()]
        with torch.cuda.stream(side):
            for _ in range(warmup):   # allocator, weight-layout and mask-descriptor caches
                self._body()
        torch.cuda.current_stream().wait_stream(side)
        prep = getattr(self.loss_fn, "prepare_capture", None)
        if prep is not None:   # the range assert's sticky flag, allocated outside the capture
            prep(self.x.device)
        self.graph = torch.cuda.CUDAGraph()
        # thread-local capture: RCCL's watchdog thread queries events while the
        # capture runs (a global-mode capture would fail those queries)
        mode = "thread_local" if self.dp else "global"
        with torch.cuda.graph(self.graph, capture_error_mode=mode):   # recorded, not run
            self.loss = self._body()
        # the warm-up steps leave no trace: the model and optimizer are as
        # they were before the constructor
        with torch.no_grad():
            for t, v in zip(self._state(), saved):
                t.copy_(v)
        self._hyp = self._hyper()
        self._ptrs = self._addresses()

    def __call__(self, x=None, y=None):
        """One step: copy the batch in (if given), replay; returns the loss
        tensor (device, unscaled). The first call after a hyper-parameter
        change re-captures first (no eager steps: the caches are warm)."""
        if x is not None:
            self.x.detach().copy_(x)
        if y is not None:
            self.y.copy_(y)
        if self._addresses() != self._ptrs:
            raise RuntimeError("GraphedTrainStep: parameters or buffers were re-allocated after "
                               "capture — build a new step")
        if self._hyper() != self._hyp:
            self.graph = None
            self._capture(warmup=0)   # the caches are warm
        self.graph.replay()
        # the replay rewrote the parameters and the BN buffers with HIP kernels;
        # the Python-side version bumps (FlatAdamW's, the forward's BN one) ran
        # only at capture: bump them here so version-keyed caches
        # (infer.GraphedUnet's frozen layouts and eval BN vectors) refresh
        _bump(list(self.model.parameters()) + list(self.model.buffers()))
        self.replays += 1
        if self.range_check_every and self.replays % self.range_check_every == 0:
            check = getattr(self.loss_fn, "check_range_now", None)
            if check is not None:
                check()
        return self.loss
