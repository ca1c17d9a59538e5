"""Inference path (BASELINE config 5: 1x7x1080x1920 eval forward), captured in
one HIP graph.

The reference's inference (`infer.py:34-43,65`: `model.eval()`, `torch.no_grad()`,
one `model(x)` per frame) launches ~200 kernels per frame from Python. Here
the whole eval forward of a fixed input shape is captured once with
`torch.cuda.graph` (hipStreamBeginCapture underneath: every libnsm entry point
launches asynchronously on the caller's stream and never allocates or
synchronises, so the C ABI is capturable as is) and each frame is one
`hipGraphLaunch`. Eval BatchNorm is folded into per-channel scale/shift that
the consumers' operand loaders apply (no separate BN pass exists in eval).

    g = GraphedUnet(model, example_input)     # model on the GPU, any mode
    out = g(x)                                # x: same shape/dtype/device

The returned tensor is the graph's static output buffer: it is overwritten by
the next call (clone it to keep it).

Frozen weights (static_weights=True, default): the weight layouts of the step
(the prep launches) and the eval BatchNorm vectors are prepared once, before
the capture (unet.FrozenWeights), so a frame replays only the per-frame
kernels — the reference's infer.py loads its weights once and runs frames.
The parameters' and BN buffers' version counters are checked at each call:
after any change (a torch optimizer step, load_state_dict, a FlatAdamW step or
a training forward, which bump them) the kept layouts are rewritten in place
(refresh()) before the replay, so the output always reflects the current
weights.
"""
import torch

from ._lib import require_gpu


class GraphedUnet:
    def __init__(self, model, example, warmup=2, static_weights=True):
        from .unet import FrozenWeights
        require_gpu(example, "GraphedUnet example input")
        self.model = model
        self.was_training = model.training
        model.eval()
        self.shape, self.dtype = tuple(example.shape), example.dtype
        self.static_in = example.detach().clone()
        self.frozen = FrozenWeights(model) if static_weights else None
        side = torch.cuda.Stream(device=example.device)
        side.wait_stream(torch.cuda.current_stream())
        if self.frozen is not None:
            self.frozen.__enter__()
        try:
            with torch.cuda.stream(side), torch.no_grad():
                for _ in range(warmup):           # settle the caching allocator (and the layouts)
                    model(self.static_in)
            torch.cuda.current_stream().wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(self.graph):
                self.static_out = model(self.static_in)
        finally:
            if self.frozen is not None:
                self.frozen.__exit__(None, None, None)
        model.train(self.was_training)
        # the graph holds raw parameter / buffer addresses: replay must see the same storage
        self._ptrs = self._addresses()
        self._vers = self._versions()

    def _versions(self):
        return [t._version for t in list(self.model.parameters()) + list(self.model.buffers())]

    def refresh(self):
        """Rewrite the frozen weight layouts / BN vectors from the current
        parameters and running statistics (in place; eager, on the current
        stream). Called automatically when a version counter moved."""
        if self.frozen is not None:
            with torch.no_grad():
                self.frozen.refresh()
        self._vers = self._versions()

    def _addresses(self):
        return [t.data_ptr() for t in list(self.model.parameters()) + list(self.model.buffers())]

    def _check(self):
        if self._addresses() != self._ptrs:
            raise RuntimeError("GraphedUnet: the model's parameters or buffers were re-allocated "
                               "after capture (e.g. FlatAdamW re-homed them, or .to()); the "
                               "captured graph would read freed memory — capture again")
        if self.frozen is not None and self._versions() != self._vers:
            self.refresh()

    def __call__(self, x):
        if tuple(x.shape) != self.shape or x.dtype != self.dtype:
            raise ValueError(f"GraphedUnet captured for {self.shape} {self.dtype}, "
                             f"got {tuple(x.shape)} {x.dtype}")
        self._check()
        self.static_in.copy_(x)
        self.graph.replay()
        return self.static_out

    def replay(self):
        """Run the captured forward on whatever is in static_in."""
        self._check()
        self.graph.replay()
        return self.static_out
