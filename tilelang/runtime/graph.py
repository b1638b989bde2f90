"""HIP graph capture of launch-bound call sequences (MI355X-native; no reference counterpart: the
reference relies on per-call CUDA launches).

Every tilelang kernel launches on PyTorch's current HIP stream with no allocation or host sync in
the launch path (``csrc/tl_runtime.cpp``), so a sequence of them -- a MoE layer (router, align,
two expert GEMMs, combine), a decode step -- can be recorded once into a hipGraph and replayed
with one launch.  ``capture`` records ``fn(*static_args)`` after ``warmup`` eager calls (which
also compile and load every kernel) and returns a callable that copies new inputs into the
static input tensors, replays the graph and returns the static outputs::

    step = tilelang.runtime.graph.capture(moe, x)
    y = step(x_next)          # same shapes/dtypes/devices as x; y is overwritten by the next replay

Rules: inputs must keep their shapes; outputs are the graph's own tensors (clone to keep them);
code under capture must not synchronise with the host (``.item()``, ``.cpu()``, ``torch.cuda.synchronize``),
which PyTorch reports as a capture error.
"""
from __future__ import annotations

from typing import Any, Callable


def _tensors(x):
    import torch
    if isinstance(x, torch.Tensor):
        return [x]
    if isinstance(x, (list, tuple)):
        return [t for e in x for t in _tensors(e)]
    if isinstance(x, dict):
        return [t for e in x.values() for t in _tensors(e)]
    return []


class GraphStep:
    """A captured call: ``step(*args)`` copies tensor args into the static inputs and replays."""

    def __init__(self, graph, static_args, static_out, stream):
        self.graph = graph
        self.static_args = static_args
        self.static_out = static_out
        self.stream = stream
        self._inputs = _tensors(static_args)

    def __call__(self, *args) -> Any:
        new = _tensors(args)
        if len(new) != len(self._inputs):
            raise ValueError(f"captured with {len(self._inputs)} tensor inputs, got {len(new)}")
        for dst, src in zip(self._inputs, new):
            if src is not dst:
                if src.shape != dst.shape or src.dtype != dst.dtype:
                    raise ValueError(f"input {tuple(src.shape)} {src.dtype} does not match the captured "
                                     f"{tuple(dst.shape)} {dst.dtype}")
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out

    def replay(self):
        self.graph.replay()
        return self.static_out


def capture(fn: Callable, *static_args, warmup: int = 2) -> GraphStep:
    """Record ``fn(*static_args)`` into a hipGraph (after ``warmup`` eager calls on a side
    stream, as PyTorch requires) and return a :class:`GraphStep`."""
    import torch
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn(*static_args)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn(*static_args)
    return GraphStep(g, static_args, out, s)
