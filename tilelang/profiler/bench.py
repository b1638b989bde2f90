"""Kernel timing (reference ``tilelang/profiler/bench.py:63-204``).

MI355X specifics: the cache flush before every timed launch READS a 512 MiB buffer so that
both the per-XCD L2s (8 x 4 MiB) and the 256 MiB Infinity Cache are evicted (the reference
writes 256 MB, sized for NVIDIA L2).  Reading matters on MI355X: a zero-fill leaves up to
256 MiB of dirty Infinity-Cache lines that the timed kernel then pays to write back -- a
streaming copy measured 4.4 TB/s after a write flush (gpurun_out r3 membound sweep), i.e. the
flush's write-back was being billed to the kernel.  Timing uses HIP events on the
current stream; ``backend="profiler"`` uses torch.profiler device time (rocprofiler).

``flush_mode="write"`` (or ``TL_BENCH_FLUSH=write``) restores the reference's zero-fill flush for
like-for-like comparisons with numbers measured that way; docs/RESULTS.md says which rows used
which flush.
"""
from __future__ import annotations

from typing import Callable, List, Optional

_FLUSH = {}


def _flush_buffer(device):
    import torch
    b = _FLUSH.get(device)
    if b is None:
        b = torch.zeros(512 * 1024 * 1024 // 4, dtype=torch.int32, device=device)
        _FLUSH[device] = (b, torch.empty(1, dtype=torch.int32, device=device))
    return _FLUSH[device]


def _flush(cache, mode: str = "read"):
    """Evict L2 + Infinity Cache: "read" = a max-reduction over 512 MiB (leaves no dirty lines),
    "write" = the reference's zero-fill."""
    import torch
    buf, out = cache
    if mode == "write":
        buf.zero_()
    else:
        torch.amax(buf, dim=0, keepdim=True, out=out)


def do_bench(fn: Callable, warmup: float = 25, rep: float = 100, _n_warmup: int = 0, _n_repeat: int = 0,
             quantiles: Optional[List[float]] = None, fast_flush: bool = True, return_mode: str = "mean",
             backend: str = "event", flush_l2: bool = True, flush_mode: Optional[str] = None) -> float:
    """Median/mean runtime of ``fn`` in milliseconds."""
    import os
    import torch
    flush_mode = flush_mode or os.environ.get("TL_BENCH_FLUSH", "read")
    if flush_mode not in ("read", "write"):
        raise ValueError(f"flush_mode must be 'read' or 'write', got {flush_mode!r}")
    assert return_mode in ("min", "max", "mean", "median")
    if backend in ("cupti", "profiler"):
        return _bench_profiler(fn, warmup, rep)
    fn()
    torch.cuda.synchronize()
    dev = torch.cuda.current_device()
    cache = _flush_buffer(dev) if flush_l2 else None
    # estimate
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        if cache is not None:
            _flush(cache, flush_mode)
        fn()
    e.record()
    torch.cuda.synchronize()
    est = max(s.elapsed_time(e) / 5, 1e-4)
    n_warmup = _n_warmup or max(1, int(warmup / est))
    n_repeat = _n_repeat or max(1, int(rep / est))
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(n_repeat)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n_repeat)]
    for _ in range(n_warmup):
        fn()
    for i in range(n_repeat):
        if cache is not None:
            _flush(cache, flush_mode)
        starts[i].record()
        fn()
        ends[i].record()
    torch.cuda.synchronize()
    times = torch.tensor([a.elapsed_time(b) for a, b in zip(starts, ends)], dtype=torch.float)
    if quantiles is not None:
        ret = torch.quantile(times, torch.tensor(quantiles, dtype=torch.float)).tolist()
        return ret[0] if len(ret) == 1 else ret
    return getattr(torch, return_mode)(times).item()


def _bench_profiler(fn, warmup, rep):
    import torch
    from torch.profiler import profile, ProfilerActivity
    fn()
    torch.cuda.synchronize()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    n = 20
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
    total = 0.0
    for evt in prof.key_averages():
        total += evt.device_time_total if hasattr(evt, "device_time_total") else evt.cuda_time_total
    return total / n / 1e3
