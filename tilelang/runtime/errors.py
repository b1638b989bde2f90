"""Asynchronous device-error reporting for kernels with bounded waits.

Kernels that wait on other workgroups (``T.sync_grid``) or on other GPUs (``T.comm.*``) never
spin forever: a wait that exceeds its wall-clock budget records a code in a device error word
and lets the kernel finish (a hung kernel would hold the GPU).  This module turns those codes
into Python exceptions without adding a host synchronisation to every launch:

* after a launch, ``record()`` enqueues a 4-byte device→pinned-host copy of the word and an event
  on the launch stream;
* ``poll()`` (run at the start of every ``JITKernel`` call) reads the words of launches whose
  event has completed and raises ``GridSyncTimeout`` / ``MeshError`` for a non-zero one — the
  same "sticky error at the next call" contract as HIP's own asynchronous errors;
* ``check()`` synchronises and polls (a hard check point: tests, the end of a step).

A raised word is zeroed so that one timeout raises once.  Codes: 1/2/4 mesh waits (receiver slot,
sender data, barrier — ``tl/mesh.h``), 8 grid barrier (``tl/common.h``).
"""
from __future__ import annotations

import collections
import threading


class DeviceError(RuntimeError):
    """A bounded device-side wait timed out (the kernel finished with stale data)."""


class GridSyncTimeout(DeviceError):
    """``T.sync_grid``: not every workgroup of the grid reached the barrier in time."""


GRID_SYNC_CODE = 8

_lock = threading.Lock()
_words = {}                       # device index -> int32 device tensor [1] (grid-barrier kernels)
_pending = collections.deque()   # (event, pinned host tensor, device word, label, decoder)


def device_word(device):
    """The process-wide error word of ``device`` (int32 device tensor, zero when healthy)."""
    import torch
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _lock:
        w = _words.get(idx)
        if w is None:
            w = _words[idx] = torch.zeros(1, dtype=torch.int32, device=f"cuda:{idx}")
        return w


def _grid_decoder(label, code):
    what = []
    if code & GRID_SYNC_CODE:
        what.append("a workgroup did not reach T.sync_grid within the time budget "
                    "(block-dependent barrier, or a grid that is not fully resident)")
    rest = code & ~GRID_SYNC_CODE
    if rest:
        what.append(f"device error bits {rest:#x}")
    return GridSyncTimeout(f"{label}: " + "; ".join(what))


def record(word, label: str, decoder=None):
    """Queue a non-blocking read-back of ``word`` behind the launch just issued on the current
    stream (call right after the launch)."""
    import torch
    host = torch.empty(1, dtype=torch.int32, pin_memory=True)
    host.copy_(word, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    with _lock:
        _pending.append((ev, host, word, label, decoder or _grid_decoder))
        # bound the queue: completed clean entries are dropped by poll(); keep the newest ones
        while len(_pending) > 4096:
            _pending.popleft()


def poll():
    """Raise for the first completed launch whose error word was set (non-blocking)."""
    if not _pending:
        return
    err = None
    with _lock:
        keep = collections.deque()
        while _pending:
            ev, host, word, label, dec = _pending.popleft()
            if not ev.query():
                keep.append((ev, host, word, label, dec))
                continue
            code = int(host.item())
            if code and err is None:
                err = dec(label, code)
                word.zero_()
                # later launches copied the same (not yet cleared) word: one timeout raises once
                keep = collections.deque(p for p in keep if p[2] is not word)
                rest = [p for p in _pending if p[2] is not word]
                _pending.clear()
                _pending.extend(rest)
        _pending.extendleft(reversed(keep))
    if err is not None:
        raise err


def check():
    """Synchronise the current device and raise any recorded device error."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    poll()


def pending() -> int:
    return len(_pending)
