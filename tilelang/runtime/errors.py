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
_pending = collections.deque()   # (ring, slot, device word, label, decoder)


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


class _Ring:
    """Per-device pool of pinned 4-byte read-back slots and their events, allocated once: a
    launch's read-back is one async copy + one event record, no pinned allocation or event
    creation on the launch path (EP / TP mesh kernels launch every layer)."""
    SIZE = 1024

    def __init__(self, dev_idx: int):
        import torch
        self.host = torch.zeros(self.SIZE, dtype=torch.int32, pin_memory=True)
        self.views = [self.host[i:i + 1] for i in range(self.SIZE)]
        with torch.cuda.device(dev_idx):
            self.events = [torch.cuda.Event() for _ in range(self.SIZE)]
        self.busy = [False] * self.SIZE
        self.next = 0


_rings = {}
_captured = {}  # id -> (error word, label, decoder) of launches recorded during a graph capture


def _ring(word) -> _Ring:
    idx = word.device.index
    r = _rings.get(idx)
    if r is None:
        r = _rings[idx] = _Ring(idx)
    return r


def record(word, label: str, decoder=None):
    """Queue a non-blocking read-back of ``word`` behind the launch just issued on the current
    stream (call right after the launch)."""
    import torch
    if torch.cuda.is_current_stream_capturing():
        # inside tilelang.runtime.graph.capture: an event record + host sync on the launch path
        # is illegal there, and a captured read-back would only report the capture-time launch.
        # Replayed graphs leave the error word set; errors.check() after a replay reads it
        with _lock:
            _captured[id(word)] = (word, label, decoder or _grid_decoder)
        return
    with _lock:
        ring = _ring(word)
        i = ring.next
        ring.next = (i + 1) % ring.SIZE
        wrapped = ring.busy[i]
    if wrapped:
        # the ring wrapped onto a read-back that was never polled: retire the oldest entries
        _drain_slot(ring, i)
    ring.views[i].copy_(word, non_blocking=True)
    ring.events[i].record()
    with _lock:
        ring.busy[i] = True
        _pending.append((ring, i, word, label, decoder or _grid_decoder))


def _drain_slot(ring, i):
    ring.events[i].synchronize()
    poll()
    with _lock:
        still = ring.busy[i]
    if still:  # still queued behind an unfinished entry: drop it (it was clean or raised)
        with _lock:
            keep = [p for p in _pending if not (p[0] is ring and p[1] == i)]
            _pending.clear()
            _pending.extend(keep)
            ring.busy[i] = False


def poll():
    """Raise for the first completed launch whose error word was set (non-blocking)."""
    if not _pending:
        return
    err = None
    with _lock:
        keep = collections.deque()
        while _pending:
            ring, i, word, label, dec = _pending.popleft()
            if not ring.events[i].query():
                keep.append((ring, i, word, label, dec))
                continue
            code = int(ring.host[i])
            ring.busy[i] = False
            if code and err is None:
                err = dec(label, code)
                word.zero_()
                # later launches copied the same (not yet cleared) word: one timeout raises once
                for p in list(keep) + list(_pending):
                    if p[2] is word:
                        p[0].busy[p[1]] = False
                keep = collections.deque(p for p in keep if p[2] is not word)
                rest = [p for p in _pending if p[2] is not word]
                _pending.clear()
                _pending.extend(rest)
        _pending.extendleft(reversed(keep))
    if err is not None:
        raise err


def check():
    """Synchronise the current device and raise any recorded device error (including the error
    words of launches recorded inside a hipGraph capture, read here synchronously)."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    poll()
    with _lock:
        words = list(_captured.values())
    for word, label, dec in words:
        code = int(word.item())
        if code:
            word.zero_()
            raise dec(label, code)


def pending() -> int:
    return len(_pending)
