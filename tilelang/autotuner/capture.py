"""``set_autotune_inputs`` (reference ``tilelang/autotuner/capture.py:101``): real tensors for the
tuning runs.

    with tilelang.autotuner.set_autotune_inputs(a, b):
        kernel = matmul(M, N, K)          # an @autotune'd factory: every config runs on (a, b)

Inside the ``with`` block the autotuner benchmarks (and checks) every config on the captured
tensors instead of synthesising inputs from the kernel signature -- the way to tune on
data-dependent work (sparse indices, routing tables, ragged lengths).  Captures nest per thread;
the innermost one wins.
"""
from __future__ import annotations

import threading
from typing import Any, List, Optional

_local = threading.local()


def _stack() -> list:
    st = getattr(_local, "stack", None)
    if st is None:
        st = _local.stack = []
    return st


class AutotuneInputsCapture:
    """Context manager holding one list of input tensors (positional kernel arguments)."""

    __slots__ = ("tensors", )

    def __init__(self, tensors: List[Any]):
        self.tensors = list(tensors)

    def __enter__(self) -> "AutotuneInputsCapture":
        _stack().append(self)
        return self

    def __exit__(self, exc_type, exc, tb):
        st = _stack()
        if not st or st[-1] is not self:
            raise RuntimeError("set_autotune_inputs contexts exited out of order")
        st.pop()
        return False


def set_autotune_inputs(*args) -> AutotuneInputsCapture:
    """``set_autotune_inputs(a, b, c)`` or ``set_autotune_inputs([a, b, c])``."""
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        return AutotuneInputsCapture(list(args[0]))
    return AutotuneInputsCapture(list(args))


def get_autotune_inputs() -> Optional[List[Any]]:
    """The innermost captured input list of this thread, or None."""
    st = _stack()
    return st[-1].tensors if st else None
