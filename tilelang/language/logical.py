"""``T.any_of`` / ``T.all_of`` (reference ``tilelang/language/logical.py:10-77``).

The reference lowers them to a ``tl.any_of(ptr, n)`` device loop.  Here the region is expanded
into an OR / AND of its element loads at trace time, so the condition goes through the ordinary
load lowering of whatever scope the buffer lives in (global mask tensor, LDS, per-thread local)
and clang sees straight-line compares.  As in the reference only the last dimension may span
more than one element; its extent must be static (at most 1024 elements).
"""
from __future__ import annotations

from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import BufferLoad, IntImm, as_int, binop, const


def _elements(target):
    if isinstance(target, Buffer):
        region = [(IntImm(0), s) for s in target.shape]
        buf = target
    elif isinstance(target, BufferRegion):
        buf, region = target.buffer, target.region
    else:
        raise ValueError(f"T.any_of / T.all_of expect a buffer or buffer region, got {type(target).__name__}")
    for i, (_, e) in enumerate(region[:-1]):
        if as_int(e) != 1:
            raise ValueError("T.any_of / T.all_of: only the last dimension may span more than one element")
    n = as_int(region[-1][1])
    if n is None or n > 1024:
        raise ValueError("T.any_of / T.all_of: the last dimension needs a static extent <= 1024")
    base = [m for m, _ in region]
    out = []
    for j in range(n):
        idx = base[:-1] + [binop("+", base[-1], j)]
        v = BufferLoad(buf, idx)
        out.append(v if buf.dtype.is_bool else binop("!=", v, const(0, buf.dtype)))
    return out


def any_of(target):
    """True if any element of the buffer (region) is non-zero."""
    acc = None
    for v in _elements(target):
        acc = v if acc is None else binop("||", acc, v)
    return acc


def all_of(target):
    """True if every element of the buffer (region) is non-zero."""
    acc = None
    for v in _elements(target):
        acc = v if acc is None else binop("&&", acc, v)
    return acc
