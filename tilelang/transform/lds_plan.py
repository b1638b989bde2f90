"""LDS arena planning: every shared buffer of a kernel lives in ONE ``__shared__`` array.

Reference: ``src/transform/merge_shared_memory_allocations.cc`` (packs shared
buffers into one dynamic arena with liveness-based reuse) and
``align_dynamic_shared_memory_allocations.cc``.  One arena is also what gfx950
needs for LDS-DMA pipelines: a second ``__shared__`` object next to the DMA staging
array can make hipcc emit ``s_waitcnt vmcnt(0)`` before every ``ds_read``
(guide §5 "Projection GEMM" item 4(a)).

Buffers are placed at 256-byte (one LDS bank row) aligned offsets so the bank
model used to choose swizzles holds for every buffer.  Buffers whose live ranges
(first/last top-level statement touching them) do not overlap share space.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

from ..ir import stmt as S
from ..ir import lowered as L
from ..ir.buffer import Buffer
from ..ir.expr import BufferLoad, post_order

LDS_LIMIT = 160 * 1024
ALIGN = 256


class LDSPlanError(Exception):
    pass


def _touches(s, out: set):
    for x in S.walk(s):
        if isinstance(x, S.StoreStmt) and x.buffer.scope == "shared":
            out.add(x.buffer)
        exprs = []
        if isinstance(x, S.StoreStmt):
            exprs = [x.value] + list(x.indices)
        elif isinstance(x, S.LetStmt):
            exprs = [x.value]
        elif isinstance(x, S.EvaluateStmt):
            exprs = [x.expr]
        elif isinstance(x, S.IfStmt):
            exprs = [x.cond]
        elif isinstance(x, L.CallStmt):
            exprs = list(x.args)
        elif isinstance(x, L.VecStoreStmt):
            out.add(x.buffer)
            exprs = list(x.values) + [x.index]
        elif isinstance(x, (L.VecLoadStmt, L.CopyBytesStmt)):
            for b in (x.src, x.dst):
                if b.scope == "shared":
                    out.add(b)
        for e in exprs:
            if hasattr(e, "dtype"):
                for n in post_order(e):
                    if isinstance(n, (BufferLoad, L.BufferPtr)) and n.buffer.scope == "shared":
                        out.add(n.buffer)
                    if isinstance(n, L.BufferPtr) and n.buffer.scope == "shared":
                        out.add(n.buffer)
            if isinstance(e, L.BufferPtr) and e.buffer.scope == "shared":
                out.add(e.buffer)


def plan_lds(kernel: S.KernelStmt, reuse: bool = False) -> Tuple[Dict[Buffer, int], int]:
    """``reuse`` (liveness-based sharing) is off by default: the barrier pass tracks hazards per
    buffer, so aliasing two buffers also needs ``tl.enable_aggressive_shared_memory_merge``
    (which re-runs the barrier pass on the merged arena)."""
    shared = []
    for s in S.walk(kernel):
        if isinstance(s, S.AllocStmt) and s.buffer.scope == "shared" and s.buffer not in shared:
            shared.append(s.buffer)
    sizes = {b: int(b.shape[0]) * b.dtype.bytes for b in shared}
    # live ranges over the top-level statements of the kernel body
    top = []
    body = kernel.body
    stack = [body]
    while stack:
        b = stack.pop(0)
        if isinstance(b, S.SeqStmt):
            stack = list(b.stmts) + stack
        else:
            top.append(b)
    first, last = {}, {}
    for i, st in enumerate(top):
        t = set()
        _touches(st, t)
        for b in t:
            first.setdefault(b, i)
            last[b] = i
    # placement by the native arena planner (csrc/core/lds.cc plan_arena)
    from .._native import core
    try:
        offs, total = core().plan_arena([sizes[b] for b in shared], [first.get(b, 0) for b in shared],
                                        [last.get(b, len(top)) for b in shared], ALIGN, bool(reuse), LDS_LIMIT)
    except ValueError as e:  # std::length_error -> ValueError
        raise LDSPlanError(str(e)) from None
    offsets: Dict[Buffer, int] = dict(zip(shared, offs))
    return offsets, total
