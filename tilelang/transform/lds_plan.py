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

from typing import Dict, List

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


def _top_level(body) -> List:
    """Flattened top-level statement list (scoped blocks stay whole: their declarations)."""
    top = []
    stack = [body]
    while stack:
        b = stack.pop(0)
        if isinstance(b, S.SeqStmt) and not getattr(b, "scoped", False):
            stack = list(b.stmts) + stack
        else:
            top.append(b)
    return top


ITER_LOCAL = "lds_iteration_local"


def _iter_local_body(st):
    """(loop, body statements, guard) for a loop annotated ``lds_iteration_local`` (its shared
    buffers hold nothing across iterations), else None.  A body that is one ``if`` without an else
    (a persistent loop's bound check; block-uniform like every statement with a barrier inside)
    is opened too: ``guard`` is that if."""
    if not (isinstance(st, S.ForStmt) and st.annotations.get(ITER_LOCAL)):
        return None
    body, guard = st.body, None
    if isinstance(body, S.IfStmt) and body.else_body is None:
        guard, body = body, body.then_body
    return st, _top_level(body), guard


def _expand(body):
    """Top-level statements, with the bodies of iteration-local loops expanded in place:
    ``[(stmt, group)]``; group is None at the top level, else the index of its loop."""
    out, loops = [], []
    for st in _top_level(body):
        il = _iter_local_body(st)
        if il is None:
            out.append((st, None))
        else:
            loops.append(il)
            out += [(x, len(loops) - 1) for x in il[1]]
    return out, loops


def _dma_targets(s) -> set:
    out = set()
    for x in S.walk(s):
        if isinstance(x, L.CallStmt) and x.name.startswith(("tl::glds", "tl::buffer_lds")):
            for a in x.args:
                if isinstance(a, L.BufferPtr) and a.buffer.scope == "shared":
                    out.add(a.buffer)
    return out


def plan_lds(kernel: S.KernelStmt, reuse: bool = True, aggressive: bool = False):
    """Place every shared buffer in one arena.

    ``reuse``: buffers whose live ranges (first/last top-level statement of the kernel body that
    touches them) do not overlap share bytes; a ``__syncthreads()`` is inserted in front of the
    first statement that touches a buffer re-using bytes of a buffer that died earlier, so every
    access of the old tenant (any thread) is ordered before the new tenant's first access.
    ``aggressive`` (``tl.enable_aggressive_shared_memory_merge``, default on): LDS-DMA (pipeline
    stage) buffers die at their last top-level use too, and the switch into their bytes is
    preceded by ``s_waitcnt vmcnt(0)`` so no DMA still in flight can land in the new tenant (e.g.
    the LDS ring of a GEMM main loop re-used by its C staging tile).  Off: DMA targets keep their
    bytes for the whole kernel.

    Returns ``(kernel, offsets, total_bytes)``."""
    shared = []
    for s in S.walk(kernel):
        if isinstance(s, S.AllocStmt) and s.buffer.scope == "shared" and s.buffer not in shared:
            shared.append(s.buffer)
    sizes = {b: int(b.shape[0]) * b.dtype.bytes for b in shared}
    # statements in order; the bodies of loops annotated ``lds_iteration_local`` (T.serial(...,
    # annotations={"lds_iteration_local": True}): no shared value crosses an iteration, e.g. a
    # persistent tile loop whose operand ring and C staging tile are rewritten every tile) are
    # expanded, so buffers confined to one iteration's stretch of statements can share bytes
    top, loops = _expand(kernel.body) if reuse and not kernel.is_cpu else ([(x, None) for x in _top_level(
        kernel.body)], [])
    group = [g for _, g in top]
    top = [x for x, _ in top]
    first, last = {}, {}
    for i, st in enumerate(top):
        t = set()
        _touches(st, t)
        for b in t:
            first.setdefault(b, i)
            last[b] = i
    # a buffer touched in an iteration-local loop AND outside it lives across the whole loop
    span = {}
    for i, g in enumerate(group):
        if g is not None:
            lo, hi = span.get(g, (i, i))
            span[g] = (min(lo, i), max(hi, i))
    for b in list(first):
        for g, (lo, hi) in span.items():
            inside = lo <= first[b] and last[b] <= hi
            touches = not (last[b] < lo or first[b] > hi)
            if touches and not inside:
                first[b], last[b] = min(first[b], lo), max(last[b], hi)
    dma = _dma_targets(kernel)
    pinned = set() if aggressive else dma
    n_top = len(top)
    f = [0 if (b in pinned or b not in first) else first[b] for b in shared]
    l_ = [n_top if (b in pinned or b not in last) else last[b] for b in shared]
    # placement by the native arena planner (csrc/core/lds.cc plan_arena)
    from .._native import core
    try:
        offs, total = core().plan_arena([sizes[b] for b in shared], f, l_, ALIGN, bool(reuse), LDS_LIMIT)
    except ValueError as e:  # std::length_error -> ValueError
        raise LDSPlanError(str(e)) from None
    offsets: Dict[Buffer, int] = dict(zip(shared, offs))
    if not reuse or kernel.is_cpu:
        return kernel, offsets, total
    # region switches: statement index -> needs a barrier in front
    switch, drain = set(), set()
    for i, b in enumerate(shared):
        for j, a in enumerate(shared):
            if a is b or l_[j] >= f[i]:
                continue
            oa, ob = offsets[a], offsets[b]
            if oa < ob + sizes[b] and ob < oa + sizes[a]:
                switch.add(f[i])
                if a in dma:
                    drain.add(f[i])
    # iteration wrap: a later tenant of iteration i precedes an earlier tenant of iteration i + 1
    for g, (lo, hi) in span.items():
        for i, b in enumerate(shared):
            for j, a in enumerate(shared):
                if a is b or not (lo <= f[i] <= l_[i] <= hi and lo <= f[j] <= l_[j] <= hi) or l_[i] >= f[j]:
                    continue
                oa, ob = offsets[a], offsets[b]
                if oa < ob + sizes[b] and ob < oa + sizes[a]:
                    switch.add(lo)
                    if a in dma:
                        drain.add(lo)
    if not switch:
        return kernel, offsets, total
    from .thread_sync import _sync

    def marks(i):
        out = []
        if i in drain:
            out.append(L.CallStmt("tl::wait_vmcnt", [], [0]))
        if i in switch:
            out.append(_sync())
        return out

    new_top, i = [], 0
    while i < len(top):
        g = group[i]
        if g is None:
            new_top += marks(i) + [top[i]]
            i += 1
            continue
        loop, stmts, guard = loops[g]
        body = []
        for _ in stmts:
            body += marks(i) + [top[i]]
            i += 1
        nb = S.SeqStmt(body)
        if guard is not None:
            nb = S.IfStmt(guard.cond, nb, None)
        new_top.append(S.ForStmt(loop.var, loop.min, loop.extent, loop.kind, nb, loop.annotations))
    k = S.KernelStmt(kernel.grid, kernel.threads, kernel.block_vars, kernel.thread_vars, S.SeqStmt(new_top),
                     kernel.is_cpu, kernel.prelude)
    k.attrs = dict(kernel.attrs)
    return k, offsets, total
