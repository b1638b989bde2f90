"""StorageRewrite for per-thread ``local`` buffers (reference ``src/transform/storage_rewrite.cc:2011``,
the TVM pass that lets buffers with disjoint lifetimes share one allocation).

On gfx950 the two other storage classes are already planned elsewhere: LDS tiles share the
dynamic-LDS arena by liveness (``lds_plan.py``), and register fragments are promoted to SSA values by
clang (SROA) whose register allocator reuses them.  ``T.alloc_local`` arrays are the remaining
case: an array indexed with a runtime value stays an array in the private (scratch) segment, so
two such arrays that are never live at the same time should be one array.

Rule (conservative): over the statements at the top level of the kernel body (a statement that
contains a use covers it entirely, loops included), a ``local`` buffer is live from its first to
its last referencing statement; buffers of identical dtype and shape whose live ranges do not
overlap are merged onto the earliest one (greedy interval colouring).  Disabled with
``tir.disable_storage_rewrite``.

In-place detection (``tl.storage_rewrite_detect_inplace``, reference ``storage_rewrite.cc:975-1004``
and its ``InplaceOpVerifier``): a buffer whose first statement is the LAST statement of another
buffer of the same dtype and shape may take over its storage when that statement is a pure
element-wise map ``dst[idx] = f(src[idx], ...)``: every access of either buffer uses one index
tuple made of distinct loop variables covering every enclosing loop (so no iteration reads an
element another iteration has already overwritten), ``src`` is only read and ``dst`` only written,
and no read of ``src`` follows the first write of ``dst`` in program order (a second same-index read
after the store would see the new value once the two share storage).
"""
from __future__ import annotations

from typing import Dict, List

from ..ir import stmt as S
from .utils import BufferReplacer, flatten_seq


def _uses(stmt) -> set:
    from .pipeline import _referenced_buffers
    return _referenced_buffers(stmt)


def _inplace_ok(stmt, src, dst) -> bool:
    """``stmt`` computes dst from src element-wise at one injective index tuple (see module doc)."""
    from ..ir.expr import BufferLoad, Var, post_order
    loops = []
    idx_seen = []
    ok = [True]
    stored = [False]  # a store to dst has been seen (program order)

    def visit_expr(e):
        for n in post_order(e):
            if isinstance(n, BufferLoad):
                if n.buffer is dst:
                    ok[0] = False
                elif n.buffer is src:
                    if stored[0]:
                        # src read after dst was written: once merged, it reads the new value
                        ok[0] = False
                    idx_seen.append(tuple(n.indices))

    def visit(x):
        if not ok[0] or x is None:
            return
        if isinstance(x, S.SeqStmt):
            for c in x.stmts:
                visit(c)
        elif isinstance(x, S.ForStmt):
            loops.append(x.var)
            visit(x.body)
        elif isinstance(x, S.StoreStmt):
            if x.buffer is src:
                ok[0] = False
                return
            if x.buffer is dst:
                idx_seen.append(tuple(x.indices))
            for i in x.indices:
                visit_expr(i)
            visit_expr(x.value)
            if x.buffer is dst:
                stored[0] = True
        elif isinstance(x, S.LetStmt):
            visit_expr(x.value)
        else:
            ok[0] = False  # tile ops, calls, branches: not provably element-wise

    visit(stmt)
    if not ok[0] or not idx_seen:
        return False
    first = idx_seen[0]
    if any(len(t) != len(first) or any(a is not b for a, b in zip(t, first)) for t in idx_seen):
        return False
    if not all(isinstance(i, Var) for i in first) or len(set(map(id, first))) != len(first):
        return False
    return set(map(id, loops)) <= set(map(id, first))


def rewrite_local_storage(kernel: S.KernelStmt, detect_inplace: bool = False):
    """Returns (kernel, {merged buffer name: kept buffer name})."""
    body = flatten_seq(kernel.body)
    allocs = [st for st in body if isinstance(st, S.AllocStmt) and st.buffer.scope == "local" and
              st.buffer.static_shape() is not None]
    if len(allocs) < 2:
        return kernel, {}
    live: Dict[object, List[int]] = {}
    for i, st in enumerate(body):
        if isinstance(st, S.AllocStmt):
            continue
        for b in _uses(st):
            if b.scope == "local":
                rng = live.setdefault(b, [i, i])
                rng[1] = i
    slots = []  # [kept buffer, last use, buffer of the last use]
    mapping = {}
    for a in sorted((a for a in allocs if a.buffer in live), key=lambda a: live[a.buffer][0]):
        b = a.buffer
        first, last = live[b]
        for slot in slots:
            kb = slot[0]
            if kb.dtype == b.dtype and list(kb.static_shape()) == list(b.static_shape()) and (
                    slot[1] < first or (detect_inplace and slot[1] == first and slot[2] is not None and
                                        _inplace_ok(body[first], slot[2], b))):
                mapping[b] = (kb, [])
                slot[1] = last
                slot[2] = b
                break
        else:
            slots.append([b, last, b])
    if not mapping:
        return kernel, {}
    new_body = [st for st in body if not (isinstance(st, S.AllocStmt) and st.buffer in mapping)]
    rep = BufferReplacer(mapping)
    new_body = [rep.stmt(st) for st in new_body]
    out = S.KernelStmt(kernel.grid, kernel.threads, kernel.block_vars, kernel.thread_vars, S.SeqStmt(new_body),
                       kernel.is_cpu, kernel.prelude)
    for k, v in getattr(kernel, "__dict__", {}).items():
        if not hasattr(out, k):
            setattr(out, k, v)
    return out, {b.name: kb.name for b, (kb, _) in mapping.items()}
