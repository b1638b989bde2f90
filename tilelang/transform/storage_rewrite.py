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
``tl.storage_rewrite = False``.
"""
from __future__ import annotations

from typing import Dict, List

from ..ir import stmt as S
from .utils import BufferReplacer, flatten_seq


def _uses(stmt) -> set:
    from .pipeline import _referenced_buffers
    return _referenced_buffers(stmt)


def rewrite_local_storage(kernel: S.KernelStmt):
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
    slots = []  # [buffer, last_use]
    mapping = {}
    for a in sorted((a for a in allocs if a.buffer in live), key=lambda a: live[a.buffer][0]):
        b = a.buffer
        first, last = live[b]
        for slot in slots:
            kb = slot[0]
            if kb.dtype == b.dtype and list(kb.static_shape()) == list(b.static_shape()) and slot[1] < first:
                mapping[b] = (kb, [])
                slot[1] = last
                break
        else:
            slots.append([b, last])
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
