"""Loop constructs: ``T.Parallel``, ``T.Pipelined``, ``T.serial``, ``T.unroll``, ``T.Persistent``.

Reference: ``tilelang/language/loop.py:12-178`` and the frames in
``src/ir.cc:55-187``.  Each construct is a generator that opens an IR frame,
yields the loop variable(s) once (the body is traced once) and closes the
frame into a ``ForStmt`` when the Python ``for`` asks for the next item.
"""
from __future__ import annotations

from typing import List, Optional

from ..ir import stmt as S
from ..ir.expr import Var, convert, const
from ..ir import dtypes as _dt
from .builder import current_builder

_LOOP_NAMES = ["i", "j", "k", "l", "m", "n", "p", "q"]


def _range_args(start, stop, step):
    if stop is None:
        start, stop = 0, start
    start, stop = convert(start), convert(stop)
    if step not in (None, 1):
        step = convert(step)
    else:
        step = None
    return start, stop, step


def _loop(kind: str, start, stop, step=None, annotations=None, name="i"):
    b = current_builder()
    start, stop, step = _range_args(start, stop, step)
    v = Var(b.fresh(name), stop.dtype if stop.dtype.is_int else _dt.int32)
    b.push(kind)
    b.loop_stack.append(kind)
    if step is None:
        yield v
        body = b.pop()
        b.loop_stack.pop()
        b.emit(S.ForStmt(v, start, stop - start, kind, body, annotations))
    else:
        # strided loop: iterate k in [0, ceildiv(stop-start, step)) and bind i = start + k*step
        k = Var(b.fresh(name + "_k"))
        # body refers to v; wrap in a Let
        yield v
        body = b.pop()
        b.loop_stack.pop()
        from ..ir.expr import ceildiv
        n = ceildiv(stop - start, step)
        b.emit(S.ForStmt(k, 0, n, kind, S.seq(S.LetStmt(v, start + k * step), body), annotations))


def serial(start, stop=None, step=None, *, annotations=None):
    return _loop("serial", start, stop, step, annotations)


Serial = serial


def unroll(start, stop=None, step=None, *, explicit: bool = False, unroll_factor: Optional[int] = None,
           annotations=None):
    ann = dict(annotations or {})
    if unroll_factor is not None:
        ann["unroll_factor"] = unroll_factor
    return _loop("unroll", start, stop, step, ann)


Unroll = unroll


def vectorized(start, stop=None):
    return _loop("vectorized", start, stop)


Vectorized = vectorized


def Parallel(*extents, coalesced_width: Optional[int] = None, loop_layout=None):
    """Nested parallel loops; the compiler partitions the iterations over the block's threads."""
    b = current_builder()
    vars_: List[Var] = []
    ranges = []
    for d, e in enumerate(extents):
        if isinstance(e, (tuple, list)):
            lo, hi = e
        else:
            lo, hi = 0, e
        vars_.append(Var(b.fresh(_LOOP_NAMES[d % len(_LOOP_NAMES)])))
        ranges.append((convert(lo), convert(hi) - convert(lo)))
    b.push("parallel")
    b.loop_stack.append("parallel")
    yield vars_[0] if len(vars_) == 1 else tuple(vars_)
    body = b.pop()
    b.loop_stack.pop()
    ann = {}
    if coalesced_width is not None:
        ann["coalesced_width"] = coalesced_width
    if loop_layout is not None:
        ann["loop_layout"] = loop_layout
    for v, (lo, ext) in reversed(list(zip(vars_, ranges))):
        body = S.ForStmt(v, lo, ext, "parallel", body, ann)
        ann = dict(ann)
    b.emit(body)


def grid(*extents):
    """``T.grid``: nested serial loops."""
    b = current_builder()
    vars_ = [Var(b.fresh(_LOOP_NAMES[d % len(_LOOP_NAMES)])) for d in range(len(extents))]
    b.push("serial")
    b.loop_stack.append("serial")
    yield vars_[0] if len(vars_) == 1 else tuple(vars_)
    body = b.pop()
    b.loop_stack.pop()
    for v, e in reversed(list(zip(vars_, extents))):
        body = S.ForStmt(v, 0, e, "serial", body)
    b.emit(body)


def Pipelined(start, stop=None, num_stages: int = 0, order=None, stage=None, sync=None, group=None, order_alt=None,
              alt_cond=None, unroll: Optional[int] = None):
    """Software-pipelined loop: copies into shared buffers are multi-buffered ``num_stages`` deep.

    On gfx950 the global->LDS copies become ``global_load_lds_dwordx4`` DMA issued
    ``num_stages-1`` iterations ahead, with counted ``s_waitcnt vmcnt`` waits.

    ``order`` / ``stage`` / ``group``: user schedule (transform/stage_schedule.py).  ``sync`` is
    accepted and recorded but has no effect, exactly as in the reference (``src/ir.cc:105`` sets
    ``tl_pipeline_sync`` and no pass reads it); LDS hazards between the scheduled statements get
    their barriers from the thread-sync pass, which proves them per access.
    ``unroll``: the lowered main loop is emitted under ``#pragma unroll N`` (with N a multiple of
    the ring depth every ring slot index of an unrolled copy is a compile-time constant).
    """
    ann = {"num_stages": int(num_stages)}
    if unroll is not None:
        ann["unroll_factor"] = int(unroll)
    if order is not None:
        ann["order"] = list(order)
    if stage is not None:
        ann["stage"] = list(stage)
    if sync is not None:
        ann["sync"] = sync
    if group is not None:
        ann["group"] = group
    if (order_alt is None) != (alt_cond is None):
        raise ValueError("T.Pipelined: order_alt and alt_cond go together")
    if order_alt is not None:
        ann["order_alt"] = list(order_alt)
        ann["alt_cond"] = alt_cond
    return _loop("pipelined", start, stop, None, ann, name="k")


def Persistent(domain, wave_size, index, group_size: Optional[int] = 8, lds_iteration_local: bool = False):
    """Persistent tile loop (reference ``src/ir.cc:115-187``).

    ``domain`` is the 2-D tile grid ``[tiles_m, tiles_n]``; ``wave_size`` the number of
    concurrently running blocks; ``index`` the block id.  Yields ``(bx, by)`` for each tile this
    block owns, walking tiles in waves with grouped (L2-friendly) ordering.
    ``lds_iteration_local``: no shared-memory value crosses a tile, so the LDS planner may give
    buffers used in different stretches of one tile (the operand ring, a C staging tile) the same
    bytes (transform/lds_plan.py).
    """
    b = current_builder()
    if isinstance(domain, (list, tuple)):
        dom = [convert(d) for d in domain]
    else:
        dom = [convert(domain)]
    total = const(1)
    for d in dom:
        total = total * d
    from ..ir.expr import ceildiv
    waves = ceildiv(total, wave_size)
    w = Var(b.fresh("w"))
    b.push("serial")
    b.loop_stack.append("serial")
    tile = index + w * wave_size
    coords = []
    if len(dom) == 2 and group_size:
        # grouped ordering over the first dim (like the GEMM swizzle)
        gs = group_size
        m, n = dom
        num_in_group = gs * n
        gid = tile // num_in_group
        first_m = gid * gs
        gsz = S_min(m - first_m, gs)
        bx = first_m + (tile % num_in_group) % gsz
        by = (tile % num_in_group) // gsz
        coords = [bx, by]
    else:
        rem = tile
        for d in reversed(dom):
            coords.insert(0, rem % d)
            rem = rem // d
    from .builder import _IfFrame
    guard = _IfFrame(tile < total)
    guard.__enter__()
    yield tuple(coords) if len(coords) > 1 else coords[0]
    guard.__exit__(None, None, None)
    body = b.pop()
    b.loop_stack.pop()
    ann = {"persistent": True}
    if lds_iteration_local:
        ann["lds_iteration_local"] = True
    b.emit(S.ForStmt(w, 0, waves, "serial", body, ann))


def S_min(a, b):
    from ..ir.expr import min_expr
    return min_expr(a, b)
