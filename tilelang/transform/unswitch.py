"""Loop unswitching on a marked, loop-invariant condition (``tl.unswitch``).

``T.Pipelined(order_alt=, alt_cond=)`` (transform/stage_schedule.py) leaves the main pipelined loop
with one top-level ``if tl.unswitch(cond): <order_alt compute> else: <order compute>``.  LLVM does
not unswitch it: the loop holds convergent operations (barriers, readfirstlane) and it cannot
prove the condition uniform.  Left inside the loop, the two orders' register live ranges meet at
the join and the register allocator spills (FA fwd: 0 -> 158 spilled VGPRs).  This pass, run after
pipelining and barrier placement, rewrites

    for k: pre; if c: A else: B; post      ->      if c: (for k: pre; A; post) else: (for k: pre; B; post)

Every copy keeps the loop's barriers, so the workgroup's barrier sequence is unchanged (both wave
groups run the same number of iterations with the same barriers; only the instruction order
between two barriers differs).  The condition must be loop-invariant (checked) and is emitted as
a scalar branch (``readfirstlane``: codegen/hip.py).
"""
from __future__ import annotations

from ..ir import stmt as S
from ..ir.expr import Call, free_vars


def _marked(s) -> bool:
    return isinstance(s, S.IfStmt) and isinstance(s.cond, Call) and s.cond.op == "tl.unswitch"


def _unswitch_loop(loop: S.ForStmt):
    body = loop.body.stmts if isinstance(loop.body, S.SeqStmt) else [loop.body]
    idx = [i for i, x in enumerate(body) if _marked(x)]
    if len(idx) != 1:
        return None
    i = idx[0]
    br = body[i]
    if any(v is loop.var for v in free_vars(br.cond)):
        raise ValueError("tl.unswitch condition depends on the loop variable")
    pre, post = list(body[:i]), list(body[i + 1:])

    def copy(part):
        return S.ForStmt(loop.var, loop.min, loop.extent, loop.kind, S.seq(*(pre + [part] + post)), loop.annotations)

    return S.IfStmt(br.cond, copy(br.then_body), copy(br.else_body if br.else_body is not None else S.seq()))


def unswitch_marked(s):
    def fn(x):
        if isinstance(x, S.ForStmt):
            r = _unswitch_loop(x)
            if r is not None:
                return r
        return x

    return S.map_stmt(s, fn)
