"""Pre-lowering semantic checks.

Reference: ``tilelang/analysis/nested_loop_checker.py:11-126`` (illegal nesting of
``T.Pipelined``/``T.Parallel``) and ``fragment_loop_checker.py:9-100``
(symbolic-extent parallel loops over fragments), run by
``PreLowerSemanticCheck`` (``tilelang/engine/phase.py:112-124``).
"""
from __future__ import annotations

from ..ir import stmt as S
from ..ir.expr import as_int, BufferLoad, post_order


class SemanticError(Exception):
    pass


def _check_nesting(s, in_pipelined=False, in_parallel=False):
    if isinstance(s, S.ForStmt):
        if s.kind == "pipelined":
            if in_pipelined:
                raise SemanticError("nested T.Pipelined loops are not supported")
            if in_parallel:
                raise SemanticError("T.Pipelined inside T.Parallel is not allowed")
            _check_nesting(s.body, True, in_parallel)
            return
        if s.kind == "parallel":
            _check_nesting(s.body, in_pipelined, True)
            return
        if in_parallel and s.kind in ("serial", "unroll"):
            pass
    if isinstance(s, S.TileOpStmt) and in_parallel:
        raise SemanticError(f"tile operator T.{s.op.kind} cannot be used inside T.Parallel")
    for c in S.stmt_children(s):
        _check_nesting(c, in_pipelined, in_parallel)


def _check_fragment_loops(s):
    for x in S.walk(s):
        if isinstance(x, S.ForStmt) and x.kind == "parallel" and as_int(x.extent) is None:
            for y in S.walk(x.body):
                exprs = []
                if isinstance(y, S.StoreStmt):
                    if y.buffer.scope == "fragment":
                        raise SemanticError(f"T.Parallel with symbolic extent {x.extent} writes fragment "
                                            f"{y.buffer.name}; fragments need static loop extents")
                    exprs = [y.value]
                for e in exprs:
                    for n in post_order(e):
                        if isinstance(n, BufferLoad) and n.buffer.scope == "fragment":
                            raise SemanticError(f"T.Parallel with symbolic extent reads fragment {n.buffer.name}")


def semantic_check(func, kernel: S.KernelStmt):
    _check_nesting(kernel.body)
    _check_fragment_loops(kernel.body)
