"""Statements of the tile IR and the PrimFunc container.

Counterpart of the TIR statements the reference builds through TVM's
IRBuilder (``src/ir.cc:55-399`` frames for Kernel/Parallel/Pipelined/
Persistent) plus the ``tl.tileop.*`` calls (``src/op/operator.h:80-88``).
Tile operators are first-class statements here (``TileOpStmt``) rather than
opaque ``Evaluate(Call)`` nodes.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from .expr import PrimExpr, Var, convert


class Stmt:
    def __repr__(self):
        from .printer import stmt_str
        return stmt_str(self)


class SeqStmt(Stmt):
    def __init__(self, stmts: List[Stmt]):
        flat = []
        for s in stmts:
            if isinstance(s, SeqStmt) and not getattr(s, "scoped", False):
                flat.extend(s.stmts)
            elif s is not None:
                flat.append(s)
        self.stmts = flat


class ForStmt(Stmt):
    KINDS = ("serial", "parallel", "pipelined", "unroll", "vectorized", "persistent")

    def __init__(self, var: Var, min_, extent, kind: str, body: Stmt, annotations: Optional[Dict] = None):
        assert kind in self.KINDS, kind
        self.var = var
        self.min = convert(min_)
        self.extent = convert(extent)
        self.kind = kind
        self.body = body
        self.annotations = dict(annotations or {})


class WhileStmt(Stmt):
    def __init__(self, cond: PrimExpr, body: Stmt):
        self.cond = convert(cond)
        self.body = body


class IfStmt(Stmt):
    def __init__(self, cond: PrimExpr, then_body: Stmt, else_body: Optional[Stmt] = None):
        self.cond = convert(cond)
        self.then_body = then_body
        self.else_body = else_body


class StoreStmt(Stmt):
    def __init__(self, buffer, indices: List[PrimExpr], value: PrimExpr, predicate=None):
        self.buffer = buffer
        self.indices = [convert(i) for i in indices]
        self.value = value
        self.predicate = predicate


class EvaluateStmt(Stmt):
    def __init__(self, expr: PrimExpr):
        self.expr = expr


class LetStmt(Stmt):
    """``const <dtype> var = value;`` visible for the rest of the enclosing block."""

    def __init__(self, var: Var, value: PrimExpr):
        self.var = var
        self.value = convert(value)


class AllocStmt(Stmt):
    def __init__(self, buffer):
        self.buffer = buffer


class TileOpStmt(Stmt):
    def __init__(self, op):
        self.op = op


class BreakStmt(Stmt):
    pass


class ContinueStmt(Stmt):
    pass


class AssertStmt(Stmt):
    def __init__(self, cond, msg: str = ""):
        self.cond = convert(cond)
        self.msg = msg


class AttrStmt(Stmt):
    """Scoped attribute, e.g. ``use_swizzle`` or ``annotate_layout``."""

    def __init__(self, key: str, value, body: Optional[Stmt] = None):
        self.key = key
        self.value = value
        self.body = body


class RawStmt(Stmt):
    """Target code emitted verbatim (produced by lowering passes only)."""

    def __init__(self, code: str, kind: str = "code"):
        self.code = code
        self.kind = kind


class KernelStmt(Stmt):
    """``with T.Kernel(*grid, threads=...)`` — the device launch scope."""

    def __init__(self, grid: List[PrimExpr], threads: List[int], block_vars: List[Var],
                 thread_vars: List[Var], body: Stmt, is_cpu: bool = False, prelude: Optional[str] = None):
        self.grid = [convert(g) for g in grid]
        self.threads = list(threads)
        self.block_vars = block_vars
        self.thread_vars = thread_vars
        self.body = body
        self.is_cpu = is_cpu
        self.prelude = prelude
        self.attrs: Dict = {}

    @property
    def num_threads(self) -> int:
        n = 1
        for t in self.threads:
            n *= int(t)
        return n


class PrimFunc:
    """A kernel program: parameters (buffers / scalar vars) + body."""

    def __init__(self, name: str, params: List, body: Stmt, attrs: Optional[Dict] = None):
        self.name = name
        self.params = params          # list of Buffer (global) or Var (scalar)
        self.body = body
        self.attrs = dict(attrs or {})

    def script(self) -> str:
        from .printer import func_str
        return func_str(self)

    def __repr__(self):
        return self.script()

    # TileLang compatibility: ``func.with_attr(...)``
    def with_attr(self, key, value):
        f = PrimFunc(self.name, self.params, self.body, self.attrs)
        f.attrs[key] = value
        return f

    @property
    def buffer_map(self):
        from .buffer import Buffer
        return {p: p for p in self.params if isinstance(p, Buffer)}


# ---------------------------------------------------------------------------
# generic statement traversal helpers
# ---------------------------------------------------------------------------


def stmt_children(s: Stmt) -> List[Stmt]:
    if isinstance(s, SeqStmt):
        return list(s.stmts)
    if isinstance(s, (ForStmt, WhileStmt, KernelStmt)):
        return [s.body]
    if isinstance(s, IfStmt):
        return [s.then_body] + ([s.else_body] if s.else_body is not None else [])
    if isinstance(s, AttrStmt):
        return [s.body] if s.body is not None else []
    return []


def walk(s: Stmt):
    """Pre-order traversal of statements."""
    if s is None:
        return
    yield s
    for c in stmt_children(s):
        yield from walk(c)


def map_stmt(s: Stmt, fn):
    """Post-order rewrite: ``fn(stmt)`` returns a replacement (or the same stmt)."""
    if s is None:
        return None
    if isinstance(s, SeqStmt):
        new = [map_stmt(c, fn) for c in s.stmts]
        s = SeqStmt(new) if any(a is not b for a, b in zip(new, s.stmts)) else s
    elif isinstance(s, ForStmt):
        b = map_stmt(s.body, fn)
        if b is not s.body:
            s = ForStmt(s.var, s.min, s.extent, s.kind, b, s.annotations)
    elif isinstance(s, WhileStmt):
        b = map_stmt(s.body, fn)
        if b is not s.body:
            s = WhileStmt(s.cond, b)
    elif isinstance(s, IfStmt):
        t = map_stmt(s.then_body, fn)
        e = map_stmt(s.else_body, fn)
        if t is not s.then_body or e is not s.else_body:
            s = IfStmt(s.cond, t, e)
    elif isinstance(s, KernelStmt):
        b = map_stmt(s.body, fn)
        if b is not s.body:
            k = KernelStmt(s.grid, s.threads, s.block_vars, s.thread_vars, b, s.is_cpu, s.prelude)
            k.attrs = dict(s.attrs)
            s = k
    elif isinstance(s, AttrStmt) and s.body is not None:
        b = map_stmt(s.body, fn)
        if b is not s.body:
            s = AttrStmt(s.key, s.value, b)
    r = fn(s)
    return s if r is None else r


def seq(*stmts) -> Stmt:
    flat = [s for s in stmts if s is not None]
    if len(flat) == 1:
        return flat[0]
    return SeqStmt(flat)
