"""IR rewriting utilities shared by the passes."""
from __future__ import annotations

from typing import Dict, List

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir import lowered as L
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import BinOp, BufferLoad, Cast, PrimExpr, Var, substitute, transform as expr_transform, IntImm


class Mutator:
    """Rebuilds statements; override ``expr`` / ``region`` / ``visit_*`` as needed."""

    def expr(self, e):
        return e

    def region(self, r: BufferRegion) -> BufferRegion:
        mins = [self.expr(m) for m, _ in r.region]
        exts = [self.expr(e) if isinstance(e, PrimExpr) else e for _, e in r.region]
        return BufferRegion(r.buffer, list(zip(mins, exts)))

    def tileop(self, op):
        import copy
        op = copy.copy(op)
        for name in ("src", "dst", "A", "B", "C", "buf", "send", "recv", "tmp", "img", "col", "scale_A", "scale_B", "E",
                     "valid_m", "valid_m_min"):
            v = getattr(op, name, None)
            if isinstance(v, BufferRegion):
                setattr(op, name, self.region(v))
            elif isinstance(v, PrimExpr):
                setattr(op, name, self.expr(v))
        if isinstance(op, O.FillOp):
            op.value = self.expr(op.value)
        if isinstance(op, O.GemmOp) and isinstance(op.clear_accum, PrimExpr):
            op.clear_accum = self.expr(op.clear_accum)
        return op

    def stmt(self, s):
        if s is None:
            return None
        m = getattr(self, "visit_" + type(s).__name__, None)
        if m is not None:
            return m(s)
        return self.default(s)

    def default(self, s):
        if isinstance(s, S.SeqStmt):
            out = S.SeqStmt([self.stmt(c) for c in s.stmts])
            if getattr(s, "scoped", False):
                out.scoped = True  # a C++ block: its let bindings must not leak into siblings
            return out
        if isinstance(s, S.ForStmt):
            return S.ForStmt(s.var, self.expr(s.min), self.expr(s.extent), s.kind, self.stmt(s.body), s.annotations)
        if isinstance(s, S.WhileStmt):
            return S.WhileStmt(self.expr(s.cond), self.stmt(s.body))
        if isinstance(s, S.IfStmt):
            return S.IfStmt(self.expr(s.cond), self.stmt(s.then_body), self.stmt(s.else_body))
        if isinstance(s, S.StoreStmt):
            return self.store(s)
        if isinstance(s, S.EvaluateStmt):
            return S.EvaluateStmt(self.expr(s.expr))
        if isinstance(s, S.LetStmt):
            return S.LetStmt(s.var, self.expr(s.value))
        if isinstance(s, S.TileOpStmt):
            return S.TileOpStmt(self.tileop(s.op))
        if isinstance(s, S.KernelStmt):
            k = S.KernelStmt([self.expr(g) for g in s.grid], s.threads, s.block_vars, s.thread_vars,
                             self.stmt(s.body), s.is_cpu, s.prelude)
            k.attrs = dict(s.attrs)
            return k
        if isinstance(s, S.AssertStmt):
            return S.AssertStmt(self.expr(s.cond), s.msg)
        if isinstance(s, S.AttrStmt):
            return S.AttrStmt(s.key, s.value, self.stmt(s.body))
        if isinstance(s, L.CallStmt):
            return L.CallStmt(s.name, [self.expr(a) for a in s.args], s.targs)
        if isinstance(s, L.VecStoreStmt):
            return L.VecStoreStmt(s.buffer, self.expr(s.index), [self.expr(v) for v in s.values])
        if isinstance(s, L.VecLoadStmt):
            return L.VecLoadStmt(s.dst, s.dst_index, s.src, self.expr(s.src_index), s.n)
        if isinstance(s, L.CopyBytesStmt):
            return L.CopyBytesStmt(s.dst, self.expr(s.dst_index), s.src, self.expr(s.src_index), s.nbytes)
        return s

    def store(self, s: S.StoreStmt):
        return S.StoreStmt(s.buffer, [self.expr(i) for i in s.indices], self.expr(s.value), s.predicate)


class Substituter(Mutator):
    """Substitute variables everywhere (statements, regions, tile ops)."""

    def __init__(self, vmap: Dict[Var, PrimExpr]):
        self.vmap = vmap

    def expr(self, e):
        if isinstance(e, L.BufferPtr):
            return L.BufferPtr(e.buffer, self.expr(e.offset))
        if isinstance(e, PrimExpr):
            return substitute(e, self.vmap)
        return e


def subst_stmt(s, vmap):
    if not vmap:
        return s
    return Substituter(vmap).stmt(s)


class BufferReplacer(Mutator):
    """Replace buffer B by B' with an index transform ``fn(indices) -> indices``."""

    def __init__(self, mapping: Dict[Buffer, tuple]):
        # mapping: old buffer -> (new buffer, prefix index exprs)
        self.mapping = mapping

    def _fix_load(self, n):
        if isinstance(n, BufferLoad) and n.buffer in self.mapping:
            nb, prefix = self.mapping[n.buffer]
            return BufferLoad(nb, list(prefix) + list(n.indices))
        return None

    def expr(self, e):
        if isinstance(e, PrimExpr):
            return expr_transform(e, self._fix_load)
        return e

    def region(self, r):
        r2 = Mutator.region(self, r)
        if r2.buffer in self.mapping:
            nb, prefix = self.mapping[r2.buffer]
            return BufferRegion(nb, [(p, 1) for p in prefix] + list(r2.region))
        return r2

    def store(self, s):
        s2 = Mutator.store(self, s)
        if s2.buffer in self.mapping:
            nb, prefix = self.mapping[s2.buffer]
            return S.StoreStmt(nb, list(prefix) + s2.indices, s2.value, s2.predicate)
        return s2


def flatten_seq(s) -> List:
    if s is None:
        return []
    if isinstance(s, S.SeqStmt):
        out = []
        for c in s.stmts:
            out.extend(flatten_seq(c))
        return out
    return [s]


def stmt_uses_var(s, var: Var) -> bool:
    from ..ir.expr import uses_var
    found = [False]

    class F(Mutator):

        def expr(self, e):
            if isinstance(e, PrimExpr) and uses_var(e, var):
                found[0] = True
            return e

    F().stmt(s)
    return found[0]


# ---------------------------------------------------------------------------
# interval (bounds) analysis used to prove in-bounds accesses
# ---------------------------------------------------------------------------


def bound(e, ranges: Dict[Var, tuple]):
    """Conservative integer interval [lo, hi] of ``e`` (None when unknown).  Data-dependent
    values are unknown, but a clamp ``min(max(x, lo), hi)`` of one is still bounded."""
    r = _bound(e, ranges)
    if r is None or r[0] == -_INF or r[1] == _INF:
        return None
    return (int(r[0]), int(r[1]))


_INF = float("inf")


def _bound(e, ranges):
    if isinstance(e, int):
        return (e, e)
    if isinstance(e, IntImm):
        return (e.value, e.value)
    if isinstance(e, Var):
        return ranges.get(e)
    if isinstance(e, Cast):
        return _bound(e.value, ranges)
    if isinstance(e, BinOp):
        a = _bound(e.a, ranges)
        b = _bound(e.b, ranges)
        if e.op in ("min", "max"):
            a = a if a is not None else (-_INF, _INF)
            b = b if b is not None else (-_INF, _INF)
            if e.op == "min":
                return (min(a[0], b[0]), min(a[1], b[1]))
            return (max(a[0], b[0]), max(a[1], b[1]))
        if e.op == "%" and b is not None and b[0] == b[1] and b[0] > 0 and \
                (a is None or _INF in (abs(a[0]), abs(a[1])) or a[0] < 0):
            return (0, b[0] - 1)  # floor modulo: in [0, b) whatever the dividend
        if a is None or b is None or _INF in (abs(a[0]), abs(a[1]), abs(b[0]), abs(b[1])):
            return None
        if e.op == "+":
            return (a[0] + b[0], a[1] + b[1])
        if e.op == "-":
            return (a[0] - b[1], a[1] - b[0])
        if e.op == "*":
            c = [a[0] * b[0], a[0] * b[1], a[1] * b[0], a[1] * b[1]]
            return (min(c), max(c))
        if e.op in ("//", "/") and b[0] == b[1] and b[0] > 0 and a[0] >= 0:
            return (a[0] // b[0], a[1] // b[0])
        if e.op == "%" and b[0] == b[1] and b[0] > 0:
            if a[0] >= 0:
                return (0, min(b[0] - 1, a[1]))
            return (0, b[0] - 1)
    return None
