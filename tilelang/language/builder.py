"""IR construction context used while a ``@T.prim_func`` body executes.

The reference builds TIR through TVM's IRBuilder frames (``src/ir.cc``) and,
for ``lazy_jit``, the v2 ``Builder`` (``tilelang/language/v2/builder.py:178``).
Here the kernel body is *executed* (after the AST rewrite in ``parser.py``)
and each DSL call appends statements to the innermost open frame.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager
from typing import List, Optional

from ..ir import stmt as S
from ..ir.buffer import Buffer
from ..ir.expr import PrimExpr, Var, cast, convert, as_int, IntImm

_tls = threading.local()


class BuilderError(Exception):
    pass


class Frame:

    def __init__(self, kind: str):
        self.kind = kind
        self.stmts: List[S.Stmt] = []


class Builder:

    def __init__(self):
        self.frames: List[Frame] = [Frame("root")]
        self.kernel: Optional[S.KernelStmt] = None
        self.kernel_info = None   # (grid vars, thread vars, threads)
        self.loop_stack: List[str] = []
        self.name_counts = {}
        self.attrs = {}

    # -- naming -------------------------------------------------------------------
    def fresh(self, base: str) -> str:
        n = self.name_counts.get(base, 0)
        self.name_counts[base] = n + 1
        return base if n == 0 else f"{base}_{n}"

    # -- frames -------------------------------------------------------------------
    def emit(self, s: S.Stmt):
        self.frames[-1].stmts.append(s)

    def push(self, kind: str) -> Frame:
        f = Frame(kind)
        self.frames.append(f)
        return f

    def pop(self) -> S.Stmt:
        f = self.frames.pop()
        return S.SeqStmt(f.stmts) if len(f.stmts) != 1 else f.stmts[0]

    @property
    def in_kernel(self) -> bool:
        return self.kernel_info is not None

    def store(self, buffer: Buffer, indices, value):
        value = convert(value)
        if value.dtype != buffer.dtype:
            value = cast(value, buffer.dtype)
        self.emit(S.StoreStmt(buffer, indices, value))

    def last_stmt(self):
        st = self.frames[-1].stmts
        return st[-1] if st else None


def current_builder() -> Builder:
    b = getattr(_tls, "builder", None)
    if b is None:
        raise BuilderError("this T.* API must be called inside a @T.prim_func / @T.macro body")
    return b


def has_builder() -> bool:
    return getattr(_tls, "builder", None) is not None


@contextmanager
def building():
    prev = getattr(_tls, "builder", None)
    b = Builder()
    _tls.builder = b
    try:
        yield b
    finally:
        _tls.builder = prev


# ---------------------------------------------------------------------------
# helpers the AST rewriter targets (see parser.py); exposed as ``__tl__``
# ---------------------------------------------------------------------------


class _Undef:
    pass


UNDEF = _Undef()


def is_static(x) -> bool:
    from ..ir.expr import FloatImm
    if isinstance(x, (IntImm, FloatImm)):
        return True
    if isinstance(x, (PrimExpr, Buffer)):
        return False
    return True


def static_value(x):
    if isinstance(x, PrimExpr):
        return bool(as_int(x)) if as_int(x) is not None else bool(x.value)
    return bool(x)


class _IfFrame:

    def __init__(self, cond):
        self.cond = convert(cond)

    def __enter__(self):
        current_builder().push("if")
        return self

    def __exit__(self, et, ev, tb):
        b = current_builder()
        body = b.pop()
        if et is None:
            b.emit(S.IfStmt(self.cond, body, None))
        return False


class _ElseFrame:

    def __enter__(self):
        current_builder().push("else")
        return self

    def __exit__(self, et, ev, tb):
        b = current_builder()
        body = b.pop()
        if et is None:
            last = b.last_stmt()
            if not isinstance(last, S.IfStmt) or last.else_body is not None:
                raise BuilderError("T.Else without a matching T.If")
            last.else_body = body
        return False


class _WhileFrame:

    def __init__(self, cond):
        self.cond = convert(cond)

    def __enter__(self):
        b = current_builder()
        b.push("while")
        b.loop_stack.append("while")
        return self

    def __exit__(self, et, ev, tb):
        b = current_builder()
        b.loop_stack.pop()
        body = b.pop()
        if et is None:
            b.emit(S.WhileStmt(self.cond, body))
        return False


def assign(name: str, value, prev_thunk):
    """Semantics of ``name = value`` inside a kernel body.

    * re-assigning a ``T.alloc_var`` buffer stores into it (TileLang semantics);
    * binding an expression that reads buffers creates a ``LetStmt`` so the value is
      captured at this program point (TIR ``LetStmt`` semantics);
    * everything else is a plain Python binding.
    """
    try:
        prev = prev_thunk()
    except NameError:
        prev = UNDEF
    if not has_builder():
        return value
    b = current_builder()
    if isinstance(value, Buffer) and getattr(value, "_auto_name", False):
        value.name = b.fresh(name)
        value.data.name = value.name
        value._auto_name = False
        return value
    if isinstance(prev, Buffer) and prev.scope == "var" and prev is not value and \
            (not isinstance(value, Buffer) or value.scope == "var"):
        # `x = y` / `x = expr` with x a T.alloc_var: store (y's current value when y is a var too)
        b.store(prev, [IntImm(0)], value.as_scalar() if isinstance(value, Buffer) else value)
        return prev
    if isinstance(value, Buffer) and value.scope == "var" and b.in_kernel and prev is not value:
        value = value.as_scalar()   # `y = x` with x a T.alloc_var: capture x's current value
    if isinstance(value, PrimExpr) and b.in_kernel and _needs_let(value):
        v = Var(b.fresh(name), value.dtype, nonneg=False)
        b.emit(S.LetStmt(v, value))
        return v
    return value


def _needs_let(e) -> bool:
    from ..ir.expr import post_order, BufferLoad, Call
    for n in post_order(e):
        if isinstance(n, BufferLoad):
            return True
        if isinstance(n, Call) and n.op in ("rand", "tl.atomic", "clock"):
            return True
    return False


def land(a, b_thunk):
    if is_static(a) and not isinstance(a, PrimExpr):
        return a and b_thunk()
    if isinstance(a, PrimExpr) and is_static(a):
        return b_thunk() if static_value(a) else a
    from ..ir.expr import logical_and
    return logical_and(a, b_thunk())


def lor(a, b_thunk):
    if is_static(a) and not isinstance(a, PrimExpr):
        return a or b_thunk()
    if isinstance(a, PrimExpr) and is_static(a):
        return a if static_value(a) else b_thunk()
    from ..ir.expr import logical_or
    return logical_or(a, b_thunk())


def ifexp(c, t_thunk, f_thunk):
    if isinstance(c, Buffer):
        c = c.as_scalar()
    if not isinstance(c, PrimExpr):
        return t_thunk() if c else f_thunk()
    if is_static(c):
        return t_thunk() if static_value(c) else f_thunk()
    from ..ir.expr import select
    t, f = t_thunk(), f_thunk()
    t = t.as_scalar() if isinstance(t, Buffer) else t
    f = f.as_scalar() if isinstance(f, Buffer) else f
    return select(c, t, f)


def lnot(a):
    if isinstance(a, Buffer):
        a = a.as_scalar()
    if isinstance(a, PrimExpr):
        from ..ir.expr import logical_not
        return logical_not(a)
    return not a


def tl_range(*args, **kwargs):
    from .loop import serial
    return serial(*args, **kwargs)


def loop_break():
    current_builder().emit(S.BreakStmt())


def loop_continue():
    current_builder().emit(S.ContinueStmt())


class _Helpers:
    """Namespace object injected as ``__tl__`` into rewritten kernel bodies."""
    is_static = staticmethod(is_static)
    static_value = staticmethod(static_value)
    If = _IfFrame
    Else = _ElseFrame
    While = _WhileFrame
    assign = staticmethod(assign)
    land = staticmethod(land)
    lor = staticmethod(lor)
    lnot = staticmethod(lnot)
    ifexp = staticmethod(ifexp)
    range = staticmethod(tl_range)
    loop_break = staticmethod(loop_break)
    loop_continue = staticmethod(loop_continue)


HELPERS = _Helpers()
