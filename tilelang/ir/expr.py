"""Scalar expressions of the tile IR.

This replaces the TVM ``PrimExpr`` hierarchy the reference builds on
(``3rdparty/tvm``; used throughout ``tilelang/language/*.py``).  The design
goal is different from TVM's: expressions are small immutable Python
objects with operator overloading and *eager constant folding*, so that the
frontend can execute kernel bodies directly (tracing) and the passes can
evaluate layouts numerically.  Heavy algebraic simplification is left to
the device compiler (clang), which sees every index expression as plain C++.
"""
from __future__ import annotations

import math
import operator
from typing import Dict, Iterable, List, Optional

from . import dtypes as _dt
from .dtypes import DType, as_dtype

_var_counter = [0]


def _fresh_id() -> int:
    _var_counter[0] += 1
    return _var_counter[0]


class PrimExpr:
    """Base class of all scalar expressions."""

    __slots__ = ("dtype", )
    __array_priority__ = 1000  # win over numpy scalars in mixed arithmetic

    # ---- arithmetic -------------------------------------------------------
    def __add__(self, o):
        return binop("+", self, o)

    def __radd__(self, o):
        return binop("+", o, self)

    def __sub__(self, o):
        return binop("-", self, o)

    def __rsub__(self, o):
        return binop("-", o, self)

    def __mul__(self, o):
        return binop("*", self, o)

    def __rmul__(self, o):
        return binop("*", o, self)

    def __truediv__(self, o):
        return binop("/", self, o)

    def __rtruediv__(self, o):
        return binop("/", o, self)

    def __floordiv__(self, o):
        return binop("//", self, o)

    def __rfloordiv__(self, o):
        return binop("//", o, self)

    def __mod__(self, o):
        return binop("%", self, o)

    def __rmod__(self, o):
        return binop("%", o, self)

    def __neg__(self):
        return binop("-", const(0, self.dtype), self)

    def __pos__(self):
        return self

    def __abs__(self):
        return call("abs", [self], self.dtype)

    def __pow__(self, o):
        return call("pow", [self, o], self.dtype)

    def __lshift__(self, o):
        return binop("<<", self, o)

    def __rlshift__(self, o):
        return binop("<<", o, self)

    def __rshift__(self, o):
        return binop(">>", self, o)

    def __rrshift__(self, o):
        return binop(">>", o, self)

    def __and__(self, o):
        return binop("&", self, o)

    def __rand__(self, o):
        return binop("&", o, self)

    def __or__(self, o):
        return binop("|", self, o)

    def __ror__(self, o):
        return binop("|", o, self)

    def __xor__(self, o):
        return binop("^", self, o)

    def __rxor__(self, o):
        return binop("^", o, self)

    def __invert__(self):
        if self.dtype.is_bool:
            return logical_not(self)
        return UnOp("~", self)

    # ---- comparisons --------------------------------------------------------
    def __lt__(self, o):
        return binop("<", self, o)

    def __le__(self, o):
        return binop("<=", self, o)

    def __gt__(self, o):
        return binop(">", self, o)

    def __ge__(self, o):
        return binop(">=", self, o)

    def __eq__(self, o):  # type: ignore[override]
        return binop("==", self, o)

    def __ne__(self, o):  # type: ignore[override]
        return binop("!=", self, o)

    __hash__ = object.__hash__

    def __bool__(self):
        raise TypeError(
            f"symbolic expression `{self}` used as a Python bool; use T.if_then_else / an `if` "
            "statement inside the kernel instead")

    def __index__(self):
        raise TypeError(f"symbolic expression `{self}` cannot be used as a Python int")

    def __int__(self):
        raise TypeError(f"symbolic expression `{self}` cannot be used as a Python int")

    def __float__(self):
        raise TypeError(f"symbolic expression `{self}` cannot be used as a Python float")

    # convenience used by programs: x.astype("float32")
    def astype(self, dtype):
        return cast(self, dtype)

    def __repr__(self):
        from .printer import expr_str
        return expr_str(self)

    __str__ = __repr__

    def same_as(self, other) -> bool:
        return self is other


class IntImm(PrimExpr):
    __slots__ = ("value", )

    def __init__(self, value: int, dtype=_dt.int32):
        self.value = int(value)
        self.dtype = as_dtype(dtype)

    def __bool__(self):
        return bool(self.value)

    def __index__(self):
        return self.value

    def __int__(self):
        return self.value

    def __float__(self):
        return float(self.value)

    def __hash__(self):
        return hash(("IntImm", self.value, self.dtype))


class FloatImm(PrimExpr):
    __slots__ = ("value", )

    def __init__(self, value: float, dtype=_dt.float32):
        self.value = float(value)
        self.dtype = as_dtype(dtype)

    def __float__(self):
        return self.value

    def __hash__(self):
        return hash(("FloatImm", self.value, self.dtype))


class StringImm(PrimExpr):
    __slots__ = ("value", )

    def __init__(self, value: str):
        self.value = value
        self.dtype = _dt.handle

    def __hash__(self):
        return hash(("StringImm", self.value))


class Var(PrimExpr):
    """A scalar variable: loop var, thread/block index, shape symbol, let binding."""
    __slots__ = ("name", "uid", "nonneg", "hint")

    def __init__(self, name: str, dtype=_dt.int32, nonneg: Optional[bool] = None):
        self.name = name
        self.dtype = as_dtype(dtype)
        self.uid = _fresh_id()
        # integer vars created by the DSL (loop vars, thread ids, shapes) are >= 0
        self.nonneg = self.dtype.is_int if nonneg is None else nonneg
        self.hint = None

    __hash__ = object.__hash__


class BinOp(PrimExpr):
    __slots__ = ("op", "a", "b")

    def __init__(self, op: str, a: PrimExpr, b: PrimExpr, dtype: DType):
        self.op = op
        self.a = a
        self.b = b
        self.dtype = dtype

    def __bool__(self):
        # Mirror TVM: ``a == b`` on expressions is structural when forced to bool.
        if self.op == "==":
            return structural_equal(self.a, self.b)
        if self.op == "!=":
            return not structural_equal(self.a, self.b)
        return PrimExpr.__bool__(self)

    __hash__ = object.__hash__


class UnOp(PrimExpr):
    __slots__ = ("op", "a")

    def __init__(self, op: str, a: PrimExpr):
        self.op = op
        self.a = a
        self.dtype = _dt.boolean if op == "!" else a.dtype


class Cast(PrimExpr):
    __slots__ = ("value", )

    def __init__(self, dtype, value: PrimExpr):
        self.dtype = as_dtype(dtype)
        self.value = value


class Select(PrimExpr):
    __slots__ = ("cond", "t", "f")

    def __init__(self, cond, t, f):
        self.cond = cond
        self.t = t
        self.f = f
        self.dtype = t.dtype


class Call(PrimExpr):
    """An intrinsic / math call.  ``op`` is a name the emitters understand."""
    __slots__ = ("op", "args", "attrs")

    def __init__(self, op: str, args: List, dtype, attrs: Optional[dict] = None):
        self.op = op
        self.args = list(args)
        self.dtype = as_dtype(dtype)
        self.attrs = attrs or {}


class BufferLoad(PrimExpr):
    __slots__ = ("buffer", "indices")

    def __init__(self, buffer, indices: List[PrimExpr]):
        self.buffer = buffer
        self.indices = [convert(i) for i in indices]
        self.dtype = buffer.dtype


# ---------------------------------------------------------------------------
# construction helpers
# ---------------------------------------------------------------------------


def const(value, dtype=None) -> PrimExpr:
    if isinstance(value, PrimExpr):
        return value if dtype is None else cast(value, dtype)
    if isinstance(value, bool):
        return IntImm(int(value), _dt.boolean if dtype is None else dtype)
    if dtype is not None:
        dtype = as_dtype(dtype)
        if dtype.is_float:
            return FloatImm(float(value), dtype)
        return IntImm(int(value), dtype)
    if isinstance(value, int):
        return IntImm(value, _dt.int32 if -2**31 <= value < 2**31 else _dt.int64)
    if isinstance(value, float):
        return FloatImm(value, _dt.float32)
    try:
        import numpy as np
        if isinstance(value, np.integer):
            return IntImm(int(value))
        if isinstance(value, np.floating):
            return FloatImm(float(value))
    except ImportError:  # pragma: no cover
        pass
    raise TypeError(f"cannot convert {value!r} ({type(value).__name__}) to an expression")


def convert(value) -> PrimExpr:
    """Convert Python scalars / buffers used as scalars into PrimExpr."""
    if isinstance(value, PrimExpr):
        return value
    # a local.var buffer used as a value reads its single element
    from .buffer import Buffer
    if isinstance(value, Buffer):
        return value.as_scalar()
    return const(value)


def is_const(e) -> bool:
    return isinstance(e, (int, float, IntImm, FloatImm))


def const_value(e):
    if isinstance(e, (int, float)):
        return e
    if isinstance(e, (IntImm, FloatImm)):
        return e.value
    return None


def as_int(e) -> Optional[int]:
    """Return the Python int value of ``e`` if statically known."""
    if isinstance(e, bool):
        return int(e)
    if isinstance(e, int):
        return e
    if isinstance(e, IntImm):
        return e.value
    return None


_PYOPS = {
    "+": operator.add,
    "-": operator.sub,
    "*": operator.mul,
    "<": operator.lt,
    "<=": operator.le,
    ">": operator.gt,
    ">=": operator.ge,
    "==": operator.eq,
    "!=": operator.ne,
    "&": operator.and_,
    "|": operator.or_,
    "^": operator.xor,
    "<<": operator.lshift,
    ">>": operator.rshift,
    "min": min,
    "max": max,
    "&&": lambda a, b: bool(a) and bool(b),
    "||": lambda a, b: bool(a) or bool(b),
}

_CMP = {"<", "<=", ">", ">=", "==", "!=", "&&", "||"}


def _fold(op, a, b, dtype):
    av, bv = a.value, b.value
    if op in _PYOPS:
        r = _PYOPS[op](av, bv)
    elif op == "/":
        if dtype.is_float:
            r = av / bv
        else:
            r = int(av / bv)  # truncating, C semantics
    elif op == "//":
        r = math.floor(av / bv) if dtype.is_float else av // bv
    elif op == "%":
        r = math.fmod(av, bv) if dtype.is_float else av % bv
    else:
        return None
    if op in _CMP:
        return IntImm(int(bool(r)), _dt.boolean)
    return const(r, dtype)


def binop(op: str, a, b) -> PrimExpr:
    a = convert(a) if not isinstance(a, PrimExpr) else a
    b = convert(b) if not isinstance(b, PrimExpr) else b
    # python literals adopt the other side's type
    a, b = _unify(a, b)
    if op in _CMP:
        rdt = _dt.boolean
    elif op == "/" and not a.dtype.is_float and not b.dtype.is_float:
        rdt = a.dtype
    else:
        rdt = _dt.promote(a.dtype, b.dtype)
        if op in ("<<", ">>"):
            rdt = a.dtype
    if rdt.is_float and op not in _CMP:
        if a.dtype != rdt:
            a = cast(a, rdt)
        if b.dtype != rdt:
            b = cast(b, rdt)
    if isinstance(a, (IntImm, FloatImm)) and isinstance(b, (IntImm, FloatImm)):
        try:
            r = _fold(op, a, b, rdt)
        except ZeroDivisionError:
            r = None
        if r is not None:
            return r
    # algebraic identities (integers only for +0/*1 safety with floats is fine too)
    av, bv = const_value(a), const_value(b)
    if op == "+":
        if av == 0 and a.dtype == rdt or (av == 0 and not rdt.is_float):
            return b if b.dtype == rdt else cast(b, rdt)
        if bv == 0:
            return a if a.dtype == rdt else cast(a, rdt)
        # (x + c1) + c2 -> x + (c1+c2)
        if bv is not None and isinstance(a, BinOp) and a.op == "+" and is_const(a.b) and not rdt.is_float:
            return binop("+", a.a, const_value(a.b) + bv)
    elif op == "-":
        if bv == 0:
            return a
        if structural_equal(a, b) and not rdt.is_float:
            return const(0, rdt)
        if not rdt.is_float:
            la, lb = _linear_form(a), _linear_form(b)
            if la is not None and lb is not None:
                diff = dict(la)
                for k, (t, c) in lb.items():
                    if k in diff:
                        diff[k] = (diff[k][0], diff[k][1] - c)
                    else:
                        diff[k] = (t, -c)
                diff = {k: v for k, v in diff.items() if v[1] != 0}
                if all(k == "__const__" for k in diff):
                    return const(diff.get("__const__", (None, 0))[1], rdt)
    elif op == "*":
        if av == 1:
            return b
        if bv == 1:
            return a
        if (av == 0 or bv == 0) and not rdt.is_float:
            return const(0, rdt)
        if av is not None and bv is None:  # canonical: constant on the right
            return binop("*", b, a)
    elif op in ("//", "/"):
        if bv == 1:
            return a
        if av == 0 and not rdt.is_float:
            return const(0, rdt)
        # (x * c) // c -> x   when c divides cleanly
        if bv is not None and isinstance(a, BinOp) and a.op == "*" and isinstance(a.b, IntImm) \
                and not rdt.is_float and bv != 0 and a.b.value % bv == 0:
            return binop("*", a.a, a.b.value // bv)
    elif op == "%":
        if bv == 1 and not rdt.is_float:
            return const(0, rdt)
        if bv is not None and isinstance(a, BinOp) and a.op == "*" and isinstance(a.b, IntImm) \
                and not rdt.is_float and bv != 0 and a.b.value % bv == 0:
            return const(0, rdt)
    elif op == "&&":
        if av is not None:
            return b if av else const(False)
        if bv is not None:
            return a if bv else const(False)
    elif op == "||":
        if av is not None:
            return const(True) if av else b
        if bv is not None:
            return const(True) if bv else a
    return BinOp(op, a, b, rdt)


_TERM_KEYS = {}


def _term_key(e) -> str:
    # memoised by identity (the entry holds the node, so its id cannot be reused while cached):
    # the linear-form simplifier keys the same sub-terms over and over
    hit = _TERM_KEYS.get(id(e))
    if hit is not None and hit[0] is e:
        return hit[1]
    from .printer import Printer
    p = Printer()
    p.names = _IdNames()
    k = p.e(e)
    if len(_TERM_KEYS) > 65536:
        _TERM_KEYS.clear()
    _TERM_KEYS[id(e)] = (e, k)
    return k


class _IdNames:
    """Name vars by identity so structurally-equal keys mean the same variables."""

    def __call__(self, obj, base):
        return f"{base}#{id(obj)}"


def _linear_form(e, depth=0):
    """{key: (term, coeff)} with '__const__' for the constant, for +,-,*const trees (ints only)."""
    if depth > 24:
        return None
    if isinstance(e, IntImm):
        return {"__const__": (None, e.value)}
    if isinstance(e, BinOp) and e.op in ("+", "-"):
        la, lb = _linear_form(e.a, depth + 1), _linear_form(e.b, depth + 1)
        if la is None or lb is None:
            return None
        out = dict(la)
        sign = 1 if e.op == "+" else -1
        for k, (t, c) in lb.items():
            if k in out:
                out[k] = (out[k][0], out[k][1] + sign * c)
            else:
                out[k] = (t, sign * c)
        return out
    if isinstance(e, BinOp) and e.op == "*":
        cb, ca = const_value(e.b), const_value(e.a)
        if cb is not None and isinstance(cb, int):
            la = _linear_form(e.a, depth + 1)
            return None if la is None else {k: (t, c * cb) for k, (t, c) in la.items()}
        if ca is not None and isinstance(ca, int):
            lb = _linear_form(e.b, depth + 1)
            return None if lb is None else {k: (t, c * ca) for k, (t, c) in lb.items()}
    if isinstance(e, (Var, BinOp, Cast, Call, BufferLoad, Select, UnOp)):
        if not e.dtype.is_int:
            return None
        return {_term_key(e): (e, 1)}
    return None


def _unify(a: PrimExpr, b: PrimExpr):
    """Literal operands take the dtype of the non-literal side."""
    if a.dtype == b.dtype:
        return a, b
    if isinstance(a, (IntImm, FloatImm)) and not isinstance(b, (IntImm, FloatImm)):
        if isinstance(a, IntImm) and (b.dtype.is_int or b.dtype.is_float) and not a.dtype.is_bool:
            return const(a.value, b.dtype), b
        if isinstance(a, FloatImm) and b.dtype.is_float:
            return FloatImm(a.value, b.dtype), b
    if isinstance(b, (IntImm, FloatImm)) and not isinstance(a, (IntImm, FloatImm)):
        if isinstance(b, IntImm) and (a.dtype.is_int or a.dtype.is_float) and not b.dtype.is_bool:
            return a, const(b.value, a.dtype)
        if isinstance(b, FloatImm) and a.dtype.is_float:
            return a, FloatImm(b.value, a.dtype)
    if a.dtype.is_int and b.dtype.is_int and a.dtype.bits != b.dtype.bits:
        t = a.dtype if a.dtype.bits > b.dtype.bits else b.dtype
        return (cast(a, t) if a.dtype != t else a), (cast(b, t) if b.dtype != t else b)
    return a, b


def cast(value, dtype) -> PrimExpr:
    dtype = as_dtype(dtype)
    value = convert(value)
    if value.dtype == dtype:
        return value
    if isinstance(value, IntImm):
        if dtype.is_float:
            return FloatImm(float(value.value), dtype)
        return IntImm(value.value, dtype)
    if isinstance(value, FloatImm):
        if dtype.is_int or dtype.is_bool:
            return IntImm(int(value.value), dtype)
        return FloatImm(value.value, dtype)
    return Cast(dtype, value)


def call(op: str, args, dtype=None, **attrs) -> Call:
    args = [convert(a) if not isinstance(a, (PrimExpr, str)) else a for a in args]
    if dtype is None:
        dtype = args[0].dtype if args and isinstance(args[0], PrimExpr) else _dt.float32
    return Call(op, args, dtype, attrs)


def select(cond, t, f) -> PrimExpr:
    cond = convert(cond)
    t = convert(t)
    f = convert(f)
    t, f = _unify(t, f)
    if t.dtype != f.dtype:
        dt = _dt.promote(t.dtype, f.dtype)
        t, f = cast(t, dt), cast(f, dt)
    cv = const_value(cond)
    if cv is not None:
        return t if cv else f
    return Select(cond, t, f)


def logical_and(a, b):
    return binop("&&", a, b)


def logical_or(a, b):
    return binop("||", a, b)


def logical_not(a):
    a = convert(a)
    v = const_value(a)
    if v is not None:
        return const(not v)
    return UnOp("!", a)


def min_expr(a, b):
    return binop("min", a, b)


def max_expr(a, b):
    return binop("max", a, b)


def ceildiv(a, b):
    ai, bi = as_int(a), as_int(b)
    if ai is not None and bi is not None:
        return -(-ai // bi)
    return (convert(a) + (convert(b) - 1)) // b


# ---------------------------------------------------------------------------
# traversal utilities
# ---------------------------------------------------------------------------


def _no_children(e):
    return ()


_CHILD_FNS = (
    (BinOp, lambda e: (e.a, e.b)),
    (UnOp, lambda e: (e.a, )),
    (Cast, lambda e: (e.value, )),
    (Select, lambda e: (e.cond, e.t, e.f)),
    (Call, lambda e: tuple(a for a in e.args if isinstance(a, PrimExpr))),
    (BufferLoad, lambda e: tuple(e.indices)),
)
_children_of_type = {}


def _children_fn(t):
    for cls, fn in _CHILD_FNS:
        if issubclass(t, cls):
            return fn
    return _no_children


def children(e: PrimExpr):
    # one dict lookup per node instead of a chain of isinstance tests (the lowering passes walk
    # ~10^5 nodes per kernel)
    t = type(e)
    fn = _children_of_type.get(t)
    if fn is None:
        fn = _children_of_type[t] = _children_fn(t)
    return fn(e)


def post_order(e: PrimExpr):
    """Every node of ``e``, children (left to right) before their parent: the reverse of a
    pre-order walk that visits the last child first (iterative; a list)."""
    out = []
    stack = [e]
    get = _children_of_type.get
    while stack:
        n = stack.pop()
        out.append(n)
        t = type(n)
        fn = get(t)
        if fn is None:
            fn = _children_of_type[t] = _children_fn(t)
        stack.extend(fn(n))
    out.reverse()
    return out


def free_vars(e) -> List[Var]:
    seen = {}
    for n in post_order(e):
        if isinstance(n, Var):
            seen[id(n)] = n
        if isinstance(n, BufferLoad):
            for s in n.buffer.shape:
                if isinstance(s, PrimExpr):
                    for v in free_vars(s):
                        seen[id(v)] = v
    return list(seen.values())


def uses_var(e, var: Var) -> bool:
    return any(n is var for n in post_order(e))


def loads_of(e) -> List[BufferLoad]:
    return [n for n in post_order(e) if isinstance(n, BufferLoad)]


def substitute(e, vmap: Dict[Var, PrimExpr]):
    """Replace Vars (by identity) and rebuild with constant folding."""
    if not vmap:
        return e
    if isinstance(e, (int, float)):
        return e
    return _subst(e, vmap)


def _subst(e, vmap):
    if isinstance(e, Var):
        r = vmap.get(e, None)
        return e if r is None else convert(r)
    if isinstance(e, (IntImm, FloatImm, StringImm)):
        return e
    if isinstance(e, BinOp):
        a, b = _subst(e.a, vmap), _subst(e.b, vmap)
        if a is e.a and b is e.b:
            return e
        return binop(e.op, a, b)
    if isinstance(e, UnOp):
        a = _subst(e.a, vmap)
        if a is e.a:
            return e
        if e.op == "!":
            return logical_not(a)
        if e.op == "~" and isinstance(a, IntImm):
            return IntImm(~a.value, a.dtype)
        return UnOp(e.op, a)
    if isinstance(e, Cast):
        v = _subst(e.value, vmap)
        return e if v is e.value else cast(v, e.dtype)
    if isinstance(e, Select):
        c, t, f = _subst(e.cond, vmap), _subst(e.t, vmap), _subst(e.f, vmap)
        if c is e.cond and t is e.t and f is e.f:
            return e
        return select(c, t, f)
    if isinstance(e, Call):
        args = [(_subst(a, vmap) if isinstance(a, PrimExpr) else a) for a in e.args]
        if all(x is y for x, y in zip(args, e.args)):
            return e
        return Call(e.op, args, e.dtype, e.attrs)
    if isinstance(e, BufferLoad):
        idx = [_subst(i, vmap) for i in e.indices]
        if all(x is y for x, y in zip(idx, e.indices)):
            return e
        return BufferLoad(e.buffer, idx)
    return e


def transform(e, fn):
    """Bottom-up rewrite: ``fn(node)`` returns a replacement or None."""
    if not isinstance(e, PrimExpr):
        return e
    if isinstance(e, BinOp):
        a, b = transform(e.a, fn), transform(e.b, fn)
        n = e if (a is e.a and b is e.b) else binop(e.op, a, b)
    elif isinstance(e, UnOp):
        a = transform(e.a, fn)
        n = e if a is e.a else (logical_not(a) if e.op == "!" else UnOp(e.op, a))
    elif isinstance(e, Cast):
        v = transform(e.value, fn)
        n = e if v is e.value else cast(v, e.dtype)
    elif isinstance(e, Select):
        c, t, f = transform(e.cond, fn), transform(e.t, fn), transform(e.f, fn)
        n = e if (c is e.cond and t is e.t and f is e.f) else select(c, t, f)
    elif isinstance(e, Call):
        args = [transform(a, fn) for a in e.args]
        n = e if all(x is y for x, y in zip(args, e.args)) else Call(e.op, args, e.dtype, e.attrs)
    elif isinstance(e, BufferLoad):
        idx = [transform(i, fn) for i in e.indices]
        n = e if all(x is y for x, y in zip(idx, e.indices)) else BufferLoad(e.buffer, idx)
    else:
        n = e
    r = fn(n)
    return n if r is None else r


def widen_int64(e):
    """``e`` re-evaluated in int64 from the leaves up.  Casting an int32 result to int64 keeps
    its overflow (``(int64_t)(bx * 512 + t)`` past 2^31); widening the leaves does not."""
    e = convert(e)
    if not e.dtype.is_int or e.dtype.bits >= 64:
        return e

    def fn(n):
        if isinstance(n, (Var, BufferLoad, Call, Cast)) and n.dtype.is_int and n.dtype.bits < 64:
            return Cast(_dt.int64, n)
        return None

    r = transform(e, fn)
    return r if r.dtype.bits >= 64 else cast(r, _dt.int64)


def structural_equal(a, b) -> bool:
    if a is b:
        return True
    if isinstance(a, (int, float)) or isinstance(b, (int, float)):
        av = const_value(a) if isinstance(a, PrimExpr) else a
        bv = const_value(b) if isinstance(b, PrimExpr) else b
        return av is not None and av == bv
    if type(a) is not type(b):
        return False
    if isinstance(a, (IntImm, FloatImm)):
        return a.value == b.value and a.dtype == b.dtype
    if isinstance(a, StringImm):
        return a.value == b.value
    if isinstance(a, Var):
        return False
    if isinstance(a, BinOp):
        return a.op == b.op and structural_equal(a.a, b.a) and structural_equal(a.b, b.b)
    if isinstance(a, UnOp):
        return a.op == b.op and structural_equal(a.a, b.a)
    if isinstance(a, Cast):
        return a.dtype == b.dtype and structural_equal(a.value, b.value)
    if isinstance(a, Select):
        return all(structural_equal(x, y) for x, y in ((a.cond, b.cond), (a.t, b.t), (a.f, b.f)))
    if isinstance(a, Call):
        return a.op == b.op and len(a.args) == len(b.args) and all(
            (structural_equal(x, y) if isinstance(x, PrimExpr) else x == y)
            for x, y in zip(a.args, b.args))
    if isinstance(a, BufferLoad):
        return a.buffer is b.buffer and all(structural_equal(x, y) for x, y in zip(a.indices, b.indices))
    return False


# ---------------------------------------------------------------------------
# numeric evaluation (used by layout inference / verification)
# ---------------------------------------------------------------------------


class EvalError(Exception):
    pass


def _c_div(a, b):
    if isinstance(a, float) or isinstance(b, float):
        return a / b
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def evaluate(e, env: Dict[Var, object]):
    """Evaluate with Python semantics matching the emitted C++ (floordiv for //)."""
    if isinstance(e, (int, float)):
        return e
    if isinstance(e, (IntImm, FloatImm)):
        return e.value
    if isinstance(e, Var):
        if e in env:
            return env[e]
        raise EvalError(f"unbound variable {e.name}")
    if isinstance(e, BinOp):
        a = evaluate(e.a, env)
        b = evaluate(e.b, env)
        op = e.op
        if op in _PYOPS:
            r = _PYOPS[op](a, b)
            return bool(r) if op in _CMP else r
        if op == "/":
            return a / b if e.dtype.is_float else _c_div(a, b)
        if op == "//":
            return math.floor(a / b) if e.dtype.is_float else a // b
        if op == "%":
            return math.fmod(a, b) if e.dtype.is_float else a % b
        raise EvalError(op)
    if isinstance(e, UnOp):
        a = evaluate(e.a, env)
        return (not a) if e.op == "!" else ~a
    if isinstance(e, Cast):
        v = evaluate(e.value, env)
        if e.dtype.is_float:
            return float(v)
        if e.dtype.is_bool:
            return bool(v)
        return int(v)
    if isinstance(e, Select):
        return evaluate(e.t, env) if evaluate(e.cond, env) else evaluate(e.f, env)
    if isinstance(e, Call):
        fn = _EVAL_CALLS.get(e.op)
        if fn is None:
            raise EvalError(f"cannot evaluate call {e.op}")
        return fn(*[evaluate(a, env) for a in e.args])
    raise EvalError(f"cannot evaluate {type(e).__name__}")


_EVAL_CALLS = {
    "exp": math.exp,
    "exp2": lambda x: 2.0**x,
    "log": math.log,
    "log2": math.log2,
    "sqrt": math.sqrt,
    "rsqrt": lambda x: 1.0 / math.sqrt(x),
    "abs": abs,
    "min": min,
    "max": max,
    "floor": math.floor,
    "ceil": math.ceil,
    "tanh": math.tanh,
    "sin": math.sin,
    "cos": math.cos,
}


def compile_py(e, vars_: Iterable[Var]):
    """Compile ``e`` into a Python lambda over ``vars_`` (fast repeated evaluation)."""
    vars_ = list(vars_)
    names = {v: f"_v{i}" for i, v in enumerate(vars_)}

    def emit(x):
        if isinstance(x, (int, float)):
            return repr(x)
        if isinstance(x, IntImm):
            return repr(x.value)
        if isinstance(x, FloatImm):
            return repr(x.value)
        if isinstance(x, Var):
            if x not in names:
                raise EvalError(f"unbound variable {x.name}")
            return names[x]
        if isinstance(x, BinOp):
            a, b = emit(x.a), emit(x.b)
            if x.op in ("min", "max"):
                return f"{x.op}({a}, {b})"
            if x.op == "&&":
                return f"({a} and {b})"
            if x.op == "||":
                return f"({a} or {b})"
            if x.op == "/" and not x.dtype.is_float:
                return f"_cdiv({a}, {b})"
            return f"({a} {x.op} {b})"
        if isinstance(x, UnOp):
            return f"(not {emit(x.a)})" if x.op == "!" else f"(~{emit(x.a)})"
        if isinstance(x, Cast):
            if x.dtype.is_float:
                return f"float({emit(x.value)})"
            return f"int({emit(x.value)})"
        if isinstance(x, Select):
            return f"({emit(x.t)} if {emit(x.cond)} else {emit(x.f)})"
        raise EvalError(f"cannot compile {type(x).__name__}")

    src = f"lambda {', '.join(names[v] for v in vars_)}: {emit(e)}"
    return eval(src, {"_cdiv": _c_div})  # noqa: S307 - generated from our own IR


# ---------------------------------------------------------------------------
# modular (divisibility) analysis, used for vectorisation legality
# ---------------------------------------------------------------------------


def modular(e, known: Optional[Dict[Var, tuple]] = None):
    """Return (coeff, base) such that e == coeff*k + base for some integer k.

    coeff == 0 means e is the constant ``base``.  Unknown vars are (1, 0).
    """
    known = known or {}
    if isinstance(e, int):
        return (0, e)
    if isinstance(e, IntImm):
        return (0, e.value)
    if isinstance(e, Var):
        return known.get(e, (1, 0))
    if isinstance(e, Cast) and e.dtype.is_int:
        return modular(e.value, known)
    if isinstance(e, BinOp):
        if e.op in ("+", "-"):
            ca, ba = modular(e.a, known)
            cb, bb = modular(e.b, known)
            c = math.gcd(ca, cb)
            b = ba + bb if e.op == "+" else ba - bb
            return (c, b % c if c else b)
        if e.op == "*":
            ca, ba = modular(e.a, known)
            cb, bb = modular(e.b, known)
            if ca == 0 and cb == 0:
                return (0, ba * bb)
            if cb == 0:
                c = abs(ca * bb)
                return (c, (ba * bb) % c if c else ba * bb)
            if ca == 0:
                c = abs(cb * ba)
                return (c, (ba * bb) % c if c else ba * bb)
            c = math.gcd(math.gcd(ca * cb, ca * bb), cb * ba)
            return (c, (ba * bb) % c if c else ba * bb)
        if e.op == "<<":
            cb, bb = modular(e.b, known)
            if cb == 0:
                return modular(binop("*", e.a, 1 << bb), known)
        if e.op in ("//", "/"):
            ca, ba = modular(e.a, known)
            cb, bb = modular(e.b, known)
            if cb == 0 and bb > 0 and ca % bb == 0 and ba % bb == 0:
                if ca == 0:
                    return (0, ba // bb)
                return (ca // bb, (ba // bb) % (ca // bb))
            return (1, 0)
        if e.op == "%":
            ca, ba = modular(e.a, known)
            cb, bb = modular(e.b, known)
            if cb == 0 and bb > 0:
                g = math.gcd(ca, bb)
                if ca == 0:
                    return (0, ba % bb)
                return (g, ba % g)
            return (1, 0)
    return (1, 0)


def divisible_by(e, n: int, known=None) -> bool:
    c, b = modular(e, known)
    if c == 0:
        return b % n == 0
    return c % n == 0 and b % n == 0


def is_nonneg(e) -> bool:
    """Conservative proof that an integer expression is >= 0."""
    if isinstance(e, int):
        return e >= 0
    if isinstance(e, IntImm):
        return e.value >= 0
    if isinstance(e, Var):
        return bool(e.nonneg)
    if isinstance(e, Cast):
        return is_nonneg(e.value)
    if isinstance(e, BufferLoad):
        return False
    if isinstance(e, BinOp):
        if e.op in ("+", "*", "//", "%", "/", "min", "max", ">>", "&"):
            if e.op == "&" and (is_nonneg(e.a) or is_nonneg(e.b)):
                return True
            return is_nonneg(e.a) and is_nonneg(e.b)
        if e.op == "-":
            a, b = const_value(e.a), const_value(e.b)
            return a is not None and b is not None and a >= b
        if e.op in _CMP:
            return True
    if isinstance(e, Select):
        return is_nonneg(e.t) and is_nonneg(e.f)
    return False
