"""Math intrinsics (reference ``tilelang/language/math_intrinsics.py``, ``fastmath.py``, TIR ``op.py``).

On gfx950 these lower to OCML (``__ocml_*``) calls or the hardware
transcendental instructions (``v_exp_f32`` = 2^x, ``v_log_f32``, ``v_rcp_f32``,
``v_rsq_f32``) for the ``__``-prefixed fast variants.
"""
from __future__ import annotations

from ..ir.expr import (call, cast as _cast, convert, select, binop, const, FloatImm, min_expr, max_expr,
                       ceildiv as _ceildiv)
from ..ir import dtypes as _dt


def _f(x):
    x = convert(x)
    if not x.dtype.is_float:
        x = _cast(x, _dt.float32)
    return x


def _unary(name):

    def fn(x):
        x = _f(x)
        return call(name, [x], x.dtype)

    fn.__name__ = name
    return fn


exp = _unary("exp")
exp2 = _unary("exp2")
exp10 = _unary("exp10")
log = _unary("log")
log2 = _unary("log2")
log10 = _unary("log10")
log1p = _unary("log1p")
expm1 = _unary("expm1")
sqrt = _unary("sqrt")
rsqrt = _unary("rsqrt")
sin = _unary("sin")
cos = _unary("cos")
tan = _unary("tan")
asin = _unary("asin")
acos = _unary("acos")
atan = _unary("atan")
sinh = _unary("sinh")
cosh = _unary("cosh")
tanh = _unary("tanh")
erf = _unary("erf")
sigmoid = _unary("sigmoid")
floor = _unary("floor")
ceil = _unary("ceil")
trunc = _unary("trunc")
round = _unary("round")  # noqa: A001
nearbyint = _unary("nearbyint")
rcp = _unary("rcp")

# fast-math (hardware transcendental) variants, reference fastmath.py
__exp = _unary("fast_exp")
__exp10 = _unary("fast_exp10")
__log = _unary("fast_log")
__log2 = _unary("fast_log2")
__log10 = _unary("fast_log10")
__tan = _unary("fast_tan")
__cos = _unary("fast_cos")
__sin = _unary("fast_sin")
fast_exp = __exp
fast_exp2 = _unary("fast_exp2")


def abs(x):  # noqa: A001
    x = convert(x)
    return call("abs", [x], x.dtype)


def fabs(x):
    return abs(x)


def pow(x, y):  # noqa: A001
    x = _f(x)
    return call("pow", [x, convert(y)], x.dtype)


def fmod(x, y):
    x = _f(x)
    return call("fmod", [x, convert(y)], x.dtype)


def atan2(y, x):
    y = _f(y)
    return call("atan2", [y, convert(x)], y.dtype)


def isnan(x):
    return call("isnan", [convert(x)], _dt.boolean)


def isinf(x):
    return call("isinf", [convert(x)], _dt.boolean)


def isfinite(x):
    return call("isfinite", [convert(x)], _dt.boolean)


def max(a, b, *rest):  # noqa: A001
    r = max_expr(a, b)
    for x in rest:
        r = max_expr(r, x)
    return r


def min(a, b, *rest):  # noqa: A001
    r = min_expr(a, b)
    for x in rest:
        r = min_expr(r, x)
    return r


def clamp(x, min_val=None, max_val=None):
    """``min(max(x, min_val), max_val)``; a bound left as None is not applied."""
    if min_val is not None:
        x = max_expr(x, min_val)
    if max_val is not None:
        x = min_expr(x, max_val)
    return x


def if_then_else(cond, t, f):
    return select(cond, t, f)


def Select(cond, t, f):  # noqa: N802 - TIR spelling
    return select(cond, t, f)


def Cast(dtype, value):  # noqa: N802 - TIR spelling
    return _cast(value, dtype)


def cast(value, dtype):
    return _cast(value, dtype)


def infinity(dtype="float32"):
    return FloatImm(float("inf"), _dt.as_dtype(dtype))


def ninf(dtype="float32"):
    return FloatImm(float("-inf"), _dt.as_dtype(dtype))


def max_value(dtype):
    return const(_dt.max_value(dtype), dtype)


def min_value(dtype):
    return const(_dt.min_value(dtype), dtype)


def ceildiv(a, b):
    return _ceildiv(a, b)


def floordiv(a, b):
    return binop("//", a, b)


def floormod(a, b):
    return binop("%", a, b)


def truncdiv(a, b):
    return binop("/", a, b)


def truncmod(a, b):
    return binop("%", a, b)


def shift_left(a, b):
    return binop("<<", a, b)


def shift_right(a, b):
    return binop(">>", a, b)


def bitwise_and(a, b):
    return binop("&", a, b)


def bitwise_or(a, b):
    return binop("|", a, b)


def bitwise_xor(a, b):
    return binop("^", a, b)


def bitwise_not(a):
    return ~convert(a)


def And(a, b):  # noqa: N802
    return binop("&&", a, b)


def Or(a, b):  # noqa: N802
    return binop("||", a, b)


def Not(a):  # noqa: N802
    from ..ir.expr import logical_not
    return logical_not(a)


def fma(a, b, c):
    a = _f(a)
    return call("fma", [a, convert(b), convert(c)], a.dtype)


# IEEE rounding-mode variants (reference math_intrinsics.py ieee_*); gfx950 uses the
# default round-to-nearest-even for these in HIP source; we keep the API.
def ieee_add(a, b, rounding="rn"):
    return binop("+", a, b)


def ieee_sub(a, b, rounding="rn"):
    return binop("-", a, b)


def ieee_mul(a, b, rounding="rn"):
    return binop("*", a, b)


def ieee_fmaf(a, b, c, rounding="rn"):
    return fma(a, b, c)


def ieee_frcp(a, rounding="rn"):
    return binop("/", const(1.0, convert(a).dtype), a)


def ieee_fsqrt(a, rounding="rn"):
    return sqrt(a)


def ieee_frsqrt(a, rounding="rn"):
    return rsqrt(a)


def ieee_fdiv(a, b, rounding="rn"):
    return binop("/", a, b)


def dp4a(a, b, c):
    """int8x4 dot product accumulate (gfx950 ``v_dot4_i32_i8``)."""
    return call("tl.dp4a", [convert(a), convert(b), convert(c)], _dt.int32)


def reinterpret(value, dtype):
    return call("tl.reinterpret", [convert(value)], _dt.as_dtype(dtype))


def pack_b16(a, b):
    return call("tl.pack_b16", [convert(a), convert(b)], _dt.uint32)
