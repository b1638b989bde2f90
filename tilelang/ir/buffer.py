"""Buffers and buffer regions.

Scopes follow the reference (``tilelang/language/allocate.py:37-158``):

* ``global``          – a kernel argument in HBM (torch tensor)
* ``shared`` / ``shared.dyn`` – LDS (one arena per kernel on gfx950)
* ``local.fragment``  – a tile distributed over the block's lanes (registers)
* ``local``           – per-thread private array (registers)
* ``local.var``       – per-thread scalar variable (``T.alloc_var``)
"""
from __future__ import annotations

from typing import List, Optional, Sequence

from . import dtypes as _dt
from .expr import (BufferLoad, PrimExpr, Var, as_int, binop, const, convert, IntImm)

_buf_counter = [0]


def _norm_scope(scope: str) -> str:
    if scope in ("shared", "shared.dyn"):
        return "shared"
    if scope in ("local.fragment", "fragment"):
        return "fragment"
    if scope in ("local.var", "var"):
        return "var"
    return scope


# data-pointer var uid -> buffer (``T.Tensor(shape, dtype, buf.data)`` re-views a buffer's storage)
DATA_OWNERS = {}


class Buffer:
    """A typed n-d buffer.  Indexing builds loads/stores/regions."""

    def __init__(self, name: str, shape: Sequence, dtype, scope: str = "global",
                 strides: Optional[Sequence] = None, offset=0):
        _buf_counter[0] += 1
        self.uid = _buf_counter[0]
        self.name = name
        self.shape: List = [s if isinstance(s, PrimExpr) else int(s) for s in shape]
        self.dtype = _dt.as_dtype(dtype)
        self.scope = _norm_scope(scope)
        self.strides = list(strides) if strides is not None else None
        self.offset = offset
        self.data = Var(name, _dt.handle)
        DATA_OWNERS[self.data.uid] = self
        # filled by passes
        self.layout = None       # Layout for shared buffers (swizzle) / Fragment for fragments
        self.param_index = None  # position in the kernel signature (global buffers)
        self.alias_of = None     # (buffer, elem offset) for T.view / T.reshape aliases
        self.init_value = None   # for alloc_var(init=...)

    # ---- shape helpers -------------------------------------------------------
    @property
    def ndim(self) -> int:
        return len(self.shape)

    def static_shape(self) -> Optional[List[int]]:
        out = []
        for s in self.shape:
            v = as_int(s)
            if v is None:
                return None
            out.append(v)
        return out

    def numel(self):
        n = 1
        for s in self.shape:
            n = n * s
        return n

    def get_strides(self) -> List:
        if self.strides is not None:
            return self.strides
        st = []
        acc = 1
        for s in reversed(self.shape):
            st.append(acc)
            acc = acc * s if not (isinstance(acc, int) and isinstance(s, int)) else acc * s
        return list(reversed(st))

    def offset_of(self, indices, wide: bool = False) -> PrimExpr:
        """Row-major linear element offset of ``indices``.  ``wide``: computed in int64 (tensors
        of 2^31 elements or more; reference ``src/transform/config_index_bitwidth.cc``)."""
        from .expr import cast
        from . import dtypes as _dt
        strides = self.get_strides()
        off = convert(self.offset) if not isinstance(self.offset, int) or self.offset else const(0)
        if wide:
            off = cast(off, _dt.int64)
        from .expr import widen_int64
        for i, s in zip(indices, strides):
            t = convert(i)
            if wide and t.dtype.bits < 64:
                t = widen_int64(t)
            off = off + t * s
        return off

    def static_numel(self) -> Optional[int]:
        shp = self.static_shape()
        if shp is None:
            return None
        n = 1
        for s in shp:
            n *= s
        return n

    def is_scope(self, *scopes) -> bool:
        return self.scope in scopes

    # ---- indexing --------------------------------------------------------------
    def _norm_index(self, key):
        if not isinstance(key, tuple):
            key = (key, )
        if any(k is Ellipsis for k in key):
            i = [k is Ellipsis for k in key].index(True)
            fill = self.ndim - (len(key) - 1)
            key = key[:i] + (slice(None), ) * fill + key[i + 1:]
        return key

    def __getitem__(self, key):
        key = self._norm_index(key)
        if any(isinstance(k, slice) for k in key) or len(key) < self.ndim:
            return BufferRegion.from_key(self, key)
        if len(key) != self.ndim:
            if self.scope == "var" and len(key) == 1 and self.ndim == 1:
                pass
            else:
                raise IndexError(f"{self.name}: expected {self.ndim} indices, got {len(key)}")
        return BufferLoad(self, [_neg_index(k, s) for k, s in zip(key, self.shape)])

    def __setitem__(self, key, value):
        from ..language.builder import current_builder
        key = self._norm_index(key)
        if any(isinstance(k, slice) for k in key):
            # ``A[0, 4:8] = A[0, 0:4]`` is a tile copy, ``A[0, 4:8] = 0`` a fill
            from ..language import tileops
            dst = BufferRegion.from_key(self, key)
            if isinstance(value, (Buffer, BufferRegion)):
                tileops.copy(value, dst)
            else:
                tileops.fill(dst, value)
            return
        if len(key) != self.ndim:
            raise IndexError(f"{self.name}: expected {self.ndim} indices, got {len(key)}")
        current_builder().store(self, [_neg_index(k, s) for k, s in zip(key, self.shape)], value)

    # ---- scalar behaviour for local.var buffers ---------------------------------
    def as_scalar(self) -> PrimExpr:
        if self.scope == "var" or (self.scope == "local" and self.ndim == 1 and as_int(self.shape[0]) == 1):
            return BufferLoad(self, [IntImm(0)])
        raise TypeError(f"buffer {self.name} ({self.scope}) used as a scalar value")

    def _s(self):
        return self.as_scalar()

    def __add__(self, o):
        return self._s() + o

    def __radd__(self, o):
        return o + self._s()

    def __sub__(self, o):
        return self._s() - o

    def __rsub__(self, o):
        return o - self._s()

    def __mul__(self, o):
        return self._s() * o

    def __rmul__(self, o):
        return o * self._s()

    def __truediv__(self, o):
        return self._s() / o

    def __rtruediv__(self, o):
        return o / self._s()

    def __floordiv__(self, o):
        return self._s() // o

    def __rfloordiv__(self, o):
        return o // self._s()

    def __mod__(self, o):
        return self._s() % o

    def __rmod__(self, o):
        return o % self._s()

    def __neg__(self):
        return -self._s()

    def __lt__(self, o):
        return self._s() < o

    def __le__(self, o):
        return self._s() <= o

    def __gt__(self, o):
        return self._s() > o

    def __ge__(self, o):
        return self._s() >= o

    def __and__(self, o):
        return self._s() & o

    def __or__(self, o):
        return self._s() | o

    def __xor__(self, o):
        return self._s() ^ o

    def __lshift__(self, o):
        return self._s() << o

    def __rshift__(self, o):
        return self._s() >> o

    __hash__ = object.__hash__

    def __eq__(self, o):  # noqa: D105
        if isinstance(o, Buffer):
            return self is o
        if self.scope == "var":
            return binop("==", self._s(), o)
        return False

    def __ne__(self, o):  # noqa: D105
        if isinstance(o, Buffer):
            return self is not o
        if self.scope == "var":
            return binop("!=", self._s(), o)
        return True

    def __repr__(self):
        return f"Buffer({self.name}, {self.shape}, {self.dtype}, {self.scope})"

    # convenience accessors used in programs
    @property
    def access_ptr(self):
        return self.data


def _neg_index(k, extent):
    v = as_int(k)
    if v is not None and v < 0:
        e = as_int(extent)
        if e is not None:
            return e + v
        return convert(extent) + v
    return convert(k)


class BufferRegion:
    """A rectangular sub-region: per dimension (min, extent)."""

    def __init__(self, buffer: Buffer, region: List[tuple]):
        self.buffer = buffer
        self.region = [(convert(m), e if isinstance(e, PrimExpr) else int(e)) for m, e in region]

    @staticmethod
    def from_key(buffer: Buffer, key) -> "BufferRegion":
        region = []
        for d in range(buffer.ndim):
            if d >= len(key):
                region.append((const(0), buffer.shape[d]))
                continue
            k = key[d]
            if isinstance(k, slice):
                if k.step not in (None, 1):
                    raise IndexError("strided slices are not supported in buffer regions")
                start = 0 if k.start is None else _neg_index(k.start, buffer.shape[d])
                stop = buffer.shape[d] if k.stop is None else _neg_index(k.stop, buffer.shape[d])
                ext = stop - start
                ev = as_int(ext)
                region.append((convert(start), ev if ev is not None else ext))
            else:
                region.append((convert(_neg_index(k, buffer.shape[d])), 1))
        return BufferRegion(buffer, region)

    @staticmethod
    def full(buffer: Buffer) -> "BufferRegion":
        return BufferRegion(buffer, [(const(0), s) for s in buffer.shape])

    @property
    def mins(self):
        return [m for m, _ in self.region]

    @property
    def extents(self):
        return [e for _, e in self.region]

    def static_extents(self):
        out = []
        for e in self.extents:
            v = as_int(e)
            if v is None:
                return None
            out.append(v)
        return out

    @property
    def dtype(self):
        return self.buffer.dtype

    def __repr__(self):
        rs = ", ".join(f"{m}:{m}+{e}" for m, e in self.region)
        return f"{self.buffer.name}[{rs}]"


def to_region(x, extents_hint=None) -> BufferRegion:
    """Accept Buffer / BufferRegion / BufferLoad (a point: extents from hint)."""
    if isinstance(x, BufferRegion):
        return x
    if isinstance(x, Buffer):
        return BufferRegion.full(x)
    if isinstance(x, BufferLoad):
        buf = x.buffer
        if extents_hint is None:
            return BufferRegion(buf, [(i, 1) for i in x.indices])
        # align the hint to the trailing dims (reference: legalize_pairwise_extents,
        # tilelang/utils/language.py:408)
        nd = len(x.indices)
        hint = list(extents_hint)
        if len(hint) < nd:
            hint = [1] * (nd - len(hint)) + hint
        elif len(hint) > nd:
            # drop leading unit dims of the hint
            while len(hint) > nd and as_int(hint[0]) == 1:
                hint = hint[1:]
            if len(hint) > nd:
                raise ValueError(f"cannot map a {len(extents_hint)}-d tile onto {buf.name}[{nd}-d]")
        return BufferRegion(buf, list(zip(x.indices, hint)))
    raise TypeError(f"expected a buffer or region, got {type(x).__name__}")
