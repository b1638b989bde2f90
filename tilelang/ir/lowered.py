"""Lowered (per-thread / SIMT) IR constructs produced by ``transform/lower_tile_op.py``.

After lowering every buffer access is *flat*: global tensors are indexed by
their linear element offset (strides applied), shared buffers by their
physical (swizzled) element offset inside the buffer's LDS slot, fragments by
the per-thread register index of their ``local`` array.
"""
from __future__ import annotations

from typing import List, Sequence

from .expr import PrimExpr, convert
from . import dtypes as _dt
from .stmt import Stmt


class BufferPtr(PrimExpr):
    """``&buffer[offset]`` — a typed pointer into a (flat) buffer."""
    __slots__ = ("buffer", "offset")

    def __init__(self, buffer, offset=0):
        self.buffer = buffer
        self.offset = convert(offset)
        self.dtype = _dt.handle


class CallStmt(Stmt):
    """``name<targs...>(args...);`` — a device-library template call."""

    def __init__(self, name: str, args: Sequence = (), targs: Sequence = ()):
        self.name = name
        self.args = list(args)
        self.targs = [str(t) for t in targs]


class VecStoreStmt(Stmt):
    """Store ``len(values)`` consecutive elements ``buffer[index : index+n]`` as one vector."""

    def __init__(self, buffer, index, values: List[PrimExpr]):
        self.buffer = buffer
        self.index = convert(index)
        self.values = list(values)


class VecLoadStmt(Stmt):
    """Load ``n`` consecutive elements of ``src[src_index:]`` into ``dst[dst_index:]`` (a local array)."""

    def __init__(self, dst, dst_index: int, src, src_index, n: int):
        self.dst = dst
        self.dst_index = dst_index
        self.src = src
        self.src_index = convert(src_index)
        self.n = n


class CopyBytesStmt(Stmt):
    """Vectorised raw copy of ``nbytes`` (1..16) between flat buffers of the same dtype."""

    def __init__(self, dst, dst_index, src, src_index, nbytes: int):
        self.dst = dst
        self.dst_index = convert(dst_index)
        self.src = src
        self.src_index = convert(src_index)
        self.nbytes = nbytes


class CommentStmt(Stmt):

    def __init__(self, text: str):
        self.text = text


class PtrDeclStmt(Stmt):
    """``T* name = reinterpret_cast<T*>(ptr);`` — a flat global view at a runtime address
    (e.g. a peer GPU's mesh workspace slot)."""

    def __init__(self, buffer, ptr):
        self.buffer = buffer
        self.ptr = ptr


class ObjDeclStmt(Stmt):
    """``ctype name;`` — a value of a device-library struct type (e.g. ``tl::ss_frags<...>``, the
    register fragments a prefetched GEMM keeps across pipeline phases)."""

    def __init__(self, ctype: str, var):
        self.ctype = ctype
        self.var = var


class AutoLetStmt(Stmt):
    """``const auto name = value;`` for values of device-library struct type."""

    def __init__(self, var, value):
        self.var = var
        self.value = value
