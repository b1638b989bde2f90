"""Buffer / region helpers (reference: tilelang/utils/language.py): scope predicates,
region conversion and shape/stride/offset retrieval used by tile ops and the Mesh comm ops."""
from __future__ import annotations

from typing import List

from ..ir.buffer import Buffer, BufferRegion, to_region
from ..ir.expr import BufferLoad, PrimExpr, as_int


def _buf(x) -> Buffer:
    if isinstance(x, Buffer):
        return x
    if isinstance(x, (BufferRegion, BufferLoad)):
        return x.buffer
    raise TypeError(f"expected a buffer, region or load, got {type(x).__name__}")


def is_global(x) -> bool:
    return _buf(x).scope == "global"


def is_shared(x, allow_dynamic: bool = True) -> bool:
    return _buf(x).scope in ("shared", "shared.dyn")


def is_shared_dynamic(x) -> bool:
    return is_shared(x)


def is_fragment(x) -> bool:
    return _buf(x).scope == "fragment"


def is_local(x) -> bool:
    return _buf(x).scope in ("local", "var")


def to_buffer_region(x, extents=None) -> BufferRegion:
    """Buffer / BufferLoad / BufferRegion -> BufferRegion (point loads take ``extents``)."""
    return to_region(x, extents)


def retrieve_shape(x) -> List[PrimExpr]:
    if isinstance(x, Buffer):
        return list(x.shape)
    return list(to_region(x).extents)


def retrieve_stride(x) -> List[PrimExpr]:
    return list(_buf(x).get_strides())


def retrieve_offset(x) -> List[PrimExpr]:
    if isinstance(x, Buffer):
        return [0] * len(x.shape)
    return list(to_region(x).mins)


def retrieve_ptr(x):
    """The ``tl.address_of`` expression of the region's first element."""
    from ..language.builtin import address_of
    r = to_region(x)
    return address_of(BufferLoad(r.buffer, list(r.mins)))


def prim_expr_equal(a, b) -> bool:
    from ..ir.expr import structural_equal
    return structural_equal(a, b)


def legalize_pairwise_extents(src_extents, dst_extents):
    """Right-align two extent lists, dropping leading unit dims of the longer one (the rule
    ``T.copy`` uses to pair a tile with a tensor region)."""
    s, d = list(src_extents), list(dst_extents)
    while len(s) > len(d) and as_int(s[0]) == 1:
        s = s[1:]
    while len(d) > len(s) and as_int(d[0]) == 1:
        d = d[1:]
    return s, d
