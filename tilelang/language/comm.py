"""``T.comm``: inter-core (inter-GPU) tile communication on a 2-D device mesh.

Reference (fork addition): ``tilelang/language/comm.py:1-474`` + ``src/op/comm.cc``.
The reference stops at TIR (``tl.broadcast_`` has no code generator); here a
mesh core is one MI355X GPU of the node and the ops lower to device-initiated
xGMI peer stores into IPC-mapped symmetric workspaces with flag hand-offs
(``include/tl/mesh.h``, ``tilelang/parallel/mesh.py``).

Conventions kept from the reference:
  * mesh shape ``{"x": nrow, "y": ncol}``; linear core id = ``row*ncol + col``;
  * direction "horizontal"/"h" moves along a row (ncol peers), "vertical"/"v" along a
    column (nrow peers), "all"/"a" over the whole mesh;
  * ``all_gather`` recv shape must be ``[n] + send.shape``.
"""
from __future__ import annotations

from typing import Tuple, Union

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.buffer import Buffer, to_region
from ..ir.expr import IntImm, call, convert
from ..ir import dtypes as _dt
from .builder import current_builder

DIRECTION_MAP = {"horizontal": 0, "h": 0, "vertical": 1, "v": 1, "all": 2, "a": 2}
DIRECTION_NAMES = {0: "h", 1: "v", 2: "all"}
REDUCE_TYPE_LIST = ("sum", "abssum", "max", "min", "absmax", "bitand", "bitor", "bitxor")


def get_target_mesh_shape():
    from ..parallel.mesh import get_device_mesh_config
    nrow, ncol = get_device_mesh_config()
    return {"x": nrow, "y": ncol}


def core_tuple_to_id(core_id: Tuple[int, int]) -> int:
    m = get_target_mesh_shape()
    row, col = core_id
    assert 0 <= row < m["x"], f"Row {row} out of bounds for mesh shape {m}."
    assert 0 <= col < m["y"], f"Col {col} out of bounds for mesh shape {m}."
    return row * m["y"] + col


def core_id_to_tuple(core_id):
    m = get_target_mesh_shape()
    return (core_id // m["y"], core_id % m["y"])


def CoreId(core_id: Union[int, Tuple[int, int]]):  # noqa: N802
    m = get_target_mesh_shape()
    if isinstance(core_id, tuple):
        v = core_tuple_to_id(core_id)
    elif isinstance(core_id, int):
        assert 0 <= core_id < m["x"] * m["y"], f"Core ID {core_id} out of bounds for mesh shape {m}"
        v = core_id
    else:
        raise ValueError("core_id must be either a tuple[int, int] or an int.")
    return IntImm(v)


def current_core():
    return call("tl.mesh_rank", [], _dt.int32)


def is_current_core(core):
    return current_core() == convert(core)


def _mesh_tuple():
    m = get_target_mesh_shape()
    return (m["x"], m["y"])


def _emit(op):
    op.mesh = _mesh_tuple()
    current_builder().emit(S.TileOpStmt(op))


def _shape(b):
    return list(b.shape) if isinstance(b, Buffer) else list(b.extents)


def _numel(shape):
    n = 1
    for s in shape:
        n *= int(s)
    return n


def _check_core(c, m, what):
    assert isinstance(c, tuple) and len(c) == 2, f"{what} must be a tuple of (row, col)."
    assert 0 <= c[0] < m["x"], f"{what} row {c[0]} out of bounds for mesh shape {m}."
    assert 0 <= c[1] < m["y"], f"{what} col {c[1]} out of bounds for mesh shape {m}."


def _check_pair(src, dst, what):
    assert src.dtype == dst.dtype, (f"Source and destination buffer dtypes must match for {what}. "
                                    f"Got {src.dtype} vs {dst.dtype}.")
    ss, ds = _shape(src), _shape(dst)
    if len(ss) != len(ds):
        raise ValueError(f"Source and destination buffer must have the same number of dimensions for {what}.")
    for a, b in zip(ss, ds):
        assert a == b or a == 1 or b == 1, f"Source buffer shape and destination buffer shape must match for {what}."


def broadcast(src, dst, src_core, direction: str = "all", size: int = -1):
    _check_pair(src, dst, "broadcast")
    m = get_target_mesh_shape()
    _check_core(src_core, m, "src_core")
    n = _numel(_shape(src))
    assert isinstance(size, int) and size >= -1, "size must be an integer >= -1."
    assert size <= n, f"size {size} exceeds source buffer size {n}."
    assert direction.lower() in DIRECTION_MAP, f"Invalid direction string: {direction}"
    op = O.CommBroadcastOp(to_region(src), to_region(dst), core_tuple_to_id(src_core),
                           DIRECTION_NAMES[DIRECTION_MAP[direction.lower()]], n if size == -1 else size)
    _emit(op)


def put(src, dst, src_core, dst_core, size: int = -1):
    _check_pair(src, dst, "put")
    m = get_target_mesh_shape()
    _check_core(src_core, m, "src_core")
    _check_core(dst_core, m, "dst_core")
    n = _numel(_shape(src))
    assert isinstance(size, int) and size >= -1, "size must be an integer >= -1."
    assert size <= n, f"size {size} exceeds source buffer size {n}."
    op = O.CommPutOp(to_region(src), to_region(dst), core_tuple_to_id(src_core), core_tuple_to_id(dst_core),
                     n if size == -1 else size)
    _emit(op)


def all_gather(send_buffer, recv_buffer, direction: str = "all", size: int = -1):
    assert direction.lower() in DIRECTION_MAP, f"Invalid direction string: {direction}"
    assert send_buffer.dtype == recv_buffer.dtype, "Source and destination buffer dtypes must match for all_gather."
    m = get_target_mesh_shape()
    d = DIRECTION_MAP[direction.lower()]
    recv_num = {0: m["y"], 1: m["x"], 2: m["x"] * m["y"]}[d]
    expected = [recv_num] + _shape(send_buffer)
    assert [int(x) for x in _shape(recv_buffer)] == [int(x) for x in expected], (
        f"Receive buffer shape must be {expected} to hold gathered data from {recv_num} cores, "
        f"but got {_shape(recv_buffer)}.")
    n = _numel(_shape(send_buffer))
    assert isinstance(size, int) and size >= -1, "size must be an integer >= -1."
    assert size <= n, f"size {size} exceeds send buffer size {n}."
    op = O.CommAllGatherOp(to_region(send_buffer), to_region(recv_buffer), DIRECTION_NAMES[d],
                           n if size == -1 else size)
    _emit(op)


def all_reduce(buffer, out, reduce_type: str, direction: str = "all", dim: int = -1, clear: bool = True):
    shape = [int(x) for x in _shape(buffer)]
    assert isinstance(dim, int) and -1 <= dim < len(shape), f"dim {dim} out of bounds"
    if dim == -1:
        dim = len(shape) - 1
    oshape = [int(x) for x in _shape(out)]
    expected = [shape[:dim] + shape[dim + 1:], shape[:dim] + [1] + shape[dim + 1:]]
    if oshape not in expected:
        raise ValueError(f"Invalid reduce output shape, buffer shape is {shape}, dim is {dim}, "
                         f"output shape is {oshape}, expected shapes are {expected[0]} or {expected[1]}")
    reduce_type = reduce_type.lower()
    assert reduce_type in REDUCE_TYPE_LIST, f"Reduction op must be one of {REDUCE_TYPE_LIST}, but got {reduce_type}."
    assert direction.lower() in DIRECTION_MAP, f"Invalid direction string: {direction}"
    assert clear in (True, False), "clear must be a boolean value."
    op = O.CommAllReduceOp(to_region(buffer), to_region(out), reduce_type,
                           DIRECTION_NAMES[DIRECTION_MAP[direction.lower()]], dim, clear)
    # per-core partial (local reduce along `dim`), same scope as `out` — the reference allocates
    # its row/col gather fragments here too (language/comm.py:340-433)
    ob = out if isinstance(out, Buffer) else out.buffer
    from .allocate import alloc_fragment, alloc_shared
    alloc = alloc_shared if ob.scope == "shared" else alloc_fragment
    tmp = alloc(oshape, ob.dtype)
    tmp.name = f"{ob.name}_partial"
    tmp._auto_name = False
    op.tmp = to_region(tmp)
    _emit(op)


def all_reduce_tile(src, dst, reduce_type: str = "sum", direction: str = "all", clear: bool = True):
    """Element-wise reduction of a whole tile across the cores of a group (no local reduce):
    ``dst = op_{c in group} src@c`` (``clear=False``: ``dst = dst op ...``).  Extension over the
    reference API for tensor-parallel partial sums (e.g. a row-parallel GEMM's output tile)."""
    assert src.dtype == dst.dtype if isinstance(src, Buffer) and isinstance(dst, Buffer) else True
    if [int(x) for x in _shape(src)] != [int(x) for x in _shape(dst)]:
        raise ValueError(f"all_reduce_tile: src shape {_shape(src)} != dst shape {_shape(dst)}")
    reduce_type = reduce_type.lower()
    assert reduce_type in ("sum", "max", "min", "bitand", "bitor", "bitxor"), f"bad reduce type {reduce_type}"
    assert direction.lower() in DIRECTION_MAP, f"Invalid direction string: {direction}"
    op = O.CommAllReduceOp(to_region(src), to_region(dst), reduce_type,
                           DIRECTION_NAMES[DIRECTION_MAP[direction.lower()]], None, clear)
    _emit(op)


def barrier(group=None):
    """Synchronise a group of cores (default: the whole mesh).  ``group`` is an iterable of
    ``(row, col)`` tuples (reference ``language/comm.py:436-459``)."""
    m = get_target_mesh_shape()
    ids = None
    if group is not None:
        ids = []
        for c in group:
            _check_core(tuple(c), m, "barrier core")
            ids.append(core_tuple_to_id(tuple(c)))
        if len(set(ids)) != len(ids):
            raise ValueError(f"duplicate core in barrier group {group}")
    _emit(O.CommBarrierOp(ids))


def fence():
    _emit(O.CommFenceOp())
