"""Tile operator records.

The reference registers each operator as ``tl.tileop.<name>`` with a
``TileOperatorNode`` that implements ``InferLayout`` and ``Lower``
(``src/op/operator.h:55-88``).  Here the records are plain data; layout
inference lives in ``tilelang/transform/layout_inference.py`` and lowering in
``tilelang/transform/lower_tile_op.py``.
"""
from __future__ import annotations

from typing import List, Optional

from .buffer import BufferRegion


class TileOp:
    kind = "tileop"

    def regions(self) -> List[BufferRegion]:
        return []

    def reads(self) -> List[BufferRegion]:
        return []

    def writes(self) -> List[BufferRegion]:
        return []


class CopyOp(TileOp):
    """``T.copy`` (reference ``src/op/copy.cc:131``)."""
    kind = "copy"

    def __init__(self, src: BufferRegion, dst: BufferRegion, coalesced_width: Optional[int] = None,
                 disable_tma: bool = False, eviction_policy: Optional[str] = None):
        self.src = src
        self.dst = dst
        self.coalesced_width = coalesced_width
        self.disable_tma = disable_tma
        self.eviction_policy = eviction_policy

    def regions(self):
        return [self.src, self.dst]

    def reads(self):
        return [self.src]

    def writes(self):
        return [self.dst]


class GatherRowsOp(TileOp):
    """``T.gather_rows(src, indices, dst)``: ``dst[r, :] = src[..., indices[r], ..., c0:c0+C]``;
    rows whose index falls outside ``[0, src.shape[row_dim])`` read zeros.  Data-dependent row
    gathers (sparse attention over selected KV rows, MoE token gathers) on MI355X map onto
    lane-addressed buffer LDS-DMA, so inside ``T.Pipelined`` they are asynchronous producers
    like a plain ``T.copy`` (no reference counterpart; the reference writes such gathers as
    SIMT ``T.Parallel`` loops)."""
    kind = "gather_rows"

    def __init__(self, src: BufferRegion, idx: BufferRegion, dst: BufferRegion, row_dim: int):
        self.src, self.idx, self.dst, self.row_dim = src, idx, dst, row_dim

    def regions(self):
        return [self.src, self.idx, self.dst]

    def reads(self):
        return [self.src, self.idx]

    def writes(self):
        return [self.dst]


class Im2ColOp(TileOp):
    """``T.c2d_im2col`` (reference ``src/op/copy.cc:1878``)."""
    kind = "im2col"

    def __init__(self, img: BufferRegion, col: BufferRegion, nhw_step, c_step, kernel, stride, dilation, pad):
        self.img, self.col = img, col
        self.nhw_step, self.c_step = nhw_step, c_step
        self.kernel, self.stride, self.dilation, self.pad = kernel, stride, dilation, pad

    def regions(self):
        return [self.img, self.col]

    def reads(self):
        return [self.img]

    def writes(self):
        return [self.col]


class GemmOp(TileOp):
    """``T.gemm`` (reference ``src/op/gemm_py.cc``, ``tilelang/tileop/gemm/gemm_mfma.py``)."""
    kind = "gemm"

    def __init__(self, A: BufferRegion, B: BufferRegion, C: BufferRegion, trans_A=False, trans_B=False,
                 policy=0, clear_accum=False, k_pack=1, wg_wait=0, scale_A=None, scale_B=None):
        self.A, self.B, self.C = A, B, C
        self.trans_A = bool(trans_A)
        self.trans_B = bool(trans_B)
        self.policy = int(policy)
        self.clear_accum = clear_accum
        self.k_pack = int(k_pack)
        self.wg_wait = wg_wait
        self.scale_A = scale_A  # block-scaled MX gemm (e8m0 scales), gfx950 only
        self.scale_B = scale_B
        self.a_fmt = self.b_fmt = None  # MX element formats ("e4m3", "e5m2", "e2m1")
        self.mfma_shape = None  # "16x16" / "32x32" (T.gemm(mfma_shape=...))
        self.E = None  # 2:4 sparse metadata of A (T.gemm_sp): A is then the compressed [M, K/2] tile
        self.valid_m = None  # T.gemm(valid_m=): block-uniform count of rows that need results
        self.valid_m_min = None  # T.gemm(valid_m_min=): rows below it need no update (register-A GEMMs)

    @property
    def is_mx(self) -> bool:
        return self.scale_A is not None

    @property
    def is_sp(self) -> bool:
        return self.E is not None

    def _extra(self):
        return ([self.scale_A, self.scale_B] if self.is_mx else []) + ([self.E] if self.is_sp else [])

    def regions(self):
        return [self.A, self.B, self.C] + self._extra()

    def reads(self):
        return [self.A, self.B, self.C] + self._extra()

    def writes(self):
        return [self.C]

    @property
    def M(self):
        e = self.C.static_extents()
        return e[-2]

    @property
    def N(self):
        e = self.C.static_extents()
        return e[-1]

    @property
    def K(self):
        e = self.A.static_extents()
        k = e[-2] if self.trans_A else e[-1]
        return 2 * k if self.a_fmt == "e2m1" else k


class FillOp(TileOp):
    """``T.fill`` / ``T.clear`` (reference ``src/op/fill.cc:61``)."""
    kind = "fill"

    def __init__(self, dst: BufferRegion, value):
        self.dst = dst
        self.value = value

    def regions(self):
        return [self.dst]

    def writes(self):
        return [self.dst]


REDUCE_KINDS = ("sum", "abssum", "max", "min", "absmax", "bitand", "bitor", "bitxor")


class ReduceOp(TileOp):
    """``T.reduce_*`` (reference ``src/op/reduce.cc:30``)."""
    kind = "reduce"

    def __init__(self, src: BufferRegion, dst: BufferRegion, reduce_type: str, dim: int, clear: bool):
        assert reduce_type in REDUCE_KINDS, reduce_type
        self.src = src
        self.dst = dst
        self.reduce_type = reduce_type
        self.dim = dim
        self.clear = clear

    def regions(self):
        return [self.src, self.dst]

    def reads(self):
        return [self.src] + ([] if self.clear else [self.dst])

    def writes(self):
        return [self.dst]


class CumSumOp(TileOp):
    """``T.cumsum`` (reference ``src/op/reduce.cc:496-560``)."""
    kind = "cumsum"

    def __init__(self, src: BufferRegion, dst: BufferRegion, dim: int, reverse: bool):
        self.src, self.dst, self.dim, self.reverse = src, dst, dim, reverse

    def regions(self):
        return [self.src, self.dst]

    def reads(self):
        return [self.src]

    def writes(self):
        return [self.dst]


class AtomicOp(TileOp):
    """Tile-level atomics ``T.atomic_add/max/min`` on regions (reference ``src/op/atomic_add.cc``)."""
    kind = "atomic"

    def __init__(self, op: str, dst: BufferRegion, src, return_prev=False, memory_order=None):
        self.op = op
        self.dst = dst
        self.src = src  # BufferRegion or scalar expr
        self.return_prev = return_prev
        self.memory_order = memory_order

    def regions(self):
        return [self.dst] + ([self.src] if isinstance(self.src, BufferRegion) else [])

    def reads(self):
        return [self.src] if isinstance(self.src, BufferRegion) else []

    def writes(self):
        return [self.dst]


class FinalizeReducerOp(TileOp):
    """``T.finalize_reducer`` (reference ``src/op/finalize_reducer.cc:72``)."""
    kind = "finalize_reducer"

    def __init__(self, buf: BufferRegion):
        self.buf = buf

    def regions(self):
        return [self.buf]

    def writes(self):
        return [self.buf]


# ---------------------------------------------------------------------------
# Mesh communication ops (reference fork additions: src/op/comm.cc)
# ---------------------------------------------------------------------------


class CommOp(TileOp):
    kind = "comm"
    mesh = None  # (nrow, ncol) the op was traced for


class CommBroadcastOp(CommOp):
    kind = "comm_broadcast"

    def __init__(self, src: BufferRegion, dst: BufferRegion, src_core, direction: str, size: int):
        self.src, self.dst, self.src_core, self.direction, self.size = src, dst, src_core, direction, size

    def regions(self):
        return [self.src, self.dst]

    def reads(self):
        return [self.src]

    def writes(self):
        return [self.dst]


class CommPutOp(CommOp):
    kind = "comm_put"

    def __init__(self, src: BufferRegion, dst: BufferRegion, src_core, dst_core, size: int):
        self.src, self.dst, self.src_core, self.dst_core, self.size = src, dst, src_core, dst_core, size

    def regions(self):
        return [self.src, self.dst]

    def reads(self):
        return [self.src]

    def writes(self):
        return [self.dst]


class CommAllGatherOp(CommOp):
    kind = "comm_allgather"

    def __init__(self, send: BufferRegion, recv: BufferRegion, direction: str, size: int):
        self.send, self.recv, self.direction, self.size = send, recv, direction, size

    def regions(self):
        return [self.send, self.recv]

    def reads(self):
        return [self.send]

    def writes(self):
        return [self.recv]


class CommAllReduceOp(CommOp):
    kind = "comm_allreduce"

    def __init__(self, src: BufferRegion, dst: BufferRegion, reduce_type: str, direction: str, dim: int,
                 clear: bool):
        self.src, self.dst, self.reduce_type = src, dst, reduce_type
        self.direction, self.dim, self.clear = direction, dim, clear
        self.tmp = None  # per-core partial reduction (allocated by T.comm.all_reduce)

    def regions(self):
        return [self.src, self.dst] + ([self.tmp] if self.tmp is not None else [])

    def reads(self):
        return [self.src]

    def writes(self):
        return [self.dst]


class CommBarrierOp(CommOp):
    kind = "comm_barrier"

    def __init__(self, group=None):
        self.group = group


class CommFenceOp(CommOp):
    kind = "comm_fence"
