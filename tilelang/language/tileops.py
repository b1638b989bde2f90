"""Tile operators: ``T.copy``, ``T.gemm``, ``T.fill``, ``T.reduce_*``, ``T.cumsum``, atomics.

Reference frontends: ``tilelang/language/{copy,gemm,fill,reduce,atomic,customize}.py``.
"""
from __future__ import annotations

from enum import IntEnum
from typing import Optional

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.buffer import Buffer, BufferRegion, to_region
from ..ir.expr import BufferLoad, PrimExpr, convert, call, const, as_int
from .builder import current_builder


def _emit(op):
    current_builder().emit(S.TileOpStmt(op))
    return None


def _extents_of(x):
    if isinstance(x, Buffer):
        return list(x.shape)
    if isinstance(x, BufferRegion):
        return list(x.extents)
    return None


def _pair_regions(src, dst):
    """Resolve point loads against the other operand's extents (legalize_pairwise_extents)."""
    se, de = _extents_of(src), _extents_of(dst)
    if se is None and de is None:
        # both points: a single-element copy
        return to_region(src), to_region(dst)
    s = to_region(src, de if se is None else None)
    d = to_region(dst, se if de is None else None)
    return s, d


def copy(src, dst, coalesced_width: Optional[int] = None, disable_tma: bool = False,
         eviction_policy: Optional[str] = None, loop_layout=None):
    if isinstance(src, (int, float, PrimExpr)) and not isinstance(src, BufferLoad):
        # T.copy(scalar, dst) == fill
        return fill(dst, src)
    if isinstance(src, BufferLoad) and isinstance(dst, BufferLoad):
        # one element to one element (also inside T.Parallel): a plain store
        current_builder().store(dst.buffer, list(dst.indices), src)
        return None
    s, d = _pair_regions(src, dst)
    if eviction_policy not in (None, "evict_normal", "evict_first", "evict_last"):
        raise ValueError(f"T.copy: eviction_policy must be evict_normal / evict_first / evict_last, "
                         f"got {eviction_policy!r}")
    if eviction_policy == "evict_first":
        # streamed-once global operand: non-temporal vector accesses (codegen/hip.py _nt)
        for r in (s, d):
            if r.buffer.scope == "global":
                r.buffer.nontemporal = True
    return _emit(O.CopyOp(s, d, coalesced_width, disable_tma, eviction_policy))


def gather_rows(src, indices, dst, row_dim: Optional[int] = None):
    """Row gather into a shared tile: ``dst[r, :] = src[..., indices[r], ..., cols]``.

    ``src`` is a global tensor region whose ``row_dim`` is the gathered dimension (its region
    start/extent are ignored; write ``:``) and whose last non-unit dim gives the columns;
    ``indices`` is a 1-D region (global or shared int32) with one index per tile row.  Indices
    outside ``[0, src.shape[row_dim])`` yield zero rows.  Inside ``T.Pipelined`` it is issued
    asynchronously (buffer LDS-DMA with per-lane row addresses)."""
    s, i, d = to_region(src), to_region(indices), to_region(dst)
    if row_dim is None:
        nonunit = [k for k, e in enumerate(s.extents) if as_int(e) != 1]
        if len(nonunit) != 2:
            raise ValueError("T.gather_rows: give row_dim (source region needs one row and one column dim)")
        row_dim = nonunit[0]
    return _emit(O.GatherRowsOp(s, i, d, int(row_dim)))


def c2d_im2col(img, col, nhw_step, c_step, kernel, stride, dilation, pad, eviction_policy=None):
    return _emit(O.Im2ColOp(to_region(img), to_region(col), convert(nhw_step), convert(c_step), kernel, stride,
                            dilation, pad))


class GemmWarpPolicy(IntEnum):
    """Warp partition policy (reference ``tilelang/primitives/gemm/base.py:8-15``)."""
    Square = 0
    FullRow = 1
    FullCol = 2

    def compute_warp_partition(self, M: int, N: int, num_warps: int):
        from ..transform.gemm_lower import compute_warp_partition
        return compute_warp_partition(M, N, num_warps, int(self))


def gemm(A, B, C, transpose_A: bool = False, transpose_B: bool = False, policy=GemmWarpPolicy.Square,
         clear_accum=False, k_pack: int = 1, wg_wait: int = 0, mbar=None, mfma_shape: Optional[str] = None,
         valid_m=None, valid_m_min=None):
    """Tile GEMM ``C (+)= op(A) @ op(B)`` on the gfx950 matrix cores.  Inputs f16/bf16 (MFMA
    16x16x32, or 32x32x16 with ``mfma_shape="32x32"`` / pass config ``tl.mfma_shape``), fp8
    (16x16x32 / scaled 16x16x128), int8 (int32 accumulator; 16x16x64 or 32x32x32) and fp32
    (16x16x4, exact f32).  ``wg_wait`` / ``mbar`` are NVIDIA-only and must stay at their defaults.

    ``valid_m`` (MI355X extension, f16/bf16 shared-operand GEMMs): a block-uniform row count; waves
    whose accumulator rows all lie at or past it skip their MFMAs and operand reads, leaving those
    rows of C unspecified.  For row tiles that are only partly filled (the padded per-expert row
    tiles of a MoE grouped GEMM): a 20-row tail tile costs one wave's MFMAs, not the whole tile's.

    ``valid_m_min`` (register-A GEMMs, MI355X extension): a block-uniform row index; waves whose
    accumulator rows all lie BELOW it skip their MFMAs.  The caller guarantees those rows would
    receive nothing (e.g. the query rows of a causal-diagonal attention tile that see none of its
    keys: -inf scores, zero probabilities), so C is the same either way (the CPU target computes
    them)."""
    if wg_wait not in (0, None) or mbar is not None:
        raise NotImplementedError("T.gemm: wg_wait / mbar are WGMMA / mbarrier (NVIDIA) features")
    A, B, C = to_region(A), to_region(B), to_region(C)
    op = O.GemmOp(A, B, C, transpose_A, transpose_B, int(policy), clear_accum, k_pack, wg_wait)
    op.mfma_shape = mfma_shape
    if valid_m is not None:
        op.valid_m = convert(valid_m)
    if valid_m_min is not None:
        op.valid_m_min = convert(valid_m_min)
    return _emit(op)


gemm_v1 = gemm
gemm_v2 = gemm


def gemm_sp(A_sparse, E, B, C, transpose_A: bool = False, transpose_B: bool = False,
            policy=GemmWarpPolicy.Square, clear_accum=False, k_pack: int = 1, wg_wait: int = 0):
    """2:4 structured-sparse tile GEMM ``C (+)= decompress(A_sparse, E) @ op(B)`` on gfx950
    ``v_smfmac_f32_16x16x64_{f16,bf16}`` (reference ``tilelang/language/experimental/gemm_sp.py:17``,
    ``src/op/gemm_sp.cc:147``).

    ``A_sparse``: ``[M, K/2]`` (or ``[K/2, M]`` with ``transpose_A``) f16/bf16 — the two kept
    values of every group of 4 along K, in order.  ``E``: ``[M, K/16]`` int16 metadata — bits
    ``[2v+1:2v]`` of word ``c`` give the position (0..3) inside its group of value ``v`` of the
    16-wide K slice ``c`` (the smfmac index format, see ``tilelang.utils.sparse.compress``).
    ``B``: ``[K, N]`` or ``[N, K]`` (``transpose_B``).  K must be a multiple of 64; the
    accumulator is fp32."""
    if wg_wait not in (0, None):
        raise NotImplementedError("T.gemm_sp: wg_wait is a WGMMA (NVIDIA) feature")
    A, Er, B, C = to_region(A_sparse), to_region(E), to_region(B), to_region(C)
    op = O.GemmOp(A, B, C, transpose_A, transpose_B, int(policy), clear_accum, k_pack, wg_wait)
    op.E = Er
    return _emit(op)


gemm_sp_v2 = gemm_sp


_MX_FORMATS = {"e4m3": 0, "e5m2": 1, "e2m3": 2, "e3m2": 3, "e2m1": 4}


def _mx_format(region, fmt):
    dt = region.buffer.dtype
    if fmt is None:
        fmt = {"float8_e4m3fn": "e4m3", "float8_e5m2": "e5m2", "float4_e2m1fn_x2": "e2m1"}.get(dt.name)
        if fmt is None:
            raise ValueError(f"T.gemm_scaled: cannot infer the MX element format of a {dt} operand; pass "
                             f"a_format/b_format (one of {sorted(_MX_FORMATS)})")
    if fmt not in _MX_FORMATS:
        raise ValueError(f"T.gemm_scaled: unknown MX format {fmt!r} (one of {sorted(_MX_FORMATS)})")
    if dt.bits != 8:
        raise ValueError(f"T.gemm_scaled: MX operands are byte buffers (fp8, packed fp6 or packed fp4 pairs), "
                         f"got {dt}")
    return fmt


def gemm_scaled(A, B, C, scale_A, scale_B, transpose_A=False, transpose_B=True, policy=GemmWarpPolicy.Square,
                clear_accum=False, a_format=None, b_format=None, scale_layout="rows"):
    """Block-scaled MX GEMM: ``C (+)= (A * 2^(scale_A-127)) @ (B * 2^(scale_B-127))^T``.

    gfx950 ``v_mfma_scale_f32_16x16x128_f8f6f4``: the hardware applies one e8m0 scale per
    32 consecutive K elements of every row.  ``A``: ``[M, K]`` fp8 (e4m3/e5m2) or ``[M, K/2]``
    packed fp4 pairs (``float4_e2m1fn_x2`` / uint8 with ``a_format="e2m1"``, low nibble =
    even element) or ``[M, 3K/4]`` packed fp6 (uint8 with ``a_format="e2m3"`` / ``"e3m2"``, four
    elements per three bytes, ``tilelang.quantize.pack_fp6``); ``B``: ``[N, K]`` likewise
    (``transpose_B=True``, both K-contiguous);
    ``scale_A``: ``[M, K/32]`` and ``scale_B``: ``[N, K/32]`` e8m0 bytes (shared or global).
    K must be a multiple of 128.

    ``scale_layout="preshuffled"``: the scale tiles are 1-D shared buffers of ``rows * K / 32``
    bytes in the order ``tilelang.quantize.preshuffle_mx_scales`` writes (four 16-row fragments'
    bytes per dword): one ds_read_b32 per four fragments instead of a byte read per fragment, the
    MFMA's op_sel picks the byte.  Needs warp tiles of 64 rows / columns."""
    A, B, C = to_region(A), to_region(B), to_region(C)
    fa, fb = _mx_format(A, a_format), _mx_format(B, b_format)
    if scale_layout not in ("rows", "preshuffled"):
        raise ValueError(f"T.gemm_scaled: scale_layout must be 'rows' or 'preshuffled', got {scale_layout!r}")
    if transpose_A or not transpose_B:
        raise ValueError("T.gemm_scaled needs K-contiguous operands: A [M, K] and B [N, K] (transpose_B=True)")
    op = O.GemmOp(A, B, C, transpose_A, transpose_B, int(policy), clear_accum, 1, 0, to_region(scale_A),
                  to_region(scale_B))
    op.a_fmt, op.b_fmt = fa, fb
    op.scale_ps = scale_layout == "preshuffled"
    return _emit(op)


def fill(buffer, value):
    r = to_region(buffer)
    return _emit(O.FillOp(r, convert(value)))


def clear(buffer):
    r = to_region(buffer)
    return fill(r, const(0, r.dtype))


def reduce(buffer, out, reduce_type: str, dim: int = -1, clear: bool = True):
    src, dst = to_region(buffer), to_region(out)
    nd = len(src.region)
    if dim < 0:
        dim += nd
    if not (0 <= dim < nd):
        raise ValueError(f"reduce dim {dim} out of range for a {nd}-d tile")
    return _emit(O.ReduceOp(src, dst, reduce_type, dim, clear))


def reduce_max(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "max", dim, clear)


def reduce_min(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "min", dim, clear)


def reduce_sum(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "sum", dim, clear)


def reduce_abssum(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "abssum", dim, clear)


def reduce_absmax(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "absmax", dim, clear)


def reduce_bitand(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "bitand", dim, clear)


def reduce_bitor(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "bitor", dim, clear)


def reduce_bitxor(buffer, out, dim: int = -1, clear: bool = True):
    return reduce(buffer, out, "bitxor", dim, clear)


def cumsum(src, dst=None, dim: int = 0, reverse: bool = False):
    s = to_region(src)
    d = to_region(dst) if dst is not None else s
    nd = len(s.region)
    if dim < 0:
        dim += nd
    return _emit(O.CumSumOp(s, d, dim, reverse))


def finalize_reducer(reducer):
    return _emit(O.FinalizeReducerOp(to_region(reducer)))


# ---- warp (wave64) reductions on scalars ------------------------------------------------


def _wave_reduce(kind, value):
    value = convert(value)
    return call(f"tl.wave_reduce_{kind}", [value], value.dtype)


def warp_reduce_sum(value):
    return _wave_reduce("sum", value)


def warp_reduce_max(value):
    return _wave_reduce("max", value)


def warp_reduce_min(value):
    return _wave_reduce("min", value)


def warp_reduce_bitand(value):
    return _wave_reduce("bitand", value)


def warp_reduce_bitor(value):
    return _wave_reduce("bitor", value)


# ---- atomics ------------------------------------------------------------------------------


def _atomic(op, dst, value, memory_order=None, return_prev=False):
    _check_order(memory_order)
    if isinstance(dst, BufferLoad) and isinstance(value, (Buffer, BufferRegion)):
        # tile form with a point destination: T.atomic_add(C[by * bm, bx * bn], C_local)
        dst = to_region(dst, _extents_of(value))
    if isinstance(dst, BufferLoad):
        # scalar atomic on one element
        e = call(f"tl.atomic_{op}", [dst, convert(value)], dst.dtype, memory_order=memory_order,
                 return_prev=return_prev)
        if return_prev:
            return e
        current_builder().emit(S.EvaluateStmt(e))
        return None
    d = to_region(dst)
    if isinstance(value, (Buffer, BufferRegion, BufferLoad)):
        src = to_region(value, d.extents)
    else:
        src = convert(value)
    return _emit(O.AtomicOp(op, d, src, return_prev, memory_order))


def atomic_add(dst, value, memory_order=None, return_prev=False, use_tma=False):
    return _atomic("add", dst, value, memory_order, return_prev)


def atomic_max(dst, value, memory_order=None, return_prev=False):
    return _atomic("max", dst, value, memory_order, return_prev)


def atomic_min(dst, value, memory_order=None, return_prev=False):
    return _atomic("min", dst, value, memory_order, return_prev)


_MEMORY_ORDERS = ("relaxed", "consume", "acquire", "release", "acq_rel", "seq_cst")


def _check_order(memory_order):
    if memory_order is not None and memory_order not in _MEMORY_ORDERS:
        raise KeyError(f"unknown memory_order {memory_order!r}; one of {_MEMORY_ORDERS}")
    return memory_order


def _point(x):
    """The first element of a point load / region / buffer, as a BufferLoad."""
    if isinstance(x, BufferLoad):
        return x
    if isinstance(x, BufferRegion):
        return BufferLoad(x.buffer, list(x.mins))
    if isinstance(x, Buffer):
        return BufferLoad(x, [const(0, "int32")] * x.ndim)
    return None


def _atomic_vec(n, dst, value, return_prev, memory_order):
    """``AtomicAddx2`` / ``AtomicAddx4`` (reference ``tilelang/language/atomic.py:221-296``): add
    ``n`` consecutive elements of ``value`` to ``n`` consecutive elements of ``dst`` starting at
    the given (naturally aligned) element.  f16 / bf16 pairs are one packed atomic
    (``global_atomic_pk_add_{f16,bf16}``, ``ds_pk_add_*`` on LDS); f32 is ``n`` scalar adds.
    With ``return_prev`` the previous value of the first element is returned."""
    d = _point(dst)
    v = _point(value)
    if d is None or v is None:
        raise TypeError(f"T.atomic_addx{n}: dst and value must be buffer elements (a load, region or buffer)")
    vals = []
    for k in range(n):
        idx = list(v.indices)
        idx[-1] = idx[-1] + k if k else idx[-1]
        vals.append(BufferLoad(v.buffer, idx))
    e = call(f"tl.atomic_addx{n}", [d] + vals, d.dtype, memory_order=_check_order(memory_order),
             return_prev=return_prev)
    if return_prev:
        return e
    current_builder().emit(S.EvaluateStmt(e))
    return None


def atomic_addx2(dst, value, return_prev=False, memory_order=None):
    return _atomic_vec(2, dst, value, return_prev, memory_order)


def atomic_addx4(dst, value, return_prev=False, memory_order=None):
    return _atomic_vec(4, dst, value, return_prev, memory_order)


def atomic_load(src, memory_order="seq_cst"):
    src = _point(src)
    return call("tl.atomic_load", [src], src.dtype, memory_order=_check_order(memory_order))


def atomic_store(dst, value, memory_order="seq_cst"):
    dst = _point(dst)
    current_builder().emit(S.EvaluateStmt(call("tl.atomic_store", [dst, convert(value)], dst.dtype,
                                               memory_order=_check_order(memory_order))))


# ---- views --------------------------------------------------------------------------------


def reshape(src: Buffer, shape):
    """A view of ``src`` with a new row-major shape (same storage)."""
    b = Buffer(src.name + "_view", list(shape), src.dtype, src.scope)
    b.alias_of = (src, 0)
    b._auto_name = False
    return b


def view(src: Buffer, shape=None, dtype=None):
    """A view of ``src`` with a new shape and/or dtype (same bytes, reference ``T.view``)."""
    from ..ir import dtypes as _dt
    shape = list(shape) if shape is not None else list(src.shape)
    ndt = _dt.as_dtype(dtype) if dtype is not None else src.dtype
    n_old, n_new = src.static_numel(), 1
    for d in shape:
        n_new = None if n_new is None or as_int(d) is None else n_new * as_int(d)
    if n_old is not None and n_new is not None:
        assert n_old * src.dtype.bits == n_new * ndt.bits, (
            f"T.view({src.name}): {n_old} x {src.dtype.name} cannot be viewed as {shape} x {ndt.name}")
    b = Buffer(src.name + "_view", shape, ndt, src.scope)
    b.alias_of = (src, 0)
    return b
