"""``T.gemm`` planning and lowering for gfx950 MFMA.

Reference: ``src/op/gemm.cc`` (instruction choice ``:129-141``, warp partition
``:144-354``, CDNA ``tl::gemm_ss/rs`` template call ``:437-592``) and the Python
``GemmMFMA`` lowering (``tilelang/tileop/gemm/gemm_mfma.py:62-233``).

The plan fixes: MFMA shape (16x16x32 for f16/bf16), warp partition, the
accumulator fragment (swapped-operand CDNA4 C layout), the LDS swizzle of each
shared operand (searched against the gfx950 bank model for the exact read
instruction: ``ds_read_b128`` for K-contiguous, ``ds_read_b64_tr_b16`` for
MN-contiguous operands) and whether a register A operand uses the k-permuted
order of an accumulator (``kperm``).
"""
from __future__ import annotations

from typing import Dict, Optional

from ..ir import tileop as O
from ..layout import mfma as MF
from ..layout.fragment import make_linear_fragment, Fragment
from ..layout.layout import LinearLayout, SwizzleLayout

compute_warp_partition = MF.compute_warp_partition


def _trailing2(region):
    ext = region.static_extents()
    if ext is None:
        raise ValueError("T.gemm operands need static tile shapes")
    # drop leading unit dims (e.g. a pipeline stage index)
    while len(ext) > 2 and ext[0] == 1:
        ext = ext[1:]
    if len(ext) != 2:
        raise ValueError(f"T.gemm operand must be 2-D, got extents {region.static_extents()}")
    return ext


def encode_swizzle(layout) -> int:
    if not isinstance(layout, SwizzleLayout):
        return 0
    v = 0
    for rb, cb in layout.bits:
        v |= (rb + 1) << (4 * cb)
    return v


MX_CODES = {"e4m3": 0, "e5m2": 1, "e2m3": 2, "e3m2": 3, "e2m1": 4}


_FP6 = ("e2m3", "e3m2")
# LDS read pattern of each operand format (layout/mfma.py _read_patterns)
_MX_KIND = {"e2m1": "k_rows16", "e2m3": "k_rows24mx", "e3m2": "k_rows24mx"}


def _mx_k(cols: int, fmt: str, name: str) -> int:
    """K elements in a row of ``cols`` bytes: fp8 1 per byte, fp4 2, fp6 4 per 3 bytes."""
    if fmt == "e2m1":
        return cols * 2
    if fmt in ("e2m3", "e3m2"):
        if cols % 3:
            raise ValueError(f"T.gemm_scaled: packed fp6 operand {name} has {cols} bytes per row, not a multiple of 3")
        return cols * 4 // 3
    return cols


def _mx_plan(op: O.GemmOp, plan: Dict, num_threads: int, a_ext, b_ext, is_cpu: bool = False) -> Dict:
    """Block-scaled MX GEMM (v_mfma_scale_f32_16x16x128_f8f6f4): both operands K-contiguous in LDS,
    one e8m0 scale per 32 K of every row of A and of B."""
    A, B = op.A.buffer, op.B.buffer
    M, N = plan["M"], plan["N"]
    ka, kb = _mx_k(a_ext[1], op.a_fmt, "A"), _mx_k(b_ext[1], op.b_fmt, "B")
    if ka != kb:
        raise ValueError(f"T.gemm_scaled: A holds K={ka} and B holds K={kb} elements")
    K = ka
    if K % 128:
        raise ValueError(f"T.gemm_scaled: K={K} must be a multiple of 128 (one scaled MFMA step)")
    if A.scope != "shared" or B.scope != "shared":
        raise ValueError("T.gemm_scaled: A and B must be shared-memory tiles")
    sa, sb = _trailing2(op.scale_A), _trailing2(op.scale_B)
    if getattr(op, "scale_ps", False):  # pre-shuffled tiles: [rows * K/32 / 64, 64] bytes
        if tuple(sa) != (M * K // 2048, 64) or tuple(sb) != (N * K // 2048, 64):
            raise ValueError(f"T.gemm_scaled(scale_layout='preshuffled'): scale tiles must be "
                             f"[{M * K // 2048}, 64] and [{N * K // 2048}, 64], got {sa} and {sb}")
    elif tuple(sa) != (M, K // 32) or tuple(sb) != (N, K // 32):
        raise ValueError(f"T.gemm_scaled: scales must be [M, K/32]=[{M}, {K // 32}] and [N, K/32]=[{N}, {K // 32}], "
                         f"got {sa} and {sb}")
    for r in (op.scale_A, op.scale_B):
        if r.buffer.dtype.bits != 8 or r.buffer.scope not in ("shared", "global"):
            raise ValueError("T.gemm_scaled: scales are e8m0 bytes in shared or global memory")
    plan.update(a_code=MX_CODES[op.a_fmt], b_code=MX_CODES[op.b_fmt], K=K)
    if is_cpu:
        plan.update(warp_m=1, warp_n=1, mfma=None, mx=True,
                    c_layout=make_linear_fragment([M, N], num_threads, 1, "cpu_c"),
                    a_smem_layout=LinearLayout(A.static_shape()), b_smem_layout=LinearLayout(B.static_shape()))
        return plan
    if num_threads % 64:
        raise ValueError(f"block size {num_threads} is not a multiple of the 64-lane wavefront")
    warp_m, warp_n = MF.compute_warp_partition(M, N, num_threads // 64, op.policy)
    plan.update(K=K, warp_m=warp_m, warp_n=warp_n, mfma=(16, 16, 128), mx=True,
                a_code=MX_CODES[op.a_fmt], b_code=MX_CODES[op.b_fmt])
    plan["c_layout"] = MF.mfma_c_fragment(M, N, warp_m, warp_n)
    ka_kind, kb_kind = _MX_KIND.get(op.a_fmt, "k_rows32mx"), _MX_KIND.get(op.b_fmt, "k_rows32mx")
    plan["a_kind"], plan["b_kind"] = ka_kind, kb_kind
    plan["a_smem_layout"] = MF.operand_swizzle(ka_kind, A.static_shape(), 1)
    plan["b_smem_layout"] = MF.operand_swizzle(kb_kind, B.static_shape(), 1)
    return plan


def _mfma_shape(op, target) -> str:
    """'16x16' (default) or '32x32': ``T.gemm(..., mfma_shape=)`` > ``tl.mfma_shape`` pass config."""
    sh = getattr(op, "mfma_shape", None) or getattr(target, "mfma_shape", None) or "16x16"
    if sh not in ("16x16", "32x32"):
        raise ValueError(f"mfma_shape must be '16x16' or '32x32', got {sh!r}")
    return sh


def _try_32x32(op: O.GemmOp, plan: Dict, nw: int, num_threads: int = 0, a_layout: Optional[Fragment] = None):
    """v_mfma_f32_32x32x16_{f16,bf16} plan, or None when the tile does not fit.

    A in LDS (``tl::gemm_ss_32``) or in registers (``tl::gemm_rs_32``): a register A operand that
    came from a 32x32 accumulator keeps its k order (``kperm=1``, layout.mfma._mfma_a_fragment32)
    and the B tile is then read in that order (``tr32_kperm``)."""
    M, N, K = plan["M"], plan["N"], plan["K"]
    A, B = op.A.buffer, op.B.buffer
    if K % 16:
        return None
    try:
        warp_m, warp_n = MF.compute_warp_partition(M, N, nw, op.policy, 32, 32)
    except ValueError:
        return None
    plan.update(warp_m=warp_m, warp_n=warp_n, mfma=(32, 32, 16))
    plan["c_layout"] = MF.mfma_c_fragment(M, N, warp_m, warp_n, (32, 32))
    if A.scope == "fragment":
        if a_layout is not None:
            k1 = MF.mfma_a_fragment(M, K, warp_m, warp_n, 1, (32, 32), op.trans_A)
            k1r = k1 if k1.num_threads == num_threads else k1.replicate(num_threads // k1.num_threads)
            if a_layout.is_equal(k1r) or a_layout.is_equal(k1):
                plan["a_kperm"] = 1
    else:
        plan["a_kind"] = "tr32" if op.trans_A else "k_rows_32"
        plan["a_smem_layout"] = MF.operand_swizzle(plan["a_kind"], A.static_shape(), 2)
    plan["b_kind"] = "k_rows_32" if op.trans_B else ("tr32_kperm" if plan["a_kperm"] else "tr32")
    plan["b_smem_layout"] = MF.operand_swizzle(plan["b_kind"], B.static_shape(), 2)
    return plan


def _int8_plan(op: O.GemmOp, plan: Dict, nw: int, target) -> Dict:
    """int8 x int8 -> int32: v_mfma_i32_16x16x64_i8 / v_mfma_i32_32x32x32_i8, K-contiguous operands."""
    M, N, K = plan["M"], plan["N"], plan["K"]
    A, B, C = op.A.buffer, op.B.buffer, op.C.buffer
    if op.trans_A or not op.trans_B or A.scope != "shared" or B.scope != "shared":
        raise ValueError("int8 T.gemm on gfx950 needs K-contiguous shared operands: A [M,K] and B [N,K] "
                         "(transpose_B=True)")
    if C.dtype.name != "int32":
        raise ValueError(f"int8 T.gemm accumulates in int32, got a {C.dtype} accumulator")
    ms = 32 if _mfma_shape(op, target) == "32x32" else 16
    ks = 64 if ms == 16 else 32
    if K % ks:
        raise ValueError(f"int8 T.gemm: K={K} must be a multiple of {ks} (MFMA {ms}x{ms}x{ks})")
    warp_m, warp_n = MF.compute_warp_partition(M, N, nw, op.policy, ms, ms)
    plan.update(warp_m=warp_m, warp_n=warp_n, mfma=(ms, ms, ks), int8=True)
    plan["c_layout"] = MF.mfma_c_fragment(M, N, warp_m, warp_n, (ms, ms))
    kind = "k_rows16" if ms == 16 else "k_rows_i8_32"
    plan["a_kind"] = plan["b_kind"] = kind
    plan["a_smem_layout"] = MF.operand_swizzle(kind, A.static_shape(), 1)
    plan["b_smem_layout"] = MF.operand_swizzle(kind, B.static_shape(), 1)
    return plan


def _f32_plan(op: O.GemmOp, plan: Dict, nw: int) -> Dict:
    """fp32 x fp32 -> fp32 on v_mfma_f32_16x16x4_f32 (exact f32 products, the f32 VALU rate)."""
    M, N, K = plan["M"], plan["N"], plan["K"]
    A, B = op.A.buffer, op.B.buffer
    if A.scope != "shared" or B.scope != "shared":
        raise ValueError("fp32 T.gemm on gfx950 needs shared-memory operands")
    if K % 4:
        raise ValueError(f"fp32 T.gemm: K={K} must be a multiple of 4 (MFMA 16x16x4)")
    warp_m, warp_n = MF.compute_warp_partition(M, N, nw, op.policy)
    plan.update(warp_m=warp_m, warp_n=warp_n, mfma=(16, 16, 4), f32=True)
    plan["c_layout"] = MF.mfma_c_fragment(M, N, warp_m, warp_n)
    plan["a_kind"] = plan["b_kind"] = "f32"
    plan["a_smem_layout"] = LinearLayout(A.static_shape())
    plan["b_smem_layout"] = LinearLayout(B.static_shape())
    return plan


def _sp_plan(op: O.GemmOp, plan: Dict, num_threads: int, is_cpu: bool) -> Dict:
    """2:4 sparse A (``v_smfmac_f32_16x16x64_{f16,bf16}``).  Per 64-wide K step the lane
    (row/col ``l&15``, slice ``g=l>>4``) holds 8 kept A values of original K ``[16g, 16g+16)``
    (one 16-byte read of the compressed row at ``8g``), the 16-bit index field ``E[row][g]``, and
    the B values of K ``8g+j`` and ``32+8g+j`` — i.e. exactly two dense 16x16x32 B fragments
    (measured on gfx950: scripts/probes/smfmac_map.hip).  Issued as ``smfmac(A, B)``, so C is
    held in the direct (unswapped) MFMA layout."""
    A, B, C, E = op.A.buffer, op.B.buffer, op.C.buffer, op.E.buffer
    M, N, K = plan["M"], plan["N"], plan["K"]
    if A.dtype.name not in ("float16", "bfloat16") or B.dtype != A.dtype:
        raise ValueError(f"T.gemm_sp on gfx950 supports f16/bf16 operands (v_smfmac_f32_16x16x64), got "
                         f"{A.dtype} x {B.dtype}")
    if C.dtype.name != "float32":
        raise ValueError(f"T.gemm_sp accumulates in float32, got a {C.dtype} accumulator")
    if K % 64:
        raise ValueError(f"T.gemm_sp: K={K} must be a multiple of 64 (one v_smfmac_f32_16x16x64 step)")
    e_ext = _trailing2(op.E)
    if tuple(e_ext) != (M, K // 16) or E.dtype.bits != 16:
        raise ValueError(f"T.gemm_sp: metadata E must be a [M, K/16]=[{M}, {K // 16}] int16 tile, got "
                         f"{list(e_ext)} {E.dtype}")
    if A.scope != "shared" or B.scope != "shared" or E.scope not in ("shared", "global"):
        raise ValueError("T.gemm_sp: A_sparse and B must be shared-memory tiles, E shared or global")
    plan["sp"] = True
    if is_cpu:
        plan.update(warp_m=1, warp_n=1, mfma=None,
                    c_layout=make_linear_fragment([M, N], num_threads, 1, "cpu_c"),
                    a_smem_layout=LinearLayout(A.static_shape()), b_smem_layout=LinearLayout(B.static_shape()))
        return plan
    if num_threads % 64:
        raise ValueError(f"block size {num_threads} is not a multiple of the 64-lane wavefront")
    warp_m, warp_n = MF.compute_warp_partition(M, N, num_threads // 64, op.policy)
    plan.update(warp_m=warp_m, warp_n=warp_n, mfma=(16, 16, 64))
    plan["c_layout"] = MF.mfma_c_fragment_direct(M, N, warp_m, warp_n)
    plan["a_kind"] = "tr" if op.trans_A else "k_rows"
    plan["b_kind"] = "k_rows" if op.trans_B else "tr"
    plan["a_smem_layout"] = MF.operand_swizzle(plan["a_kind"], A.static_shape(), 2)
    plan["b_smem_layout"] = MF.operand_swizzle(plan["b_kind"], B.static_shape(), 2)
    return plan


def gemm_plan(op: O.GemmOp, num_threads: int, target=None, a_layout: Optional[Fragment] = None) -> Dict:
    a_ext, b_ext, c_ext = _trailing2(op.A), _trailing2(op.B), _trailing2(op.C)
    M, N = c_ext
    K = a_ext[0] if op.trans_A else a_ext[1]
    if op.is_sp:
        K *= 2  # A_sparse keeps 2 of every 4 K values
    kb = b_ext[1] if op.trans_B else b_ext[0]
    am = a_ext[1] if op.trans_A else a_ext[0]
    bn = b_ext[0] if op.trans_B else b_ext[1]
    if op.is_mx:
        kb = K  # packed fp4 rows hold 2 elements per byte: _mx_plan checks the logical K
    if kb != K or am != M or bn != N:
        raise ValueError(f"T.gemm shape mismatch: A{a_ext} B{b_ext} C{c_ext} "
                         f"(transpose_A={op.trans_A}, transpose_B={op.trans_B})")
    is_cpu = target is not None and getattr(target, "kind", "hip") == "cpu"
    A, B, C = op.A.buffer, op.B.buffer, op.C.buffer
    plan = dict(M=M, N=N, K=K, a_kperm=0)
    if op.is_sp:
        return _sp_plan(op, plan, num_threads, is_cpu)
    if is_cpu and not op.is_mx:
        plan.update(warp_m=1, warp_n=1, mfma=None, c_layout=make_linear_fragment([M, N], num_threads, 1, "cpu_c"),
                    a_smem_layout=LinearLayout(A.static_shape() or a_ext),
                    b_smem_layout=LinearLayout(B.static_shape() or b_ext))
        return plan
    if op.is_mx:
        return _mx_plan(op, plan, num_threads, a_ext, b_ext, is_cpu)
    eb = A.dtype.bits
    if A.dtype != B.dtype:
        raise ValueError(f"T.gemm needs matching A/B dtypes, got {A.dtype} and {B.dtype}")
    if num_threads % 64:
        raise ValueError(f"block size {num_threads} is not a multiple of the 64-lane wavefront")
    nw = num_threads // 64
    if A.dtype.name == "int8":
        return _int8_plan(op, plan, nw, target)
    if A.dtype.name == "float32":
        return _f32_plan(op, plan, nw)
    if eb not in (16, 8):
        raise ValueError(f"T.gemm on gfx950 supports f16/bf16, fp8, int8 and fp32 inputs, got {A.dtype}")
    shape = _mfma_shape(op, target)
    if eb == 16 and shape == "32x32" and A.scope in ("shared", "fragment") and B.scope == "shared":
        r = _try_32x32(op, plan, nw, num_threads, a_layout if A.scope == "fragment" else None)
        if r is not None:
            return r
        if getattr(op, "mfma_shape", None) == "32x32":
            raise ValueError(f"T.gemm(mfma_shape='32x32'): a {M}x{N} tile over {nw} waves needs per-wave tiles "
                             f"that are multiples of 32 and K % 16 == 0")
    rc = None
    if eb == 16 and A.scope == "shared" and B.scope == "shared" and getattr(op, "khalf", None) is not None:
        # only for the K-split GEMM main loop (transform/gemm_ksplit.py): other GEMMs that share
        # an accumulator fragment must keep one partition whatever their operand orientation
        rc = (2 if op.trans_A else 1, 1 if op.trans_B else 2)
    warp_m, warp_n = MF.compute_warp_partition(M, N, nw, op.policy, read_cost=rc)
    plan.update(warp_m=warp_m, warp_n=warp_n, mfma=(16, 16, 32))
    plan["c_layout"] = MF.mfma_c_fragment(M, N, warp_m, warp_n)
    if K % 32:
        raise ValueError(f"T.gemm K={K} must be a multiple of 32 on gfx950 (MFMA 16x16x32)")
    if a_layout is not None and A.scope == "fragment":
        k1 = MF.mfma_a_fragment(M, K, warp_m, warp_n, 1, trans=op.trans_A)
        k1r = k1 if k1.num_threads == num_threads else k1.replicate(num_threads // k1.num_threads)
        if a_layout.is_equal(k1r) or a_layout.is_equal(k1):
            plan["a_kperm"] = 1
    ebytes = A.dtype.bytes
    if eb == 8:
        if op.trans_A or A.scope != "shared" or B.scope != "shared":
            raise ValueError("fp8 T.gemm on gfx950 needs shared operands with A K-contiguous ([M,K]); B is "
                             "[N,K] (transpose_B=True) or [K,N] (ds_read_b64_tr_b8 transposed reads)")
        kind = "k_rows32" if K % 128 == 0 else "k_rows"
        plan["f8_kind"] = kind
        plan["a_kind"] = kind
        plan["b_kind"] = kind if op.trans_B else ("tr8_32" if K % 128 == 0 else "tr8")
        plan["a_smem_layout"] = MF.operand_swizzle(kind, A.static_shape(), 1)
        plan["b_smem_layout"] = MF.operand_swizzle(plan["b_kind"], B.static_shape(), 1)
        return plan
    if A.scope == "shared":
        shp = A.static_shape()
        kind = "tr" if op.trans_A else "k_rows"
        plan["a_kind"] = kind
        plan["a_smem_layout"] = MF.operand_swizzle(kind, shp, ebytes) if ebytes == 2 else LinearLayout(shp)
    if B.scope == "shared":
        shp = B.static_shape()
        if op.trans_B:
            kind = "k_rows"
        else:
            kind = "tr_kperm" if plan["a_kperm"] == 1 else "tr"
        plan["b_kind"] = kind
        plan["b_smem_layout"] = MF.operand_swizzle(kind, shp, ebytes) if ebytes == 2 else LinearLayout(shp)
    return plan
