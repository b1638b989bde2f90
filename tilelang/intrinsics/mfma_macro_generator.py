"""User-level MFMA emitter (reference: tilelang/intrinsics/mfma_macro_generator.py,
``MatrixCoreIntrinEmitter`` / ``MatrixCorePreshuffleIntrinEmitter``; example
examples/gemm/example_gemm_intrinsics.py, tests testing/python/amd/test_tilelang_gemm_mfma_*.py).

For programs that schedule the matrix cores by hand instead of through ``T.gemm``: the emitter
writes per-thread register tiles (``T.alloc_local``) from LDS or global memory (``ldmatrix_a/b``),
issues one MFMA per (warp-row, warp-col, k_pack) triple (``mfma``) and scatters the accumulators
(``stmatrix``).  The block is ``block_row_warps x block_col_warps`` wave64s, each owning a
``warp_row_tiles x warp_col_tiles`` C sub-tile; ``chunk`` is the K extent of one LDS stage.

    emitter = MatrixCoreIntrinEmitter("float16", "float16", "float32", b_transposed=True, ...)
    A_local = T.alloc_local((emitter.warp_rows * emitter.local_size_a,), "float16")
    ...
    for ki in T.serial(chunk // (emitter.k_pack * emitter.micro_size_k)):
        emitter.ldmatrix_a(A_local, A_shared, ki)
        emitter.ldmatrix_b(B_local, B_shared, ki)
        emitter.mfma(A_local, B_local, C_local)
    emitter.stmatrix(C_local, C_shared)     # or (C_local, C, pid_m=by, pid_n=bx) straight to global

gfx950 instruction forms (``micro_size`` 16 or 32, include/tl/gemm.h ``tl::mfma_emit``):

    dtype                      16x16 tile          32x32 tile          k per lane (k_dim)
    float16 / bfloat16         16x16x32            32x32x16            8
    int8 (int32 accumulator)   16x16x64            32x32x32            16
    float8_e4m3fn / e5m2       16x16x128 (scaled)  32x32x64 (scaled)   32  (k_dim=128/64, default)
                               16x16x32            32x32x16            8   (fp8_k_dim=32 / 16)
    float32                    16x16x4             32x32x2             1

OCP fp8 is gfx950's native format: the reference's ``float8_e4m3fnuz`` (CDNA3) is refused rather
than silently reinterpreted.  The f8f6f4 forms run at twice the rate of the 8-k ones; their
in-lane k order is a fixed permutation applied to A and B alike, which leaves the contraction
unchanged.

Operand loads: a lane's fragment is ``local_size = k_per * k_pack`` consecutive k of one row, so
K-contiguous operands load as 16-byte runs (``tl::ld_run`` -> ``ds_read_b128`` /
``global_load_dwordx4``), one run per 16-byte swizzle chunk of an annotated LDS layout
(``make_mfma_swizzle_layout``).  MN-contiguous operands (``a_transposed`` / not ``b_transposed``)
gather element-wise.

``b_preshuffle`` (``a_preshuffle``): the operand is stored tile-major,
``[N / micro, K / (micro_k * k_pack), micro, micro_k * k_pack]`` (``b_transposed``) or
``[K / pk, N / micro, pk, micro]``, so one wave's fragment of one tile is a contiguous 1 KiB (16-bit)
block: ``ldmatrix_b(B_local, B, k_step, pid_m=, pid_n=)`` then loads it straight from global
memory with fully coalesced 16-byte lanes (the reference's ``b_g2l_load``), or from an LDS copy of
the same shape.  ``shuffle_weight`` produces the layout on the host.
"""
from __future__ import annotations

from .. import language as T
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import BufferLoad
from . import mfma_layout as ML

WAVE = 64

_CTYPE = {"float16": "half_t", "bfloat16": "bfloat16_t", "int8": "int8_t", "float8_e4m3fn": "fp8_e4_t",
          "float8_e4m3": "fp8_e4_t", "float8_e5m2": "fp8_e5_t", "float32": "float", "float": "float"}
_FP8 = ("float8_e4m3fn", "float8_e4m3", "float8_e5m2")


def _bytes(dtype: str) -> int:
    return 4 if dtype in ("float32", "float") else 1 if dtype in _FP8 + ("int8", ) else 2


class MatrixCoreIntrinEmitter:
    WARP_SIZE = WAVE
    # thread binding (tx, warp_n, warp_m) when True, as the reference's ``is_m_first``
    is_m_first = False

    def __init__(self, a_dtype="float16", b_dtype="float16", accum_dtype="float32", a_transposed=False,
                 b_transposed=False, block_row_warps=2, block_col_warps=2, warp_row_tiles=64, warp_col_tiles=64,
                 chunk=32, reduce_k=1, num_elems_per_byte=1, k_pack=None, is_m_first=False, b_preshuffle=False,
                 thread_var=None, micro_size=16, fp8_k_dim=None, a_preshuffle=False):
        for d in (a_dtype, b_dtype):
            if d == "float8_e4m3fnuz":
                raise NotImplementedError("gfx950 MFMA consumes OCP fp8: use float8_e4m3fn "
                                          "(e4m3fnuz is CDNA3's format)")
            if d not in _CTYPE:
                raise NotImplementedError(f"MFMA emitter: unsupported input dtype {d} "
                                          "(float16, bfloat16, int8, float8_e4m3fn, float8_e5m2, float32)")
        fp8 = a_dtype in _FP8
        if (a_dtype != b_dtype) and not (fp8 and b_dtype in _FP8):
            raise ValueError("MatrixCoreIntrinEmitter: A and B need the same dtype (fp8 formats may mix)")
        if micro_size not in (16, 32):
            raise ValueError("MFMA emitter: micro_size is 16 or 32")
        if reduce_k < 1:
            raise ValueError("MFMA emitter: reduce_k >= 1")
        if num_elems_per_byte != 1:
            raise NotImplementedError("MFMA emitter: packed sub-byte operands go through T.gemm / the MX path")
        int_acc = accum_dtype in ("int32", )
        if (a_dtype == "int8") != int_acc or accum_dtype not in ("float32", "float", "int32"):
            raise ValueError(f"MFMA emitter: accumulator {accum_dtype} does not match {a_dtype} "
                             "(float32 for float inputs, int32 for int8)")
        self.a_dtype, self.b_dtype, self.accum_dtype = a_dtype, b_dtype, accum_dtype
        self.a_transposed, self.b_transposed = a_transposed, b_transposed
        self.block_row_warps, self.block_col_warps = block_row_warps, block_col_warps
        self.warp_row_tiles, self.warp_col_tiles = warp_row_tiles, warp_col_tiles
        self.chunk = chunk
        self.reduce_k = reduce_k
        self.num_elems_per_byte = num_elems_per_byte
        self.k_pack = 1 if k_pack is None else int(k_pack)
        if is_m_first is not None:
            self.is_m_first = bool(is_m_first)
        self.a_preshuffle, self.b_preshuffle = bool(a_preshuffle), bool(b_preshuffle)
        self.micro_size_x = self.micro_size_y = self.M_DIM = self.N_DIM = micro_size
        groups = WAVE // micro_size  # lane groups along k: 4 (16x16) or 2 (32x32)
        if fp8:
            full = 128 if micro_size == 16 else 64
            kd = full if fp8_k_dim is None else int(fp8_k_dim)
            if kd not in (full, 8 * groups):
                raise ValueError(f"fp8 MFMA {micro_size}x{micro_size}: k_dim {full} (scaled form) or {8 * groups}")
            self.k_per = kd // groups
        elif a_dtype == "int8":
            self.k_per = 16
        elif a_dtype in ("float32", "float"):
            self.k_per = 1
        else:
            self.k_per = 8
        self.k_dim = self.micro_size_k = self.k_per * groups
        self.local_size_a = self.local_size_b = self.k_per * self.k_pack
        self.local_size_out = micro_size * micro_size // WAVE
        pk = self.micro_size_k * self.k_pack
        if warp_row_tiles % micro_size or warp_col_tiles % micro_size or chunk % pk:
            raise ValueError(f"MFMA emitter: warp tiles must be multiples of {micro_size} and chunk of {pk}")
        self.warp_rows = warp_row_tiles // micro_size
        self.warp_cols = warp_col_tiles // micro_size
        # reduce_k > 1: split-K inside the block.  The block is launched with threads
        # (WAVE * block_row_warps * block_col_warps, reduce_k); wave group rk (thread binding 1)
        # takes K slice [rk * chunk, (rk + 1) * chunk) of every stage (``ldmatrix_*(..., rk=rk)``)
        # and ``reduce_k_sum`` adds the groups' accumulators through LDS.
        self.threads = WAVE * block_row_warps * block_col_warps * reduce_k
        self.thread_var = thread_var

    # -- thread geometry -------------------------------------------------------------------
    def get_thread_binding(self):
        return self.thread_var if self.thread_var is not None else T.get_thread_binding(0)

    def extract_thread_binding(self, thread_id, is_m_first=None):
        """(lane, warp_n, warp_m) of ``thread_id``; ``is_m_first``: consecutive waves walk N."""
        m_first = self.is_m_first if is_m_first is None else is_m_first
        lane = thread_id % WAVE
        w = thread_id // WAVE
        if m_first:
            return lane, w % self.block_col_warps, (w // self.block_col_warps) % self.block_row_warps
        return lane, (w // self.block_row_warps) % self.block_col_warps, w % self.block_row_warps

    def _lane_warp(self):
        lane, wn, wm = self.extract_thread_binding(self._tx())
        return lane, wm, wn

    def _tx(self):
        return self.get_thread_binding()

    # -- operand loads ---------------------------------------------------------------------
    @staticmethod
    def _region(buf):
        """(buffer, base offsets of the last two dims) of a Buffer / BufferRegion / BufferLoad."""
        if isinstance(buf, Buffer):
            return buf, [0] * len(buf.shape)
        if isinstance(buf, BufferRegion):
            return buf.buffer, [m for m, _ in buf.region]
        if isinstance(buf, BufferLoad):
            return buf.buffer, list(buf.indices)
        raise TypeError(f"MFMA emitter: expected a buffer, got {type(buf).__name__}")

    def _load_run(self, local, lbase, buf, idx_of, n, dtype, contiguous):
        """local[lbase + t] <- buf[idx_of(t)] for t < n; contiguous: one ld_run per 16 bytes."""
        if contiguous:
            eb = _bytes(dtype)
            per = max(1, 16 // eb)
            for c in range(0, n, per):
                m = min(per, n - c)
                T.evaluate(T.call_extern("handle", f"tl::ld_run<{_CTYPE[dtype]}, {m}>", T.address_of(local[lbase + c]),
                                         T.address_of(buf[tuple(idx_of(c))])))
        else:
            for t in range(n):
                local[lbase + t] = buf[tuple(idx_of(t))]

    def _operand(self, local, src, ki, rk, is_b, pid_m, pid_n):
        lane, wm, wn = self._lane_warp()
        ms = self.micro_size_x
        L = self.local_size_a
        pk = self.micro_size_k * self.k_pack
        buf, base = self._region(src)
        trans = self.b_transposed if is_b else self.a_transposed
        mn_contig = (not trans) if is_b else trans  # [K][MN] storage
        dtype = self.b_dtype if is_b else self.a_dtype
        pre = self.b_preshuffle if is_b else self.a_preshuffle
        tiles = self.warp_cols if is_b else self.warp_rows
        wtile = self.warp_col_tiles if is_b else self.warp_row_tiles
        w = wn if is_b else wm
        g = lane // ms
        r = lane % ms
        lead = base[:-4] if pre else base[:-2]
        for i in range(tiles):
            mn0 = w * wtile + i * ms
            if pre:
                # tile-major operand: [MN/ms, K/pk, ms, pk] (K-contiguous) or [K/pk, MN/ms, pk, ms]
                kt = ki if pid_m is not None or pid_n is not None else rk * (self.chunk // pk) + ki
                glob = pid_n if is_b else pid_m
                bm = (self.block_col_warps * self.warp_col_tiles) if is_b else (self.block_row_warps *
                                                                                 self.warp_row_tiles)
                t_mn = (mn0 // ms) if glob is None else glob * (bm // ms) + mn0 // ms
                if not mn_contig:
                    def idx(t, t_mn=t_mn):
                        return lead + [base[-4] + t_mn, base[-3] + kt, base[-2] + r, base[-1] + L * g + t]
                else:
                    def idx(t, t_mn=t_mn):
                        return lead + [base[-4] + kt, base[-3] + t_mn, base[-2] + L * g + t, base[-1] + r]
                self._load_run(local, i * L, buf, idx, L, dtype, not mn_contig)
                continue
            k0 = rk * self.chunk + ki * pk + L * g
            if pid_m is not None or pid_n is not None:
                glob = pid_n if is_b else pid_m
                bm = (self.block_col_warps * self.warp_col_tiles) if is_b else (self.block_row_warps *
                                                                                 self.warp_row_tiles)
                row = glob * bm + mn0 + r
            else:
                row = mn0 + r
            if not mn_contig:
                def idx(t, row=row):
                    return lead + [base[-2] + row, base[-1] + k0 + t]
            else:
                def idx(t, row=row):
                    return lead + [base[-2] + k0 + t, base[-1] + row]
            self._load_run(local, i * L, buf, idx, L, dtype, not mn_contig)

    def ldmatrix_a(self, A_local, A_buf, ki, rk=0, pid_m=None, pid_n=None):
        """A_local[i * local_size_a + t] <- A tile of warp-row i, K step ki.  A_buf: [M, K] / [K, M]
        LDS tile, a global tensor (``pid_m``: block row, ``ki``: global K step), or the tile-major
        preshuffled layout (``a_preshuffle``)."""
        self._operand(A_local, A_buf, ki, rk, False, pid_m, pid_n)

    def ldmatrix_b(self, B_local, B_buf, ki, rk=0, pid_m=None, pid_n=None):
        """B_local[j * local_size_b + t] <- B tile of warp-col j (B_buf [N, K] if b_transposed else
        [K, N]; preshuffled tile-major with ``b_preshuffle``; global with ``pid_n``)."""
        self._operand(B_local, B_buf, ki, rk, True, pid_m, pid_n)

    # -- matrix cores ----------------------------------------------------------------------
    def mfma(self, A_local, B_local, C_local, k_inner=0):
        """C_local[(i * warp_cols + j) * local_size_out :] += A(i) B(j), every k_pack slice."""
        ms, kp = self.micro_size_x, self.k_per
        name = f"tl::mfma_emit<{ms}, {kp}>"
        lo = self.local_size_out
        for p in range(self.k_pack):
            for i in range(self.warp_rows):
                for j in range(self.warp_cols):
                    T.evaluate(T.call_extern("handle", name, T.address_of(C_local[(i * self.warp_cols + j) * lo]),
                                             T.address_of(A_local[i * self.local_size_a + p * kp]),
                                             T.address_of(B_local[j * self.local_size_b + p * kp])))

    mma = mfma

    # -- split-K inside the block ------------------------------------------------------------
    def reduce_k_scratch_shape(self):
        """Shape of the LDS scratch ``reduce_k_sum`` needs: [reduce_k, acc, threads per group]
        (thread-minor: a wave's 64 lanes store 64 consecutive dwords, no bank conflicts)."""
        return (self.reduce_k, self.warp_rows * self.warp_cols * self.local_size_out,
                WAVE * self.block_row_warps * self.block_col_warps)

    def reduce_k_sum(self, C_local, scratch, rk=None):
        """Sum the ``reduce_k`` wave groups' partial accumulators (reference: the ``reduce_k``
        split of ``mfma_macro_generator.py:74``, summed in examples/dequantize_gemm/
        example_dequant_gemm_fine_grained.py:316-335): every group stores its accumulators into
        ``scratch`` (``reduce_k_scratch_shape()``, accum dtype, LDS), then every group reads the
        total back into ``C_local`` (the barrier between the two is placed by ThreadSync)."""
        if self.reduce_k == 1:
            return
        tx = self._tx()
        rk = T.get_thread_binding(1) if rk is None else rk
        n = self.warp_rows * self.warp_cols * self.local_size_out
        for v in range(n):
            scratch[rk, v, tx] = C_local[v]
        for v in range(n):
            acc = scratch[0, v, tx]
            for r in range(1, self.reduce_k):
                acc = acc + scratch[r, v, tx]
            C_local[v] = acc

    # -- accumulator stores ------------------------------------------------------------------
    def _c_coord(self, lane, v):
        if self.micro_size_x == 16:
            return ML.c_coord(lane, v)
        return 8 * (v // 4) + 4 * (lane // 32) + v % 4, lane % 32

    def stmatrix(self, C_local, C_buf, pid_m=None, pid_n=None):
        """Scatter the accumulators.  ``C_buf`` 4-D [M/ms, N/ms, ms, ms] (shared, reference layout)
        or 2-D [M, N] (with ``pid_m`` / ``pid_n``: the block's tile offsets in a global C)."""
        lane, wm, wn = self._lane_warp()
        ms = self.micro_size_x
        for i in range(self.warp_rows):
            for j in range(self.warp_cols):
                for v in range(self.local_size_out):
                    r, c = self._c_coord(lane, v)
                    val = C_local[(i * self.warp_cols + j) * self.local_size_out + v]
                    if len(C_buf.shape) == 4:
                        C_buf[wm * self.warp_rows + i, wn * self.warp_cols + j, r, c] = val
                    else:
                        row = wm * self.warp_row_tiles + i * ms + r
                        col = wn * self.warp_col_tiles + j * ms + c
                        if pid_m is not None:
                            row = row + pid_m * self.block_row_warps * self.warp_row_tiles
                        if pid_n is not None:
                            col = col + pid_n * self.block_col_warps * self.warp_col_tiles
                        C_buf[row, col] = val


class MatrixCorePreshuffleIntrinEmitter(MatrixCoreIntrinEmitter):
    """The reference's preshuffle emitter: same as the base with ``a_preshuffle`` / ``b_preshuffle``
    (tile-major operands, loadable straight from global memory)."""

    def __init__(self, *args, a_preshuffle=False, b_preshuffle=False, **kw):
        super().__init__(*args, a_preshuffle=a_preshuffle, b_preshuffle=b_preshuffle, **kw)


def shuffle_weight(x, layout=(16, 32), k_pack=1, is_transpose=False):
    """Host-side tile-major relayout for ``b_preshuffle``: ``layout = (micro, micro_k)``;
    [N, K] (``is_transpose``) -> [N/micro, K/pk, micro, pk], [K, N] -> [K/pk, N/micro, pk, micro]."""
    IN, IK = layout
    BK = IK * k_pack
    if is_transpose:
        N, K = x.shape[-2], x.shape[-1]
        assert N % IN == 0 and K % BK == 0
        return x.view(N // IN, IN, K // BK, BK).permute(0, 2, 1, 3).contiguous()
    K, N = x.shape[-2], x.shape[-1]
    assert N % IN == 0 and K % BK == 0
    return x.view(K // BK, BK, N // IN, IN).permute(0, 2, 1, 3).contiguous()


# the reference exports this name for its CUDA tensor-core emitter; on gfx950 it is the MFMA one
TensorCoreIntrinEmitter = MatrixCoreIntrinEmitter
