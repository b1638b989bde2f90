"""User-level MFMA emitter (reference: tilelang/intrinsics/mfma_macro_generator.py,
``MatrixCoreIntrinEmitter``; example examples/gemm/example_gemm_intrinsics.py).

For programs that schedule the matrix cores by hand instead of through ``T.gemm``: the emitter
writes per-thread register tiles (``T.alloc_local``) from LDS (``ldmatrix_a/b``), issues one
``v_mfma_*_16x16x*`` per (warp-row, warp-col) tile pair (``mma``) and scatters the accumulators
(``stmatrix``).  The block is ``block_row_warps x block_col_warps`` wave64s, each owning a
``warp_row_tiles x warp_col_tiles`` C sub-tile; ``chunk`` is the K extent of one LDS stage.

    emitter = MatrixCoreIntrinEmitter("float16", "float16", "float32", block_row_warps=2, ...)
    A_local = T.alloc_local((emitter.warp_rows * emitter.local_size_a,), "float16")
    ...
    for ki in T.serial(chunk // emitter.micro_size_k):
        emitter.ldmatrix_a(A_local, A_shared, ki)
        emitter.ldmatrix_b(B_local, B_shared, ki)
        emitter.mma(A_local, B_local, C_local)
    emitter.stmatrix(C_local, C_shared)     # or (C_local, C, pid_m=by, pid_n=bx) straight to global

Lane maps: ``mfma_layout``.  The MFMA itself is ``tl::mfma_16x16`` (include/tl/gemm.h): the
per-lane fragments are contiguous 16-byte runs of the register arrays, so clang keeps them in
VGPRs.  GPU-only (the CPU target runs one thread per block).
"""
from __future__ import annotations

from .. import language as T
from ..ir.expr import IntImm
from . import mfma_layout as ML

WAVE = 64


class MatrixCoreIntrinEmitter:
    micro_size_x = 16
    micro_size_y = 16

    def __init__(self, a_dtype="float16", b_dtype="float16", accum_dtype="float32", a_transposed=False,
                 b_transposed=True, block_row_warps=2, block_col_warps=2, warp_row_tiles=64, warp_col_tiles=64,
                 chunk=32, k_pack=1, thread_var=None):
        if a_dtype != b_dtype:
            raise ValueError("MatrixCoreIntrinEmitter: A and B need the same dtype")
        if a_dtype not in ("float16", "bfloat16", "int8"):
            raise NotImplementedError(f"MFMA emitter: unsupported input dtype {a_dtype} (f16, bf16, int8)")
        self.a_dtype, self.b_dtype, self.accum_dtype = a_dtype, b_dtype, accum_dtype
        self.a_transposed, self.b_transposed = a_transposed, b_transposed
        self.block_row_warps, self.block_col_warps = block_row_warps, block_col_warps
        self.warp_row_tiles, self.warp_col_tiles = warp_row_tiles, warp_col_tiles
        self.chunk = chunk
        self.k_per = ML.k_per_lane(a_dtype)
        self.micro_size_k = 4 * self.k_per  # 32 (16-bit) / 64 (int8)
        if warp_row_tiles % 16 or warp_col_tiles % 16 or chunk % self.micro_size_k:
            raise ValueError(f"MFMA emitter: warp tiles must be multiples of 16 and chunk of {self.micro_size_k}")
        self.warp_rows = warp_row_tiles // 16
        self.warp_cols = warp_col_tiles // 16
        self.local_size_a = self.k_per
        self.local_size_b = self.k_per
        self.local_size_out = 4
        self.threads = WAVE * block_row_warps * block_col_warps
        self.thread_var = thread_var

    # -- thread geometry -------------------------------------------------------------------
    def _tx(self):
        return self.thread_var if self.thread_var is not None else T.get_thread_binding(0)

    def _lane_warp(self):
        tx = self._tx()
        lane = tx % WAVE
        warp = tx // WAVE
        return lane, warp // self.block_col_warps, warp % self.block_col_warps

    # -- operand loads ---------------------------------------------------------------------
    def ldmatrix_a(self, A_local, A_shared, ki, rk=0):
        """A_local[i * k_per + j] <- A tile of warp-row i, K step ki (A_shared [M, K] or [K, M])."""
        lane, wm, _ = self._lane_warp()
        for i in range(self.warp_rows):
            for j in range(self.k_per):
                r, k = ML.a_coord(lane, j, self.k_per)
                row = wm * self.warp_row_tiles + i * 16 + r
                col = rk * self.chunk + ki * self.micro_size_k + k
                if self.a_transposed:
                    A_local[i * self.k_per + j] = A_shared[col, row]
                else:
                    A_local[i * self.k_per + j] = A_shared[row, col]

    def ldmatrix_b(self, B_local, B_shared, ki, rk=0):
        """B_local[i * k_per + j] <- B tile of warp-col i (B_shared [N, K] if b_transposed else [K, N])."""
        lane, _, wn = self._lane_warp()
        for i in range(self.warp_cols):
            for j in range(self.k_per):
                k, c = ML.b_coord(lane, j, self.k_per)
                n = wn * self.warp_col_tiles + i * 16 + c
                kk = rk * self.chunk + ki * self.micro_size_k + k
                if self.b_transposed:
                    B_local[i * self.k_per + j] = B_shared[n, kk]
                else:
                    B_local[i * self.k_per + j] = B_shared[kk, n]

    # -- matrix cores ----------------------------------------------------------------------
    def mma(self, A_local, B_local, C_local, k_inner=0):
        """C_local[(i * warp_cols + j) * 4 : +4] += A(i) B(j) for every warp tile pair."""
        for i in range(self.warp_rows):
            for j in range(self.warp_cols):
                T.evaluate(T.call_extern("handle", "tl::mfma_16x16",
                                         T.address_of(C_local[(i * self.warp_cols + j) * 4]),
                                         T.address_of(A_local[i * self.k_per]),
                                         T.address_of(B_local[j * self.k_per])))

    # -- accumulator stores ------------------------------------------------------------------
    def stmatrix(self, C_local, C_buf, pid_m=None, pid_n=None):
        """Scatter the accumulators.  ``C_buf`` 4-D [M/16, N/16, 16, 16] (shared, reference layout)
        or 2-D [M, N] (with ``pid_m`` / ``pid_n``: the block's tile offsets in a global C)."""
        lane, wm, wn = self._lane_warp()
        for i in range(self.warp_rows):
            for j in range(self.warp_cols):
                for v in range(4):
                    r, c = ML.c_coord(lane, v)
                    val = C_local[(i * self.warp_cols + j) * 4 + v]
                    if len(C_buf.shape) == 4:
                        C_buf[wm * self.warp_rows + i, wn * self.warp_cols + j, r, c] = val
                    else:
                        row = wm * self.warp_row_tiles + i * 16 + r
                        col = wn * self.warp_col_tiles + j * 16 + c
                        if pid_m is not None:
                            row = row + pid_m * self.block_row_warps * self.warp_row_tiles
                        if pid_n is not None:
                            col = col + pid_n * self.block_col_warps * self.warp_col_tiles
                        C_buf[row, col] = val


# the reference exports this name for its CUDA tensor-core emitter; on gfx950 it is the MFMA one
TensorCoreIntrinEmitter = MatrixCoreIntrinEmitter
