"""Hand-scheduled matrix-core programming (reference: tilelang/intrinsics)."""
from .mfma_macro_generator import (MatrixCoreIntrinEmitter, MatrixCorePreshuffleIntrinEmitter,  # noqa: F401
                                   TensorCoreIntrinEmitter, shuffle_weight)
from . import mfma_layout  # noqa: F401


def get_swizzle_layout(row, col, row_size, dtype):
    """XOR swizzle of 16-byte chunks inside a row (reference helper used with T.Layout)."""
    from ..ir import dtypes as _dt
    bits = _dt.as_dtype(dtype).bits
    per = 128 // bits                      # elements per 16 bytes
    chunks = row_size // per
    if chunks <= 1:
        return row, col
    chunk = (col // per) ^ (row % chunks)
    return row, chunk * per + col % per


def make_mfma_swizzle_layout(shared_buf, *args, **kwargs):
    """XOR-swizzled LDS layout for an MFMA operand tile (reference
    ``tilelang.intrinsics.make_mfma_swizzle_layout``): the same 16-byte-chunk swizzle ``T.gemm``
    picks, so the emitter's 16-byte fragment runs are bank-conflict-free and the tile still
    loads by LDS-DMA."""
    from ..layout.layout import make_swizzled_layout
    return make_swizzled_layout(shared_buf)
