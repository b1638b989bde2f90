"""Hand-scheduled matrix-core programming (reference: tilelang/intrinsics)."""
from .mfma_macro_generator import MatrixCoreIntrinEmitter, TensorCoreIntrinEmitter  # noqa: F401
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
