"""Layouts: memory index maps, LDS swizzles, fragment (thread/register) layouts."""
from .layout import (Layout, LinearLayout, SwizzleLayout, PaddedLayout, make_linear_layout, make_swizzled_layout,
                     make_full_bank_swizzled_layout, make_half_bank_swizzled_layout,
                     make_quarter_bank_swizzled_layout, physical_size)
from .fragment import Fragment as _DigitFragment, Digit, make_linear_fragment, make_replicated_fragment, \
    fragment_from_table
from .mfma import (mfma_c_fragment, mfma_a_fragment, compute_warp_partition, choose_swizzle, operand_swizzle,
                   swizzle_report)
from .hierarchical_layout import HierarchicalLayout, make_hierarchical_layout, make_blockwise_zz_layout


def Fragment(shape, forward_fn=None, forward_thread_fn=None, replicate: int = 1, forward_index_fn=None,
             num_threads=None, **kwargs):
    """Reference-style constructor ``T.Fragment(shape, forward_thread_fn=..., forward_index_fn=...)``.

    ``forward_fn(*idx) -> (thread, local)`` or separate thread/index functions.  The layout must be a
    mixed-radix digit placement (all CDNA MFMA layouts are); it is converted to the digit form used
    by the compiler.
    """
    shape = [int(s) for s in shape]
    if forward_fn is not None and forward_thread_fn is None:

        def ft(*idx):
            return forward_fn(*idx)[0]

        def fi(*idx):
            return forward_fn(*idx)[1]
    else:
        ft = forward_thread_fn
        fi = forward_index_fn if forward_index_fn is not None else (lambda *idx: 0)
    return fragment_from_table(shape, num_threads, ft, fi, replicate)


__all__ = [
    "Layout", "LinearLayout", "SwizzleLayout", "PaddedLayout", "Fragment", "Digit", "make_linear_fragment",
    "make_replicated_fragment", "mfma_c_fragment", "mfma_a_fragment", "compute_warp_partition", "choose_swizzle",
    "operand_swizzle", "swizzle_report", "HierarchicalLayout", "make_hierarchical_layout",
    "make_blockwise_zz_layout", "make_linear_layout", "make_swizzled_layout", "physical_size"
]


def make_metadata_layout(buffer, mma_dtype: str = "float16", block_k: int = None, arch=None, backend=None, **kwargs):
    """Layout of 2:4 sparse metadata ``E`` for ``T.gemm_sp`` (reference
    ``tilelang/layout/gemm_sp.py`` ``make_cutlass_metadata_layout``).  The NVIDIA ``mma.sp``
    metadata needs an interleaved CUTLASS layout; the gfx950 smfmac index of a lane is one
    16-bit word of the row, so ``E`` stays row-major: a linear layout for a shared tile and
    nothing to annotate (None) for a global tensor."""
    shape = buffer.static_shape() if hasattr(buffer, "static_shape") else None
    if getattr(buffer, "scope", "global") == "global" or shape is None:
        return None
    return LinearLayout(shape)


make_cutlass_metadata_layout = make_metadata_layout
