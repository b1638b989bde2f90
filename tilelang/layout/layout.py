"""Memory layouts (index maps) and LDS swizzles.

Reference: ``src/layout/layout.h`` (``LayoutNode``), ``src/layout/swizzle.{h,cc}``
and the CDNA swizzle ``makeMatrixCoreSwizzleLayout`` (``gemm_layouts.cc:441-462``,
32 banks x 32 bit, SIMD width 16).  gfx950's LDS is different: 64 banks x 4 B
per cycle for ``ds_read_b64/b128/b64_tr_b16`` with instruction-specific lane
groups (MI355X_MICROARCH §LDS), so swizzles here are *searched* against a bank
model of the exact instruction stream the GEMM lowering emits
(``tilelang/analysis/lds_bank.py``), then verified with ``SQ_LDS_BANK_CONFLICT``.

A shared tile ``[rows][cols]`` is stored row-major in 16-byte *chunks*; a
``SwizzleLayout`` XORs the chunk index with bits taken from the row index:
``pchunk = chunk ^ f(row)`` where ``f`` is a bit-gather of row bits.  XOR is an
involution, so the same map converts logical->physical and back, which is what
``global_load_lds`` needs (lane-linear LDS destination, swizzle moved to the
global *source* address — guide rule 21).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Tuple

from ..ir.expr import as_int


class Layout:
    """Generic index map ``logical idx -> physical idx`` given by Python callables."""

    def __init__(self, shape: Sequence, forward_fn: Callable, inverse_fn: Optional[Callable] = None,
                 output_shape: Optional[Sequence] = None, name: str = "layout"):
        self.shape = list(shape)
        self.forward_fn = forward_fn
        self.inverse_fn = inverse_fn
        self.output_shape = list(output_shape) if output_shape is not None else None
        self.name = name

    def forward(self, *idx):
        r = self.forward_fn(*idx)
        if not isinstance(r, (list, tuple)):
            r = [r]
        return list(r)

    def inverse(self, *phys):
        if self.inverse_fn is None:
            raise NotImplementedError(f"layout {self.name} has no inverse")
        r = self.inverse_fn(*phys)
        if not isinstance(r, (list, tuple)):
            r = [r]
        return list(r)

    def offset(self, *idx):
        """Linear element offset (for 1-output layouts)."""
        out = self.forward(*idx)
        if len(out) == 1:
            return out[0]
        oshape = self.output_shape
        off = 0
        for i, o in enumerate(out):
            off = off * oshape[i] + o if i else o
        return off

    def signature(self):
        return (self.name, tuple(self.shape))

    def is_equal(self, other) -> bool:
        return isinstance(other, Layout) and self.signature() == other.signature()

    def get_input_shape(self):
        return list(self.shape)

    def get_output_shape(self):
        return self.output_shape

    def map_forward_index(self, idx):
        return self.forward(*idx)

    def __repr__(self):
        return f"Layout({self.name}, {self.shape})"


class LinearLayout(Layout):
    """Plain row-major."""

    def __init__(self, shape):
        shape = list(shape)

        def fwd(*idx):
            off = 0
            for i, s in zip(idx, shape):
                off = off * s + i if not (isinstance(off, int) and off == 0) else i
            return [off]

        def inv(off):
            out = []
            for s in reversed(shape):
                out.append(off % s)
                off = off // s
            return list(reversed(out))

        super().__init__(shape, fwd, inv, [_prod(shape)], "linear")

    def signature(self):
        return ("linear", tuple(self.shape))


def _prod(xs):
    n = 1
    for x in xs:
        n = n * x
    return n


class SwizzleLayout(Layout):
    """``[..., rows, cols]`` tile, 16-B chunks permuted by ``chunk ^= gather(row bits)``.

    ``bits`` is a list of ``(row_bit, chunk_bit)``: bit ``row_bit`` of the row index is XORed into
    bit ``chunk_bit`` of the 16-byte chunk index within the row.
    """

    def __init__(self, shape, elem_bytes: int, bits: Sequence[Tuple[int, int]], name: str = "swizzle"):
        shape = [int(s) for s in shape]
        self.elem_bytes = elem_bytes
        self.bits = [tuple(b) for b in bits]
        self.rows = shape[-2] if len(shape) >= 2 else 1
        self.cols = shape[-1]
        row_bytes = self.cols * elem_bytes
        self.epc = 16 // elem_bytes            # elements per 16-byte chunk
        self.cpr = max(1, row_bytes // 16)     # chunks per row
        for rb, cb in self.bits:
            if (1 << cb) >= self.cpr:
                raise ValueError(f"swizzle chunk bit {cb} out of range for {self.cpr} chunks/row")
        cols, epc, lead = self.cols, self.epc, shape[:-2]

        def xor_term(row):
            t = 0
            for rb, cb in self.bits:
                bit = (row >> rb) & 1 if rb else row & 1
                term = bit << cb if cb else bit
                t = term if (isinstance(t, int) and t == 0) else (t ^ term)
            return t

        self._xor_term = xor_term

        def fwd(*idx):
            *outer, r, c = idx
            chunk = c // epc
            within = c % epc
            pchunk = chunk ^ xor_term(r) if self.bits else chunk
            off = r * cols + pchunk * epc + within
            base = 0
            for i, s in zip(outer, lead):
                base = base * s + i
            if lead:
                off = base * (self.rows * cols) + off
            return [off]

        def inv(off):
            tile = self.rows * cols
            outer = []
            if lead:
                o = off // tile
                off = off % tile
                for s in reversed(lead):
                    outer.append(o % s)
                    o = o // s
                outer.reverse()
            r = off // cols
            pc = (off % cols) // epc
            within = off % epc
            chunk = pc ^ xor_term(r) if self.bits else pc
            return outer + [r, chunk * epc + within]

        super().__init__(shape, fwd, inv, [_prod(shape)], name)

    def signature(self):
        return ("swizzle", tuple(self.shape), self.elem_bytes, tuple(self.bits))

    def __repr__(self):
        return f"SwizzleLayout({self.shape}, eb={self.elem_bytes}, bits={self.bits})"


class PaddedLayout(Layout):
    """Row padding (``pad`` elements per row) — for register-staged writes whose conflicts
    cannot be fixed by an XOR swizzle (e.g. fp32 transposed tiles)."""

    def __init__(self, shape, pad: int):
        shape = [int(s) for s in shape]
        self.pad = pad
        cols = shape[-1]
        rows = shape[-2] if len(shape) >= 2 else 1
        stride = cols + pad

        def fwd(*idx):
            *outer, r, c = idx
            base = 0
            for i, s in zip(outer, shape[:-2]):
                base = base * s + i
            off = r * stride + c
            if shape[:-2]:
                off = base * (rows * stride) + off
            return [off]

        super().__init__(shape, fwd, None, [_prod(shape[:-2] or [1]) * rows * stride], "padded")

    def signature(self):
        return ("padded", tuple(self.shape), self.pad)


def physical_size(layout: Optional[Layout], shape) -> int:
    """Elements of storage a shared buffer with this layout needs."""
    if layout is None or layout.output_shape is None:
        return int(_prod([as_int(s) for s in shape]))
    return int(_prod(layout.output_shape))


# reference-compatible constructors (tilelang/layout/swizzle.py) --------------------------


def make_linear_layout(buffer_or_shape, *args):
    shape = buffer_or_shape.shape if hasattr(buffer_or_shape, "shape") else buffer_or_shape
    return LinearLayout([as_int(s) for s in shape])


def make_swizzled_layout(buffer, k_major: bool = True, allow_pad: bool = True):
    from .mfma import default_operand_swizzle
    shape = [as_int(s) for s in buffer.shape]
    return default_operand_swizzle(shape, buffer.dtype.bytes)


def make_full_bank_swizzled_layout(buffer):
    return make_swizzled_layout(buffer)


def make_half_bank_swizzled_layout(buffer):
    return make_swizzled_layout(buffer)


def make_quarter_bank_swizzled_layout(buffer):
    return make_swizzled_layout(buffer)
