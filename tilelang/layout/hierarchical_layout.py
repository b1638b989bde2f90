"""Hierarchical (multi-level, mixed-radix) layouts and the blockwise "ZZ" layout.

Reference (fork addition): ``src/layout/hierarchical_layout.cc:19-98`` and
``tilelang/layout/hierarchical_layout.py:15-247``.  Each logical dimension ``d`` is
decomposed into the hierarchical dims ``hdims[g0:g1]`` given by ``hgroups[d] =
(g0, g1)`` (most significant first); the physical offset is
``sum_i h_i * hstrides[i]``.  On MI355X this describes how a MeshTensor shard or a
tiled HBM tensor is laid out (e.g. 32x32 blocks stored contiguously).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

from .layout import Layout


@dataclass
class HierarchicalLayout:
    hdims: Tuple[int, ...]
    hstrides: Tuple[int, ...]
    hgroups: Tuple[Tuple[int, int], ...]
    logical_shape: Tuple[int, ...] = None

    def __post_init__(self):
        self.hdims = tuple(int(x) for x in self.hdims)
        self.hstrides = tuple(int(x) for x in self.hstrides)
        self.hgroups = tuple((int(a), int(b)) for a, b in self.hgroups)
        if len(self.hdims) != len(self.hstrides):
            raise ValueError("hdims and hstrides must have the same length")
        shape = []
        covered = []
        for g0, g1 in self.hgroups:
            if not (0 <= g0 <= g1 <= len(self.hdims)):
                raise ValueError(f"invalid hierarchical group {(g0, g1)}")
            n = 1
            for i in range(g0, g1):
                n *= self.hdims[i]
                covered.append(i)
            shape.append(n)
        if sorted(covered) != list(range(len(self.hdims))):
            raise ValueError("hierarchical groups must partition the hierarchical dims")
        # the native twin validates the same invariants and evaluates integer offsets
        from .._native import core
        self._native = core().HierarchicalLayout(list(self.hdims), list(self.hstrides), list(self.hgroups))
        if self.logical_shape is None:
            self.logical_shape = tuple(shape)
        elif tuple(self.logical_shape) != tuple(shape):
            raise ValueError(f"hierarchical dims {self.hdims} do not match logical shape {self.logical_shape}")

    @property
    def ndim(self):
        return len(self.logical_shape)

    def logical_to_hierarchical(self, idx: Sequence) -> List:
        out = [0] * len(self.hdims)
        for d, (g0, g1) in enumerate(self.hgroups):
            x = idx[d]
            for i in reversed(range(g0, g1)):
                out[i] = x % self.hdims[i]
                x = x // self.hdims[i]
        return out

    def hierarchical_to_logical(self, h: Sequence) -> List:
        out = []
        for g0, g1 in self.hgroups:
            x = 0
            for i in range(g0, g1):
                x = x * self.hdims[i] + h[i]
            out.append(x)
        return out

    def offset(self, idx: Sequence):
        if all(isinstance(i, int) for i in idx):
            return self._native.offset([int(i) for i in idx])
        h = self.logical_to_hierarchical(idx)
        off = 0
        for hi, s in zip(h, self.hstrides):
            off = off + hi * s
        return off

    def offsets(self) -> List[int]:
        """Offset of every logical element in row-major order (native)."""
        return self._native.offsets()

    def is_bijective(self) -> bool:
        return self._native.is_bijective()

    def offset_to_logical(self, off: int) -> List[int]:
        """Inverse (numeric): requires the strides to describe a bijection."""
        order = sorted(range(len(self.hdims)), key=lambda i: -self.hstrides[i])
        h = [0] * len(self.hdims)
        for i in order:
            h[i] = off // self.hstrides[i]
            off = off % self.hstrides[i]
        return self.hierarchical_to_logical(h)

    def size(self) -> int:
        n = 1
        for d in self.hdims:
            n *= d
        return n

    def as_layout(self) -> Layout:
        return Layout(list(self.logical_shape), lambda *idx: [self.offset(list(idx))], None, [self.size()],
                      name="hierarchical")


def make_hierarchical_layout(hdims, hstrides, hgroups, logical_shape=None) -> HierarchicalLayout:
    return HierarchicalLayout(tuple(hdims), tuple(hstrides), tuple(tuple(g) for g in hgroups),
                              tuple(logical_shape) if logical_shape is not None else None)


def make_blockwise_zz_layout(buffer_or_shape, block_size=(32, 32)) -> HierarchicalLayout:
    """Blockwise row-major-of-blocks ("ZZ") layout: blocks of ``block_size`` stored contiguously,
    blocks ordered row-major, elements inside a block row-major."""
    shape = buffer_or_shape.shape if hasattr(buffer_or_shape, "shape") else buffer_or_shape
    shape = [int(s) for s in shape]
    if len(shape) != 2:
        raise ValueError("blockwise ZZ layout needs a 2-D tensor")
    bm, bn = block_size
    M, N = shape
    if M % bm or N % bn:
        raise ValueError(f"shape {shape} is not divisible by block size {block_size}")
    hdims = (M // bm, bm, N // bn, bn)
    hstrides = (bm * N, bn, bm * bn, 1)
    return HierarchicalLayout(hdims, hstrides, ((0, 2), (2, 4)), (M, N))
