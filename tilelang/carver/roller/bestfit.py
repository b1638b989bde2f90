"""Best-fit LDS packing for the carver's footprint model (reference ``tilelang/carver/roller/bestfit.py``).

The recommender must know how many LDS bytes a candidate needs *after* the compiler shares bytes
between buffers with disjoint lifetimes (``transform/lds_plan.py`` does this for real kernels):
a GEMM's staged C epilogue, for example, reuses the operand ring once the main loop is done, so
counting it on top of the ring would wrongly reject 256x256 tiles.

``BestFit`` is an address-ordered free list with best-fit placement and coalescing; ``pack``
places buffers with ``[start, end)`` lifetimes in the order the planner would (longest-lived and
largest first) and returns the arena size.  Offsets are aligned (16 bytes by default: the
``ds_read_b128`` / LDS-DMA granule).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass
class Block:
    start: int
    end: int
    free: bool

    @property
    def size(self) -> int:
        return self.end - self.start


class BestFit:

    def __init__(self, align: int = 16):
        self.align = align
        self.blocks: List[Block] = []
        self.limit = 0

    def _round(self, n: int) -> int:
        return (n + self.align - 1) // self.align * self.align

    def malloc(self, size: int) -> Block:
        size = self._round(max(size, 1))
        best: Optional[Block] = None
        for b in self.blocks:
            if b.free and b.size >= size and (best is None or b.size < best.size):
                best = b
        if best is not None:
            i = self.blocks.index(best)
            if best.size > size:  # split: the remainder stays free right after the allocation
                self.blocks.insert(i + 1, Block(best.start + size, best.end, True))
                best.end = best.start + size
            best.free = False
            return best
        if self.blocks and self.blocks[-1].free:  # grow the trailing free block
            tail = self.blocks[-1]
            tail.end = tail.start + size
            tail.free = False
            self.limit = tail.end
            return tail
        b = Block(self.limit, self.limit + size, False)
        self.blocks.append(b)
        self.limit = b.end
        return b

    def free(self, block: Block) -> None:
        if block.free:
            raise ValueError("double free")
        block.free = True
        merged: List[Block] = []
        for b in self.blocks:  # coalesce adjacent free blocks
            if merged and merged[-1].free and b.free and merged[-1].end == b.start:
                merged[-1].end = b.end
            else:
                merged.append(b)
        self.blocks = merged


def pack(buffers: Sequence[Tuple[str, int, int, int]], align: int = 16) -> Tuple[int, Dict[str, int]]:
    """``buffers``: (name, bytes, start, end) with a half-open live interval in program order.
    Returns (arena bytes, name -> offset)."""
    alloc = BestFit(align)
    events = []
    for name, nbytes, start, end in buffers:
        events.append((start, 1, -nbytes, name, nbytes))
        events.append((end, 0, 0, name, nbytes))
    live: Dict[str, Block] = {}
    offsets: Dict[str, int] = {}
    for _t, kind, _neg, name, nbytes in sorted(events):
        if kind == 0:  # frees before allocations at the same time step
            alloc.free(live.pop(name))
        else:
            b = alloc.malloc(nbytes)
            live[name] = b
            offsets[name] = b.start
    return alloc.limit, offsets


def gemm_lds_bytes(bm: int, bn: int, bk: int, stages: int, eb: int, staged_epilogue: bool = False,
                   out_eb: int = 2, pad: int = 8) -> int:
    """LDS arena of a pipelined GEMM tile: the ``stages``-deep A/B ring, plus (optionally) the
    row-padded C tile of the staged epilogue, which lives after the main loop and reuses the ring."""
    bufs = [("A", stages * bm * bk * eb, 0, 2), ("B", stages * bn * bk * eb, 0, 2)]
    if staged_epilogue:
        bufs.append(("C", bm * (bn + pad) * out_eb, 2, 3))
    return pack(bufs)[0]


__all__ = ["Block", "BestFit", "pack", "gemm_lds_bytes"]
