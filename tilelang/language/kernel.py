"""``T.Kernel`` launch frame and thread/block bindings.

Reference: ``tilelang/language/kernel.py:228-358`` (``KernelLaunchFrame``,
``get_thread_binding(s)``, ``get_block_binding(s)``) backed by
``src/ir.cc:233-299``.  Threads per block must be a multiple of the
64-lane CDNA wavefront (checked at lowering time).
"""
from __future__ import annotations

from typing import Optional

from ..ir import stmt as S
from ..ir.expr import Var, convert
from .builder import current_builder, BuilderError


class KernelLaunchFrame:

    def __init__(self, *grid, threads=128, is_cpu: bool = False, prelude: Optional[str] = None):
        if len(grid) == 1 and isinstance(grid[0], (list, tuple)):
            grid = tuple(grid[0])
        if len(grid) == 0:
            grid = (1, )
        if len(grid) > 3:
            raise ValueError("T.Kernel supports at most 3 grid dimensions")
        self.grid = [convert(g) for g in grid]
        if isinstance(threads, int):
            threads = [threads]
        elif threads is None:
            threads = [1] if is_cpu else [128]
        self.threads = [int(t) for t in threads]
        self.is_cpu = is_cpu
        self.prelude = prelude
        names = ["bx", "by", "bz"]
        self.block_vars = [Var(names[i]) for i in range(len(self.grid))]
        tnames = ["tx", "ty", "tz"]
        self.thread_vars = [Var(tnames[i]) for i in range(len(self.threads))]
        for v, g in zip(self.block_vars, self.grid):
            v.hint = ("block", g)

    def __enter__(self):
        b = current_builder()
        if b.in_kernel:
            raise BuilderError("nested T.Kernel is not supported")
        b.push("kernel")
        b.kernel_info = self
        if len(self.block_vars) == 1:
            return self.block_vars[0]
        return tuple(self.block_vars)

    def __exit__(self, et, ev, tb):
        b = current_builder()
        body = b.pop()
        b.kernel_info = None
        if et is None:
            k = S.KernelStmt(self.grid, self.threads, self.block_vars, self.thread_vars, body, self.is_cpu,
                             self.prelude)
            b.emit(k)
            b.kernel = k
        return False

    # reference API helpers
    def get_thread_binding(self, dim: int = 0):
        return self.thread_vars[dim]

    def get_thread_bindings(self):
        return list(self.thread_vars)

    def get_block_binding(self, dim: int = 0):
        return self.block_vars[dim]

    def get_block_bindings(self):
        return list(self.block_vars)

    def get_num_threads(self) -> int:
        n = 1
        for t in self.threads:
            n *= t
        return n


def Kernel(*grid, threads=None, is_cpu: bool = False, prelude: Optional[str] = None):
    if threads is None:
        threads = 1 if is_cpu else 128
    return KernelLaunchFrame(*grid, threads=threads, is_cpu=is_cpu, prelude=prelude)


def _kinfo() -> KernelLaunchFrame:
    k = current_builder().kernel_info
    if k is None:
        raise BuilderError("must be called inside T.Kernel")
    return k


def get_thread_binding(dim: int = 0):
    return _kinfo().thread_vars[dim]


def get_thread_bindings():
    return list(_kinfo().thread_vars)


def get_block_binding(dim: int = 0):
    return _kinfo().block_vars[dim]


def get_block_bindings():
    return list(_kinfo().block_vars)


def get_thread_extent(dim: int = 0):
    return _kinfo().threads[dim]


def get_block_extent(dim: int = 0):
    return _kinfo().grid[dim]


def get_thread_extents():
    return list(_kinfo().threads)


def get_block_extents():
    return list(_kinfo().grid)
