"""MoE expert-FFN kernels (tilelang DSL) and the token dispatch around them.

Layout (MI355X-first): tokens routed to expert ``e`` are packed into a row block of the
``padded`` activation matrix whose start is a multiple of ``block_M``; a ``tile_expert``
table gives the expert of every ``block_M`` row tile (``-1`` = empty tile, the block exits at
once).  Shapes are therefore static (``max_rows`` is the worst case), one compiled kernel
serves every routing, and the launches are hipGraph-capturable.

Reference: ``examples/grouped_gemm/example_grouped_gemm_fwd.py`` (group search per tile) and
``examples/fusedmoe/example_fusedmoe_tilelang.py`` (routed SwiGLU experts).
"""
from __future__ import annotations

import functools
from typing import Optional, Tuple

import torch

import tilelang
import tilelang.language as T


def _target(device) -> str:
    return "cpu" if torch.device(device).type == "cpu" else "hip"


def _tdt(dtype: torch.dtype) -> str:
    return {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[dtype]


@functools.lru_cache(maxsize=None)
def expert_gemm_kernel(max_rows: int, K: int, N: int, E: int, dtype: str, target: str, block_M: int = 128,
                       block_N: int = 128, block_K: int = 64, num_stages: int = 2, threads: int = 256,
                       reduce_mesh: Optional[str] = None, mesh_shape: Optional[Tuple[int, int]] = None):
    """``C[r, :] = A[r, :] @ W[tile_expert[r // block_M]].T`` for every non-empty row tile.

    ``reduce_mesh`` ("all"/"h"/"v"): tensor-parallel partial products are summed across the
    mesh inside the kernel (``T.comm.all_reduce_tile`` on the fp32 accumulator tile)."""
    n_tiles = max_rows // block_M
    accum = "float32"

    @T.prim_func
    def main(A: T.Tensor((max_rows, K), dtype), W: T.Tensor((E, N, K), dtype),
             tile_expert: T.Tensor((n_tiles,), "int32"), C: T.Tensor((max_rows, N), dtype)):
        with T.Kernel(n_tiles, T.ceildiv(N, block_N), threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, block_K), dtype)
            W_s = T.alloc_shared((block_N, block_K), dtype)
            C_l = T.alloc_fragment((block_M, block_N), accum)
            e = tile_expert[bx]
            if reduce_mesh is None:
                if e >= 0:
                    T.clear(C_l)
                    for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                        T.copy(A[bx * block_M, k * block_K], A_s)
                        T.copy(W[e, by * block_N, k * block_K], W_s)
                        T.gemm(A_s, W_s, C_l, transpose_B=True)
                    T.copy(C_l, C[bx * block_M, by * block_N])
            else:
                # every rank holds the same tile table (replicated tokens), so all ranks take
                # the same branch and meet at the same mesh op
                C_r = T.alloc_fragment((block_M, block_N), accum)
                if e >= 0:
                    T.clear(C_l)
                    for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                        T.copy(A[bx * block_M, k * block_K], A_s)
                        T.copy(W[e, by * block_N, k * block_K], W_s)
                        T.gemm(A_s, W_s, C_l, transpose_B=True)
                    T.comm.all_reduce_tile(C_l, C_r, "sum", reduce_mesh)
                    T.copy(C_r, C[bx * block_M, by * block_N])

    return tilelang.compile(main, out_idx=None, target=target)


def _mesh_shape():
    from ..parallel.mesh import get_device_mesh_config
    return get_device_mesh_config()


@functools.lru_cache(maxsize=None)
def silu_mul_kernel(rows: int, F: int, dtype: str, target: str, block_R: int = 32, threads: int = 256):
    """``out[r, j] = silu(H[r, j]) * H[r, F + j]`` (gate | up halves of the first expert GEMM)."""
    block_F = min(F, 256)
    assert F % block_F == 0 and rows % block_R == 0

    @T.prim_func
    def main(H: T.Tensor((rows, 2 * F), dtype), O: T.Tensor((rows, F), dtype)):
        with T.Kernel(rows // block_R, F // block_F, threads=threads) as (bx, by):
            for i, j in T.Parallel(block_R, block_F):
                g = T.Cast("float32", H[bx * block_R + i, by * block_F + j])
                u = T.Cast("float32", H[bx * block_R + i, F + by * block_F + j])
                O[bx * block_R + i, by * block_F + j] = T.Cast(dtype, g / (1.0 + T.exp(-g)) * u)

    return tilelang.compile(main, out_idx=None, target=target)


def max_padded_rows(n_assign: int, E: int, block_M: int) -> int:
    """Worst-case rows of the padded layout for ``n_assign`` (token, expert) pairs."""
    rows = n_assign + E * (block_M - 1)
    return (rows + block_M - 1) // block_M * block_M


def pack_by_expert(expert_ids: torch.Tensor, E: int, block_M: int, max_rows: int):
    """Padded placement of assignments grouped by expert.

    Returns ``(dest_row[n], tile_expert[max_rows // block_M], counts[E])``: assignment i goes
    to row ``dest_row[i]``; expert e's rows start at a multiple of ``block_M``."""
    dev = expert_ids.device
    n = expert_ids.numel()
    counts = torch.bincount(expert_ids, minlength=E)
    padded = (counts + block_M - 1) // block_M * block_M
    starts = torch.cumsum(padded, 0) - padded
    order = torch.argsort(expert_ids, stable=True)
    sorted_e = expert_ids[order]
    first = torch.cumsum(counts, 0) - counts
    rank_in_e = torch.arange(n, device=dev) - first[sorted_e]
    dest_sorted = starts[sorted_e] + rank_in_e
    dest = torch.empty_like(dest_sorted)
    dest[order] = dest_sorted
    n_tiles = max_rows // block_M
    tile_starts = torch.arange(n_tiles, device=dev) * block_M
    ends = starts + padded
    te = torch.full((n_tiles,), -1, dtype=torch.int32, device=dev)
    # tile t belongs to expert e if starts[e] <= t*block_M < ends[e]
    idx = torch.searchsorted(ends, tile_starts, right=True)
    valid = idx < E
    idx_c = idx.clamp(max=E - 1)
    valid &= (tile_starts >= starts[idx_c]) & (padded[idx_c] > 0)
    te[valid] = idx_c[valid].to(torch.int32)
    return dest, te, counts


def expert_ffn(x_rows: torch.Tensor, expert_ids: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor,
               block_M: int = 128, reduce_mesh: Optional[str] = None, cfg: Optional[dict] = None) -> torch.Tensor:
    """SwiGLU experts on already-dispatched rows: ``y_i = W2[e_i] (silu(g) * u)``, with
    ``[g | u] = W1[e_i] x_i``.  ``w1``: ``[E, 2F, H]``, ``w2``: ``[E, H, F]``."""
    cfg = dict(cfg or {})
    E, F2, H = w1.shape
    F = F2 // 2
    n = x_rows.shape[0]
    dev = x_rows.device
    tgt = _tdt(x_rows.dtype)
    target = _target(dev)
    # bucket the row count (power of two >= 256) so data-dependent EP receive sizes reuse a
    # handful of compiled kernels
    nb = 256
    while nb < n:
        nb *= 2
    max_rows = max_padded_rows(nb, E, block_M)
    dest, te, _ = pack_by_expert(expert_ids, E, block_M, max_rows)
    A = torch.zeros(max_rows, H, dtype=x_rows.dtype, device=dev)
    A[dest] = x_rows
    k1 = expert_gemm_kernel(max_rows, H, F2, E, tgt, target, block_M, **cfg)
    h = torch.empty(max_rows, F2, dtype=x_rows.dtype, device=dev)
    k1(A, w1, te, h)
    act = torch.empty(max_rows, F, dtype=x_rows.dtype, device=dev)
    silu_mul_kernel(max_rows, F, tgt, target)(h, act)
    k2 = expert_gemm_kernel(max_rows, F, H, E, tgt, target, block_M, reduce_mesh=reduce_mesh,
                            mesh_shape=_mesh_shape() if reduce_mesh else None, **cfg)
    y = torch.empty(max_rows, H, dtype=x_rows.dtype, device=dev)
    k2(act, w2, te, y)
    return y[dest]
