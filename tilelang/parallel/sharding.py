"""MeshTensor sharding: split a full tensor into per-core shards and put it back together.

Follows the reference's ``MeshShardingPolicy`` math (``language/v2/annot.py:525-609``):
``x`` splits a dim into ``ncol`` blocks (core column picks the block), ``y`` into ``nrow``
blocks (core row picks it), ``cross_mesh_dim`` into ``nrow*ncol`` blocks (linear core id);
block sizes are ``ceil(dim / parts)``, the last block is zero-padded so every core sees the
same sharded shape the kernel was traced with.  ``replicate`` ROW (same data along a row, no
x split), COLUMN (no y split), ALL (full copy everywhere).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ..language.annot import MeshReplicationType, MeshShardingPolicy, MeshTensorAnnot


def sharded_shape(shape: Sequence[int], policy: MeshShardingPolicy, nrow: int, ncol: int) -> Tuple[int, ...]:
    return tuple(MeshTensorAnnot._get_sharded_shape(tuple(shape), policy, nrow, ncol))


def _splits(policy: MeshShardingPolicy, row: int, col: int, nrow: int, ncol: int):
    """[(dim, block_index)] for one core."""
    if policy.replicate == MeshReplicationType.ALL:
        return []
    if policy.cross_mesh_dim is not None:
        return [(policy.cross_mesh_dim, row * ncol + col)]
    out = []
    if policy.x is not None:
        out.append((policy.x, col))
    if policy.y is not None:
        out.append((policy.y, row))
    return out


def shard_tensor(full: torch.Tensor, policy: MeshShardingPolicy, nrow: int, ncol: int, row: int,
                 col: int) -> torch.Tensor:
    """The (padded) shard held by core ``(row, col)``."""
    sshape = sharded_shape(full.shape, policy, nrow, ncol)
    out = torch.zeros(sshape, dtype=full.dtype, device=full.device)
    src = [slice(None)] * full.dim()
    dst = [slice(None)] * full.dim()
    for dim, b in _splits(policy, row, col, nrow, ncol):
        n = sshape[dim]
        lo = b * n
        hi = min(lo + n, full.shape[dim])
        if lo >= hi:
            return out
        src[dim] = slice(lo, hi)
        dst[dim] = slice(0, hi - lo)
    out[tuple(dst)] = full[tuple(src)]
    return out


def unshard_tensor(shards: List[torch.Tensor], policy: MeshShardingPolicy, full_shape: Sequence[int], nrow: int,
                   ncol: int) -> torch.Tensor:
    """Inverse of ``shard_tensor`` from all cores' shards (index = linear core id)."""
    ref = shards[0]
    out = torch.zeros(tuple(full_shape), dtype=ref.dtype, device=ref.device)
    for cid, sh in enumerate(shards):
        row, col = divmod(cid, ncol)
        dst = [slice(None)] * out.dim()
        src = [slice(None)] * out.dim()
        skip = False
        for dim, b in _splits(policy, row, col, nrow, ncol):
            n = sh.shape[dim]
            lo = b * n
            hi = min(lo + n, full_shape[dim])
            if lo >= hi:
                skip = True
                break
            dst[dim] = slice(lo, hi)
            src[dim] = slice(0, hi - lo)
        if not skip:
            out[tuple(dst)] = sh[tuple(src)]
    return out


def shard_for_rank(full: torch.Tensor, policy: MeshShardingPolicy, ctx=None) -> torch.Tensor:
    """This rank's shard under the active mesh."""
    from .mesh import current_mesh
    ctx = ctx or current_mesh()
    return shard_tensor(full, policy, ctx.nrow, ctx.ncol, ctx.row, ctx.col)


def gather_full(local: torch.Tensor, policy: MeshShardingPolicy, full_shape: Sequence[int], ctx=None) -> torch.Tensor:
    """All-gather every rank's shard over the mesh and reassemble the full tensor."""
    from . import collectives
    from .mesh import current_mesh
    ctx = ctx or current_mesh()
    g = collectives.all_gather(local.contiguous(), "all", ctx)
    return unshard_tensor(list(g.unbind(0)), policy, full_shape, ctx.nrow, ctx.ncol)
