"""Tensor-level mesh collectives (host-issued) — the T.comm semantics on whole torch tensors.

Process meshes use ``torch.distributed`` on the row / column / world groups of the
``ProcessMesh`` — with the ``nccl`` backend that is RCCL over xGMI, so each call is one
bucketed collective per group, never a chain of hops.  Virtual meshes (all ranks in one
process) exchange tensors through a thread rendezvous, so model code written against this
module runs unchanged in CPU tests.

Directions follow T.comm: ``"h"`` = the ranks of my mesh row, ``"v"`` = my mesh column,
``"all"`` = every rank.  Core ids are linear (``row * ncol + col``) or ``(row, col)`` tuples.
The reference exposes these only as in-kernel ops (``language/comm.py``); its DeepSeek-V3.2
inference example uses raw ``dist.all_reduce`` / ``all_gather`` for TP/EP
(``examples/deepseek_v32/inference/model.py:245-284,787-850``) — those map onto this module.
"""
from __future__ import annotations

from typing import List, Optional, Union

import torch

from .mesh import MeshContext, MeshError, ProcessMesh, VirtualRank, current_mesh

Core = Union[int, tuple]


def _ctx(ctx: Optional[MeshContext]) -> MeshContext:
    ctx = ctx or current_mesh()
    if ctx is None:
        raise MeshError("no active mesh (tilelang.parallel.init_mesh() or VirtualMesh.run())")
    return ctx


def _core(ctx, c: Core) -> int:
    if isinstance(c, tuple):
        r, col = c
        return r * ctx.ncol + col
    return int(c)


def _key(ctx, name):
    # the per-rank collective sequence number lives on the rank object: a table keyed by id(ctx)
    # handed a new VirtualRank the stale count of a collected one that had the same id, so ranks
    # of one mesh deposited under different keys (intermittent None results)
    n = getattr(ctx, "_coll_seq", 0)
    ctx._coll_seq = n + 1
    return (name, n)


def _virtual_gather(ctx: VirtualRank, name: str, t: torch.Tensor, direction: str) -> List[torch.Tensor]:
    vals = ctx.collectives.exchange(_key(ctx, name), ctx.rank, t)
    return [vals[r] for r in ctx.group_ranks(direction)]


_OPS = {"sum", "max", "min", "avg", "prod"}


def _device_native(ctx, t: torch.Tensor, direction: str = "all") -> bool:
    """True when the process group moves ``t`` where it lives: a GPU tensor on an ``nccl`` (RCCL)
    group.  A GPU tensor on a gloo group (tests with several ranks sharing one GPU) is staged
    through host memory instead."""
    if not t.is_cuda:
        return False
    import torch.distributed as dist
    return dist.get_backend(ctx.group(direction)) == "nccl"


def _dist_op(op: str):
    import torch.distributed as dist
    return {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
            "prod": dist.ReduceOp.PRODUCT, "avg": dist.ReduceOp.SUM}[op]


def _reduce_list(xs: List[torch.Tensor], op: str) -> torch.Tensor:
    # fixed member order -> identical results on every rank
    acc = xs[0].clone()
    for x in xs[1:]:
        if op in ("sum", "avg"):
            acc += x
        elif op == "max":
            torch.maximum(acc, x, out=acc)
        elif op == "min":
            torch.minimum(acc, x, out=acc)
        elif op == "prod":
            acc *= x
    if op == "avg":
        acc /= len(xs)
    return acc


def all_reduce(t: torch.Tensor, op: str = "sum", direction: str = "all", ctx=None) -> torch.Tensor:
    """In-place reduction of ``t`` over the group; returns ``t``."""
    ctx = _ctx(ctx)
    if op not in _OPS:
        raise ValueError(f"reduce op must be one of {sorted(_OPS)}")
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        dist.all_reduce(t, op=_dist_op(op), group=ctx.group(direction))
        if op == "avg":
            t /= len(ctx.group_ranks(direction))
        return t
    t.copy_(_reduce_list(_virtual_gather(ctx, "all_reduce", t.clone(), direction), op))
    return t


def all_gather(t: torch.Tensor, direction: str = "all", ctx=None) -> torch.Tensor:
    """``[G, *t.shape]``: slice k comes from the k-th member of my group (T.comm order)."""
    ctx = _ctx(ctx)
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        G = len(ctx.group_ranks(direction))
        grp = ctx.group(direction)
        if _device_native(ctx, t, direction):
            out = torch.empty((G,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t.contiguous(), group=grp)
            return out
        th = t.detach().cpu().contiguous()
        out = torch.empty((G,) + tuple(t.shape), dtype=t.dtype)
        dist.all_gather(list(out.unbind(0)), th, group=grp)
        return out.to(t.device)
    return torch.stack(_virtual_gather(ctx, "all_gather", t.clone(), direction))


def broadcast(t: torch.Tensor, src_core: Core, direction: str = "all", ctx=None) -> torch.Tensor:
    """Members of ``src_core``'s group receive its ``t`` (in place); others keep theirs."""
    ctx = _ctx(ctx)
    src = _core(ctx, src_core)
    # the group is the one containing src_core
    r, c = divmod(src, ctx.ncol)
    d = direction.lower()
    if d in ("h", "horizontal"):
        members = [r * ctx.ncol + j for j in range(ctx.ncol)]
    elif d in ("v", "vertical"):
        members = [i * ctx.ncol + c for i in range(ctx.nrow)]
    else:
        members = list(range(ctx.world))
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        if d in ("h", "horizontal"):
            grp = ctx.row_groups[r]
        elif d in ("v", "vertical"):
            grp = ctx.col_groups[c]
        else:
            grp = ctx.world_group
        if ctx.rank in members:
            dist.broadcast(t, src=src, group=grp)
        return t
    vals = ctx.collectives.exchange(_key(ctx, "broadcast"), ctx.rank, t.clone())
    if ctx.rank in members:
        t.copy_(vals[src])
    return t


def put(t: torch.Tensor, src_core: Core, dst_core: Core, ctx=None) -> torch.Tensor:
    """Point-to-point: ``dst_core``'s ``t`` becomes ``src_core``'s (one xGMI hop)."""
    ctx = _ctx(ctx)
    s, d = _core(ctx, src_core), _core(ctx, dst_core)
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        if s == d:
            return t
        if ctx.rank == s:
            dist.send(t.contiguous(), dst=d)
        elif ctx.rank == d:
            dist.recv(t, src=s)
        return t
    vals = ctx.collectives.exchange(_key(ctx, "put"), ctx.rank, t.clone())
    if ctx.rank == d:
        t.copy_(vals[s])
    return t


def reduce_scatter(t: torch.Tensor, op: str = "sum", direction: str = "all", ctx=None) -> torch.Tensor:
    """Reduce over the group and keep chunk k (dim 0) on the k-th member."""
    ctx = _ctx(ctx)
    members = ctx.group_ranks(direction)
    G = len(members)
    if t.shape[0] % G:
        raise ValueError(f"reduce_scatter: dim 0 ({t.shape[0]}) not divisible by group size {G}")
    k = members.index(ctx.rank)
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        out = torch.empty((t.shape[0] // G,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if t.is_cuda:
            dist.reduce_scatter_tensor(out, t.contiguous(), op=_dist_op(op), group=ctx.group(direction))
            if op == "avg":
                out /= G
            return out
        full = t.clone()
        all_reduce(full, op, direction, ctx)
        return full.chunk(G, 0)[k].clone()
    red = _reduce_list(_virtual_gather(ctx, "reduce_scatter", t.clone(), direction), op)
    return red.chunk(G, 0)[k].clone()


def all_to_all(t: torch.Tensor, direction: str = "all", ctx=None) -> torch.Tensor:
    """Chunk j of dim 0 goes to member j; the result's chunk i came from member i (EP dispatch)."""
    ctx = _ctx(ctx)
    members = ctx.group_ranks(direction)
    G = len(members)
    if t.shape[0] % G:
        raise ValueError(f"all_to_all: dim 0 ({t.shape[0]}) not divisible by group size {G}")
    k = members.index(ctx.rank)
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        out = torch.empty_like(t)
        if t.is_cuda:
            dist.all_to_all_single(out, t.contiguous(), group=ctx.group(direction))
            return out
        g = all_gather(t, direction, ctx)
        return torch.cat([g[i].chunk(G, 0)[k] for i in range(G)], 0)
    vals = _virtual_gather(ctx, "all_to_all", t.clone(), direction)
    return torch.cat([vals[i].chunk(G, 0)[k] for i in range(G)], 0)


def all_to_all_v(t: torch.Tensor, send_counts: List[int], direction: str = "all", ctx=None):
    """Variable-size all-to-all along dim 0 (MoE token dispatch). Returns (out, recv_counts)."""
    ctx = _ctx(ctx)
    members = ctx.group_ranks(direction)
    G = len(members)
    if len(send_counts) != G:
        raise ValueError("send_counts must have one entry per group member")
    if isinstance(send_counts, torch.Tensor):
        cnt = send_counts.to(device=t.device, dtype=torch.int64)
    else:
        cnt = torch.tensor(send_counts, dtype=torch.int64, device=t.device)
    all_cnt = all_gather(cnt, direction, ctx)          # [G (src), G (dst)]
    k = members.index(ctx.rank)
    both = torch.cat([all_cnt[:, k], cnt]).tolist()     # the one host sync of the exchange
    recv_counts = [int(x) for x in both[:G]]
    send_counts = [int(x) for x in both[G:]]
    if isinstance(ctx, ProcessMesh) and _device_native(ctx, t, direction):
        import torch.distributed as dist
        out = torch.empty((sum(recv_counts),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if sum(send_counts) != t.shape[0]:
            raise ValueError("send_counts must sum to t.shape[0]")
        dist.all_to_all_single(out, t.contiguous(), output_split_sizes=recv_counts, input_split_sizes=send_counts,
                               group=ctx.group(direction))
        return out, recv_counts
    if isinstance(ctx, ProcessMesh):
        # gloo: pad to the max chunk and use the gathered view
        mx = max(max(int(x) for x in all_cnt.flatten().tolist()), 1)
        chunks = list(t.split(list(send_counts), 0))
        padded = torch.zeros((G * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        for j, ch in enumerate(chunks):
            padded[j * mx:j * mx + ch.shape[0]] = ch
        g = all_gather(padded, direction, ctx)
        out = torch.cat([g[i][k * mx:k * mx + recv_counts[i]] for i in range(G)], 0)
        return out, recv_counts
    vals = _virtual_gather(ctx, "all_to_all_v", (t.clone(), list(send_counts)), direction)
    parts = []
    for (ti, ci) in vals:
        off = sum(ci[:k])
        parts.append(ti[off:off + ci[k]])
    return torch.cat(parts, 0), recv_counts


def barrier(direction: str = "all", ctx=None):
    ctx = _ctx(ctx)
    if isinstance(ctx, ProcessMesh):
        import torch.distributed as dist
        if ctx.device.type == "cuda":
            torch.cuda.synchronize(ctx.device)
        dist.barrier(group=ctx.group(direction))
        return
    ctx.collectives.exchange(_key(ctx, "barrier"), ctx.rank, None)
