"""Host-level mesh collectives (virtual mesh threads and gloo processes) and MeshTensor
sharding round trips."""
import os
import socket

import pytest
import torch

from tilelang.language.annot import MeshReplicationType, MeshShardingPolicy
from tilelang.parallel import VirtualMesh, collectives as C
from tilelang.parallel.sharding import sharded_shape, shard_tensor, unshard_tensor


def _group(nrow, ncol, rank, d):
    r, c = divmod(rank, ncol)
    if d == "h":
        return [r * ncol + j for j in range(ncol)]
    if d == "v":
        return [i * ncol + c for i in range(nrow)]
    return list(range(nrow * ncol))


@pytest.mark.parametrize("direction", ["h", "v", "all"])
def test_virtual_collectives(direction):
    nrow, ncol = 2, 3
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=4096)
    xs = [torch.randn(6, 4) for _ in range(6)]

    def fn(ctx):
        r = ctx.rank
        out = {}
        out["ar"] = C.all_reduce(xs[r].clone(), "sum", direction)
        out["mx"] = C.all_reduce(xs[r].clone(), "max", direction)
        out["ag"] = C.all_gather(xs[r], direction)
        out["bc"] = C.broadcast(xs[r].clone(), (1, 2), direction)
        out["rs"] = C.reduce_scatter(xs[r].clone(), "sum", direction)
        out["a2a"] = C.all_to_all(xs[r].clone(), direction)
        out["put"] = C.put(xs[r].clone(), (0, 1), (1, 0))
        C.barrier(direction)
        return out

    res = vm.run(fn)
    for r in range(6):
        g = _group(nrow, ncol, r, direction)
        G = len(g)
        torch.testing.assert_close(res[r]["ar"], sum(xs[m] for m in g))
        torch.testing.assert_close(res[r]["mx"], torch.stack([xs[m] for m in g]).amax(0))
        torch.testing.assert_close(res[r]["ag"], torch.stack([xs[m] for m in g]))
        bg = _group(nrow, ncol, 5, direction)
        torch.testing.assert_close(res[r]["bc"], xs[5] if r in bg else xs[r])
        k = g.index(r)
        torch.testing.assert_close(res[r]["rs"], sum(xs[m] for m in g).chunk(G, 0)[k])
        torch.testing.assert_close(res[r]["a2a"], torch.cat([xs[m].chunk(G, 0)[k] for m in g], 0))
        torch.testing.assert_close(res[r]["put"], xs[1] if r == 3 else xs[r])


def test_virtual_all_to_all_v():
    vm = VirtualMesh(1, 3, "cpu", workspace_bytes=4096)
    counts = [[1, 2, 0], [0, 1, 3], [2, 2, 2]]
    xs = [torch.arange(sum(c) * 2, dtype=torch.float32).reshape(-1, 2) + 100 * r for r, c in enumerate(counts)]

    def fn(ctx):
        return C.all_to_all_v(xs[ctx.rank], counts[ctx.rank])

    res = vm.run(fn)
    for k in range(3):
        out, rc = res[k]
        assert rc == [counts[i][k] for i in range(3)]
        exp = torch.cat([xs[i][sum(counts[i][:k]):sum(counts[i][:k + 1])] for i in range(3)], 0)
        torch.testing.assert_close(out, exp)


@pytest.mark.parametrize("policy,shape", [
    (MeshShardingPolicy(x=1), (8, 10)),
    (MeshShardingPolicy(y=0), (9, 4)),
    (MeshShardingPolicy(x=1, y=0), (8, 12)),
    (MeshShardingPolicy(cross_mesh_dim=0), (13, 3)),
    (MeshShardingPolicy(y=0, replicate=MeshReplicationType.ROW), (8, 4)),
    (MeshShardingPolicy(x=1, replicate=MeshReplicationType.COLUMN), (4, 8)),
    (MeshShardingPolicy(replicate=MeshReplicationType.ALL), (3, 5)),
])
def test_shard_roundtrip(policy, shape):
    nrow, ncol = 2, 3
    full = torch.randn(shape)
    shards = [shard_tensor(full, policy, nrow, ncol, r, c) for r in range(nrow) for c in range(ncol)]
    ss = sharded_shape(shape, policy, nrow, ncol)
    assert all(tuple(s.shape) == ss for s in shards)
    torch.testing.assert_close(unshard_tensor(shards, policy, shape, nrow, ncol), full)
    if policy.replicate == MeshReplicationType.ROW:
        assert torch.equal(shards[0], shards[1]) and torch.equal(shards[0], shards[2])
    if policy.replicate == MeshReplicationType.COLUMN:
        assert torch.equal(shards[0], shards[3])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tilelang.parallel import init_mesh, shutdown_mesh
        from tilelang.parallel.sharding import gather_full, shard_for_rank
        ctx = init_mesh(2, 2)
        torch.manual_seed(0)
        xs = [torch.randn(4, 6) for _ in range(world)]
        x = xs[rank].clone()
        for d in ("h", "v", "all"):
            g = ctx.group_ranks(d)
            torch.testing.assert_close(C.all_reduce(x.clone(), "sum", d), sum(xs[m] for m in g))
            torch.testing.assert_close(C.all_gather(x, d), torch.stack([xs[m] for m in g]))
            k = g.index(rank)
            torch.testing.assert_close(C.reduce_scatter(x.clone(), "sum", d), sum(xs[m] for m in g).chunk(len(g), 0)[k])
            torch.testing.assert_close(C.all_to_all(x.clone(), d), torch.cat([xs[m].chunk(len(g), 0)[k] for m in g]))
        torch.testing.assert_close(C.broadcast(x.clone(), (1, 0), "v"), xs[2] if rank in (0, 2) else x)
        torch.testing.assert_close(C.put(x.clone(), (0, 1), (1, 1)), xs[1] if rank == 3 else x)
        out, rc = C.all_to_all_v(torch.full((rank + 1, 2), float(rank)), [rank + 1, 0, 0, 0])
        if rank == 0:
            assert rc == [1, 2, 3, 4] and out.shape[0] == 10
        full = torch.randn(8, 6)
        dist.broadcast(full, 0)
        pol = MeshShardingPolicy(x=1, y=0)
        torch.testing.assert_close(gather_full(shard_for_rank(full, pol), pol, full.shape), full)
        C.barrier()
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_process_collectives_gloo():
    import torch.multiprocessing as mp
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res
