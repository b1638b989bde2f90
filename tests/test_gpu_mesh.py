"""T.comm on MI355X: the gfx950 protocol (peer stores into IPC/virtual workspaces, system-scope
flags) on a real GPU.  One GPU per box here, so the ranks share it: a VirtualMesh (one HIP
stream per rank) and two processes that exchange HIP IPC handles over gloo.  Results are
compared with plain PyTorch."""
import os
import socket

import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang.parallel import VirtualMesh, device_mesh_config

pytestmark = pytest.mark.gpu


def _program(nrow, ncol, M=64, N=128, blocks=2):
    world = nrow * ncol
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((M * blocks, N), "float16"), B: T.Tensor((M * blocks, N), "float16"),
                 G: T.Tensor((world, M * blocks, N), "float16"), R: T.Tensor((M * blocks,), "float32"),
                 S_: T.Tensor((M * blocks, N), "float32")):
            with T.Kernel(blocks, threads=256) as bx:
                a = T.alloc_fragment((M, N), "float16")
                b = T.alloc_fragment((M, N), "float16")
                f = T.alloc_fragment((M, N), "float32")
                f2 = T.alloc_fragment((M, N), "float32")
                g = T.alloc_shared((world, M, N), "float16")
                r = T.alloc_fragment((M,), "float32")
                T.copy(A[bx * M, 0], a)
                T.comm.broadcast(a, b, (0, ncol - 1), direction="all")
                T.copy(b, B[bx * M, 0])
                T.comm.all_gather(a, g, direction="all")
                T.copy(g, G[0:world, bx * M:(bx + 1) * M, 0:N])
                for i, j in T.Parallel(M, N):
                    f[i, j] = a[i, j]
                T.comm.all_reduce(f, r, "sum", "all", dim=1)
                T.copy(r, R[bx * M])
                # a large tile (M x N fp32 = 32 KiB): two-shot (reduce-scatter + all-gather) when
                # the group has more than two members
                T.comm.all_reduce_tile(f, f2, "sum", "all")
                T.copy(f2, S_[bx * M, 0])

        return tilelang.compile(main, target="hip")


def _check(rank, world, As, B, G, R, S_, src):
    torch.testing.assert_close(B, As[src])
    torch.testing.assert_close(G, torch.stack(As))
    ref = sum(a.float().sum(1) for a in As)
    torch.testing.assert_close(R, ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(S_, sum(a.float() for a in As), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("ncol", [2])
def test_virtual_mesh_gpu(ncol):
    """All ranks on one device, one HIP stream each: the kernels must run concurrently, so the
    mesh is limited by the process's hardware queues (GPU_MAX_HW_QUEUES = 4 on the test boxes,
    one of them the default stream): larger meshes run as processes (test_process_mesh_ipc_gpu)."""
    k = _program(1, ncol)
    vm = VirtualMesh(1, ncol, "cuda", workspace_bytes=16 << 20)
    torch.manual_seed(0)
    As = [torch.randn(128, 128, device="cuda", dtype=torch.float16) for _ in range(ncol)]
    outs = [(torch.zeros(128, 128, device="cuda", dtype=torch.float16),
             torch.zeros(ncol, 128, 128, device="cuda", dtype=torch.float16),
             torch.zeros(128, device="cuda"), torch.zeros(128, 128, device="cuda")) for _ in range(ncol)]

    def fn(ctx):
        k(As[ctx.rank], *outs[ctx.rank])

    for _ in range(3):  # several launches: epochs advance, no workspace reset
        vm.run(fn)
        vm.check()
    for r in range(ncol):
        _check(r, ncol, As, *outs[r], src=ncol - 1)
        assert torch.equal(outs[r][3], outs[0][3])  # bitwise identical on every rank


def test_mesh_grid_must_be_co_resident():
    """A T.comm kernel whose grid cannot be resident at once is refused before launch."""
    from tilelang.parallel.mesh import MeshError
    k = _program(1, 2, blocks=4096)
    vm = VirtualMesh(1, 2, "cuda", workspace_bytes=1 << 30)
    A = torch.randn(64 * 4096, 128, device="cuda", dtype=torch.float16)
    outs = (torch.zeros_like(A), torch.zeros(2, 64 * 4096, 128, device="cuda", dtype=torch.float16),
            torch.zeros(64 * 4096, device="cuda"), torch.zeros(64 * 4096, 128, device="cuda"))
    with pytest.raises(MeshError, match="co-resident"):
        vm.run(lambda ctx: k(A, *outs))


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
        # distinct GPUs when the box has them (xGMI peer stores), else all ranks share cuda:0
        dev = f"cuda:{rank % torch.cuda.device_count()}"
        torch.cuda.set_device(dev)
        ctx = init_mesh(1, world, device=dev)
        k = _program(1, world)
        torch.manual_seed(rank)
        A = torch.randn(128, 128, device=dev, dtype=torch.float16)
        B = torch.zeros_like(A)
        G = torch.zeros(world, 128, 128, device=dev, dtype=torch.float16)
        R = torch.zeros(128, device=dev)
        S_ = torch.zeros(128, 128, device=dev)
        for _ in range(3):
            k(A, B, G, R, S_)
        ctx.check()
        allA = [torch.zeros_like(A.cpu()) for _ in range(world)]
        dist.all_gather(allA, A.cpu())
        As = [a.to(dev) for a in allA]
        _check(rank, world, As, B, G, R, S_, src=world - 1)
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4])
def test_process_mesh_ipc_gpu(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=400) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res
