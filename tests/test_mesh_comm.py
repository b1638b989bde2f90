"""T.comm on a mesh: semantics of every op through the real device protocol (compiled for the
CPU target and executed by a VirtualMesh of threads, or by separate gloo processes sharing
/dev/shm workspaces), plus the reference's API validation.

Reference tests: ``testing/python/language/test_tilelang_language_comm.py`` (API + lowering
of broadcast/put/all_gather/all_reduce on a 4x4 mesh).  The reference never executes these ops
(no code generator); results here are checked against plain PyTorch.
"""
import os
import socket

import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang.parallel import VirtualMesh, device_mesh_config


def _dirs(nrow, ncol, rank, d):
    r, c = divmod(rank, ncol)
    if d == "h":
        return [r * ncol + j for j in range(ncol)]
    if d == "v":
        return [i * ncol + c for i in range(nrow)]
    return list(range(nrow * ncol))


def _run(vm, kernel, inputs, outputs):
    def fn(ctx):
        kernel(*inputs[ctx.rank], *outputs[ctx.rank])

    vm.run(fn)
    vm.check()


@pytest.mark.parametrize("nrow,ncol,direction,src", [(2, 2, "all", (1, 0)), (2, 2, "h", (0, 1)), (2, 3, "v", (1, 2)),
                                                     (1, 4, "h", (0, 3))])
def test_broadcast_cpu(nrow, ncol, direction, src):
    M, N = 8, 16
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((M, N), "float32"), B: T.Tensor((M, N), "float32")):
            with T.Kernel(2, threads=64) as bx:
                a = T.alloc_fragment((M // 2, N), "float32")
                b = T.alloc_fragment((M // 2, N), "float32")
                T.copy(A[bx * 4, 0], a)
                T.fill(b, -1.0)
                T.comm.broadcast(a, b, src, direction=direction)
                T.copy(b, B[bx * 4, 0])

        k = tilelang.compile(main, target="cpu")
    n = nrow * ncol
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=1 << 20)
    As = [torch.randn(M, N) for _ in range(n)]
    Bs = [torch.zeros(M, N) for _ in range(n)]
    _run(vm, k, [(a,) for a in As], [(b,) for b in Bs])
    s = src[0] * ncol + src[1]
    group = _dirs(nrow, ncol, s, {"all": "all", "h": "h", "v": "v"}[direction])
    for r in range(n):
        exp = As[s] if r in group else torch.full((M, N), -1.0)
        torch.testing.assert_close(Bs[r], exp)


@pytest.mark.parametrize("src,dst", [((0, 0), (0, 1)), ((0, 1), (1, 1)), ((1, 0), (0, 1)), ((1, 1), (1, 1))])
def test_put_cpu(src, dst):
    M, N = 16, 8
    with device_mesh_config(2, 2):

        @T.prim_func
        def main(A: T.Tensor((M, N), "float16"), B: T.Tensor((M, N), "float16")):
            with T.Kernel(1, threads=64) as bx:
                a = T.alloc_shared((M, N), "float16")
                b = T.alloc_fragment((M, N), "float16")
                T.copy(A, a)
                T.clear(b)
                T.comm.put(a, b, src, dst)
                T.copy(b, B)

        k = tilelang.compile(main, target="cpu")
    vm = VirtualMesh(2, 2, "cpu", workspace_bytes=1 << 20)
    As = [torch.randn(M, N).half() for _ in range(4)]
    Bs = [torch.zeros(M, N).half() for _ in range(4)]
    _run(vm, k, [(a,) for a in As], [(b,) for b in Bs])
    s, d = src[0] * 2 + src[1], dst[0] * 2 + dst[1]
    for r in range(4):
        torch.testing.assert_close(Bs[r], As[s] if r == d else torch.zeros(M, N).half())


@pytest.mark.parametrize("direction", ["h", "v", "all"])
def test_all_gather_cpu(direction):
    nrow, ncol = 2, 3
    M, N = 4, 8
    G = {"h": ncol, "v": nrow, "all": nrow * ncol}[direction]
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((M, N), "float32"), R: T.Tensor((G, M, N), "float32")):
            with T.Kernel(1, threads=64) as bx:
                a = T.alloc_fragment((M, N), "float32")
                g = T.alloc_fragment((G, M, N), "float32")
                T.copy(A, a)
                T.comm.all_gather(a, g, direction=direction)
                T.copy(g, R)

        k = tilelang.compile(main, target="cpu")
    n = nrow * ncol
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=1 << 20)
    As = [torch.randn(M, N) for _ in range(n)]
    Rs = [torch.zeros(G, M, N) for _ in range(n)]
    _run(vm, k, [(a,) for a in As], [(r,) for r in Rs])
    for r in range(n):
        torch.testing.assert_close(Rs[r], torch.stack([As[m] for m in _dirs(nrow, ncol, r, direction)]))


@pytest.mark.parametrize("kind,direction,dim,clear", [("sum", "all", -1, True), ("max", "h", 1, True),
                                                      ("absmax", "v", 0, True), ("sum", "h", 1, False),
                                                      ("min", "all", 0, True), ("abssum", "all", 1, True)])
def test_all_reduce_cpu(kind, direction, dim, clear):
    nrow, ncol = 2, 2
    M, N = 8, 16
    rd = dim % 2
    oshape = (N,) if rd == 0 else (M,)
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((M, N), "float32"), O_: T.Tensor(oshape, "float32")):
            with T.Kernel(1, threads=64) as bx:
                a = T.alloc_fragment((M, N), "float32")
                o = T.alloc_fragment(oshape, "float32")
                T.copy(A, a)
                T.fill(o, 1.0)
                T.comm.all_reduce(a, o, kind, direction, dim=dim, clear=clear)
                T.copy(o, O_)

        k = tilelang.compile(main, target="cpu")
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=1 << 20)
    As = [torch.randn(M, N) for _ in range(4)]
    Os = [torch.zeros(oshape) for _ in range(4)]
    _run(vm, k, [(a,) for a in As], [(o,) for o in Os])

    def local(x):
        if kind == "sum":
            return x.sum(rd)
        if kind == "abssum":
            return x.abs().sum(rd)
        if kind == "max":
            return x.amax(rd)
        if kind == "absmax":
            return x.abs().amax(rd)
        return x.amin(rd)

    for r in range(4):
        parts = torch.stack([local(As[m]) for m in _dirs(nrow, ncol, r, direction)])
        red = parts.sum(0) if "sum" in kind else (parts.amax(0) if "max" in kind else parts.amin(0))
        exp = red if clear else red + 1.0
        torch.testing.assert_close(Os[r], exp, rtol=1e-5, atol=1e-5)
    # every member of a group holds bitwise identical results
    for r in range(4):
        for m in _dirs(nrow, ncol, r, direction):
            assert torch.equal(Os[r], Os[m])


def test_comm_in_loop_barrier_and_core_id_cpu():
    """Repeated instances of one op inside a kernel loop (per-instance tags), several launches
    (epochs), T.comm.barrier and T.comm.current_core()."""
    nrow, ncol = 1, 2
    N = 64
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((N,), "float32"), O_: T.Tensor((N,), "float32")):
            with T.Kernel(3, threads=64) as bx:
                a = T.alloc_fragment((N,), "float32")
                o = T.alloc_fragment((2, N), "float32")
                T.copy(A, a)
                for it in T.serial(4):
                    T.comm.all_gather(a, o, direction="h")
                    for i in T.Parallel(N):
                        a[i] = o[0, i] + o[1, i]
                    T.comm.barrier()
                for i in T.Parallel(N):
                    a[i] = a[i] + T.comm.current_core() * 1000.0
                T.comm.fence()
                if bx == 0:
                    T.copy(a, O_)

        k = tilelang.compile(main, target="cpu")
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=1 << 20)
    As = [torch.randn(N) for _ in range(2)]
    Os = [torch.zeros(N) for _ in range(2)]
    for launch in range(3):
        _run(vm, k, [(a,) for a in As], [(o,) for o in Os])
        base = (As[0] + As[1]) * 8  # 4 rounds of pairwise sums: x_{k+1} = 2 x_k (both cores equal)
        for r in range(2):
            torch.testing.assert_close(Os[r], base + r * 1000.0)


def test_mesh_kernel_requires_active_mesh():
    with device_mesh_config(1, 2):

        @T.prim_func
        def main(A: T.Tensor((8,), "float32")):
            with T.Kernel(1, threads=64) as bx:
                a = T.alloc_fragment((8,), "float32")
                T.copy(A, a)
                T.comm.barrier()

        k = tilelang.compile(main, target="cpu")
    with pytest.raises(tilelang.parallel.MeshError, match="no mesh is active"):
        k(torch.zeros(8))
    vm = VirtualMesh(2, 2, "cpu", workspace_bytes=1 << 20)
    with pytest.raises(tilelang.parallel.MeshError, match="traced for a 1x2 mesh"):
        vm.run(lambda ctx: k(torch.zeros(8)))


def test_mesh_kernel_source_hip():
    """The gfx950 lowering: direct peer stores (vectorised), tagged flag protocol, mesh params."""
    with device_mesh_config(2, 4):

        @T.prim_func
        def main(A: T.Tensor((128, 128), "bfloat16"), B: T.Tensor((128, 128), "bfloat16")):
            with T.Kernel(4, threads=256) as bx:
                a = T.alloc_fragment((32, 128), "bfloat16")
                b = T.alloc_fragment((32, 128), "bfloat16")
                T.copy(A[bx * 32, 0], a)
                T.comm.broadcast(a, b, (1, 2), direction="v")
                T.copy(b, B[bx * 32, 0])

        art = tilelang.lower(main, target="hip")
    src = art.kernel_source
    assert "long long tl_mesh_ws" in src and "tl::mesh::publish" in src and "tl::mesh::wait_data" in src
    assert "tl::store_vec<bfloat16_t, 8>(&cm_out" in src  # 16-byte peer stores
    m = art.kernels[0].mesh
    assert m["shape"] == (2, 4) and m["nops"] == 1 and m["nblocks"] == 4
    assert m["slot_bytes"] == 32 * 128 * 2


# ------------------------------------------------------------------------------------------
# multi-process (gloo) — the same protocol across processes through /dev/shm workspaces
# ------------------------------------------------------------------------------------------


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _proc_worker(rank, world, port, q):
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tilelang.parallel import init_mesh, shutdown_mesh
        ctx = init_mesh(1, world)
        M, N = 8, 32

        @T.prim_func
        def main(A: T.Tensor((M, N), "float32"), O_: T.Tensor((M,), "float32"), G: T.Tensor((world, M, N), "float32")):
            with T.Kernel(2, threads=64) as bx:
                a = T.alloc_fragment((M // 2, N), "float32")
                o = T.alloc_fragment((M // 2,), "float32")
                g = T.alloc_fragment((world, M // 2, N), "float32")
                T.copy(A[bx * 4, 0], a)
                T.comm.all_reduce(a, o, "sum", "all", dim=1)
                T.comm.all_gather(a, g, direction="all")
                T.copy(o, O_[bx * 4])
                for w, i, j in T.Parallel(world, M // 2, N):
                    G[w, bx * 4 + i, j] = g[w, i, j]

        k = tilelang.compile(main, target="cpu")
        torch.manual_seed(rank)
        A = torch.randn(M, N)
        O_ = torch.zeros(M)
        G = torch.zeros(world, M, N)
        for _ in range(2):
            k(A, O_, G)
        ctx.check()
        allA = [torch.zeros(M, N) for _ in range(world)]
        dist.all_gather(allA, A)
        torch.testing.assert_close(O_, sum(x.sum(1) for x in allA), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(G, torch.stack(allA))
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_process_mesh_gloo_cpu():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_proc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


@pytest.mark.parametrize("direction,clear", [("all", True), ("h", False)])
def test_all_reduce_tile_cpu(direction, clear):
    """Tensor-parallel partial sums: element-wise tile reduction across cores."""
    nrow, ncol = 2, 2
    M, N = 16, 8
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((M, N), "float32"), O_: T.Tensor((M, N), "float32")):
            with T.Kernel(1, threads=64) as bx:
                a = T.alloc_fragment((M, N), "float32")
                o = T.alloc_fragment((M, N), "float32")
                T.copy(A, a)
                T.fill(o, 2.0)
                T.comm.all_reduce_tile(a, o, "sum", direction, clear=clear)
                T.copy(o, O_)

        k = tilelang.compile(main, target="cpu")
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=1 << 20)
    As = [torch.randn(M, N) for _ in range(4)]
    Os = [torch.zeros(M, N) for _ in range(4)]
    _run(vm, k, [(a,) for a in As], [(o,) for o in Os])
    for r in range(4):
        exp = sum(As[m] for m in _dirs(nrow, ncol, r, direction)) + (0 if clear else 2.0)
        torch.testing.assert_close(Os[r], exp)


@pytest.mark.parametrize("nrow,ncol,direction,kind", [(2, 2, "all", "sum"), (1, 4, "h", "max"), (4, 1, "v", "sum"),
                                                      (2, 4, "all", "sum")])
def test_all_reduce_tile_two_shot_cpu(nrow, ncol, direction, kind):
    """Large tiles reduce-scatter + all-gather: each member reduces one chunk (in member order)
    and broadcasts it, so every rank holds bitwise identical sums; the workspace holds chunks."""
    from tilelang.parallel import comm_lower
    M, N, blocks = 64, 64, 2
    n = nrow * ncol
    with device_mesh_config(nrow, ncol):

        @T.prim_func
        def main(A: T.Tensor((blocks * M, N), "float32"), O_: T.Tensor((blocks * M, N), "float32")):
            with T.Kernel(blocks, threads=128) as bx:
                a = T.alloc_fragment((M, N), "float32")
                o = T.alloc_fragment((M, N), "float32")
                for it in T.serial(2):  # two instances per launch
                    T.copy(A[bx * M, 0], a)
                    for i, j in T.Parallel(M, N):
                        a[i, j] = a[i, j] * (it + 1)
                    T.comm.all_reduce_tile(a, o, kind, direction)
                T.copy(o, O_[bx * M, 0])

        k = tilelang.compile(main, target="cpu")
    meta = k.artifact.kernels[0].mesh
    G = {"h": ncol, "v": nrow, "all": n}[direction]
    assert meta["slot_bytes"] == M * N * 4 // G          # chunk-sized slots
    one_shot = blocks * 1 * n * M * N * 4                 # nblocks * nops * nranks * tile
    assert meta["ws_bytes"] < one_shot * 2 // G + 8192
    vm = VirtualMesh(nrow, ncol, "cpu", workspace_bytes=4 << 20)
    As = [torch.randn(blocks * M, N) for _ in range(n)]
    Os = [torch.zeros(blocks * M, N) for _ in range(n)]
    for _ in range(2):
        _run(vm, k, [(a,) for a in As], [(o,) for o in Os])
    for r in range(n):
        parts = torch.stack([As[m] * 2 for m in _dirs(nrow, ncol, r, direction)])
        exp = parts.sum(0) if kind == "sum" else parts.amax(0)
        torch.testing.assert_close(Os[r], exp, rtol=1e-5, atol=1e-5)
        for m in _dirs(nrow, ncol, r, direction):
            assert torch.equal(Os[r], Os[m])


def test_two_shot_hip_source():
    with device_mesh_config(2, 4):

        @T.prim_func
        def main(A: T.Tensor((64, 64), "float32"), O_: T.Tensor((64, 64), "float32")):
            with T.Kernel(1, threads=256) as bx:
                a = T.alloc_fragment((64, 64), "float32")
                o = T.alloc_fragment((64, 64), "float32")
                T.copy(A, a)
                T.comm.all_reduce_tile(a, o, "sum", "all")
                T.copy(o, O_)

        src = tilelang.lower(main, target="hip").kernel_source
    assert "all-gather phase" in src and src.count("tl::mesh::publish") >= 2
