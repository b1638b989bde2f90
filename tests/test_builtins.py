"""T.print / T.sync_warp / T.sync_grid lower to real code (reference language/print.py,
builtin.py:676-701): printed values are checked on the CPU target; the grid barrier is checked
on the GPU (cooperative launch, every block sees every other block's pre-barrier writes)."""
import pytest
import torch

import tilelang
import tilelang.language as T


def print_kernel():

    @T.prim_func
    def main(A: T.Tensor((4, ), "float32"), B: T.Tensor((4, ), "float32")):
        with T.Kernel(1, threads=64):
            S = T.alloc_shared((4, ), "float32")
            T.copy(A, S)
            T.print(S, msg="shared")
            T.print(A[2], msg="scalar")
            T.sync_warp()
            T.copy(S, B)

    return main


def test_print_cpu(capfd):
    k = tilelang.compile(print_kernel(), target="cpu")
    a = torch.tensor([1.5, 2.5, 3.5, 4.5])
    b = torch.zeros(4)
    k(a, b)
    out = capfd.readouterr().out
    assert "shared S[3] = 4.5" in out and "scalar: 3.5" in out
    assert torch.equal(a, b)


def test_print_and_sync_hip_codegen():
    k = tilelang.compile(print_kernel(), target="hip")
    src = k.get_kernel_source()
    assert "tl::print_buffer" in src and "tl::print_val" in src and "tl::sync_warp()" in src
    assert len(k.code[0]) > 0


def grid_sync_kernel(nb, threads=256):

    @T.prim_func
    def main(X: T.Tensor((nb, ), "int32"), Y: T.Tensor((nb, ), "int32")):
        with T.Kernel(nb, threads=threads) as bx:
            for z in T.Parallel(1):
                X[bx + z] = bx + 1
            T.sync_grid()
            for z in T.Parallel(1):
                # every block reads its neighbour's pre-barrier write
                Y[bx + z] = X[(bx + 1) % nb]

    return main


def test_grid_sync_codegen():
    k = tilelang.compile(grid_sync_kernel(64), target="hip")
    src = k.get_kernel_source()
    # per-launch barrier workspace + device error word, no module-global barrier state
    assert "tl::sync_grid(tl_gsync_ws" in src and "tl_dev_err" in src
    assert k.artifact.kernels[0].cooperative
    names = [p["name"] for p in k.artifact.kernels[0].params]
    assert names[-2:] == ["tl_gsync_ws", "tl_dev_err"]


def grid_sync_skip_kernel(nb, threads=256):
    """Block 0 never reaches the barrier: every other block must time out, not hang."""

    @T.prim_func
    def main(X: T.Tensor((nb, ), "int32")):
        with T.Kernel(nb, threads=threads) as bx:
            if bx > 0:
                T.sync_grid()
            for z in T.Parallel(1):
                X[bx + z] = bx + 1

    return main


def test_grid_sync_skip_compiles():
    k = tilelang.compile(grid_sync_skip_kernel(64), target="hip",
                         compile_flags=["-DTL_GRID_SYNC_TIMEOUT_TICKS=2000000"])
    assert len(k.code[0]) > 0


@pytest.mark.gpu
def test_grid_sync_timeout_raises():
    """A forced grid-barrier timeout finishes the kernel and raises GridSyncTimeout at the next
    check point (and only once); a healthy launch afterwards works."""
    from tilelang.runtime import errors
    nb = 64
    k = tilelang.compile(grid_sync_skip_kernel(nb), target="hip",
                         compile_flags=["-DTL_GRID_SYNC_TIMEOUT_TICKS=2000000"])  # 20 ms
    x = torch.zeros(nb, dtype=torch.int32, device="cuda")
    k(x)
    with pytest.raises(errors.GridSyncTimeout):
        errors.check()
    errors.check()  # raised once
    good = tilelang.compile(grid_sync_kernel(nb), target="hip")
    y = torch.zeros(nb, dtype=torch.int32, device="cuda")
    good(x, y)
    errors.check()
    assert torch.equal(y, ((torch.arange(nb, device="cuda") + 1) % nb + 1).to(torch.int32))


@pytest.mark.gpu
def test_grid_sync_concurrent_streams():
    """Two launches of one grid-barrier kernel on two streams: per-launch barrier state."""
    nb = 64
    k = tilelang.compile(grid_sync_kernel(nb), target="hip")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(5):
        for s in (s1, s2):
            with torch.cuda.stream(s):
                x = torch.zeros(nb, dtype=torch.int32, device="cuda")
                y = torch.zeros(nb, dtype=torch.int32, device="cuda")
                k(x, y)
                outs.append(y)
    torch.cuda.synchronize()
    from tilelang.runtime import errors
    errors.check()
    exp = ((torch.arange(nb, device="cuda") + 1) % nb + 1).to(torch.int32)
    for y in outs:
        assert torch.equal(y, exp)


@pytest.mark.gpu
def test_grid_sync_gpu():
    nb = 256
    k = tilelang.compile(grid_sync_kernel(nb), target="hip")
    for _ in range(3):
        x = torch.zeros(nb, dtype=torch.int32, device="cuda")
        y = torch.zeros(nb, dtype=torch.int32, device="cuda")
        k(x, y)
        torch.cuda.synchronize()
        exp = (torch.arange(nb, device="cuda") + 1) % nb + 1
        assert torch.equal(y, exp.to(torch.int32))


@pytest.mark.gpu
def test_print_gpu(capfd):
    k = tilelang.compile(print_kernel(), target="hip")
    a = torch.tensor([1.5, 2.5, 3.5, 4.5], device="cuda")
    b = torch.zeros(4, device="cuda")
    k(a, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    out = capfd.readouterr().out
    assert "S[3]" in out


def test_no_barrier_inside_thread_guard():
    """Regression: the lowering's partial-thread guard (if tid < n) must never contain a block
    barrier (found in the DSA indexer backward: per-thread vector accesses to an LDS array were
    taken for cross-thread hazards and synchronised inside the guard)."""
    import os
    import sys
    import re
    import tilelang
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "examples", "dsa_sparse_finetune"))
    from indexer_bwd import indexer_bwd
    src = tilelang.lower(indexer_bwd.get_tir(128, 32, 64, 64), target="hip").kernel_source
    depth, guard_depths = 0, []
    for line in src.splitlines():
        if re.search(r"if \(\(tid_ < \d+\)\)", line):
            guard_depths.append(depth)
        if "sync_threads" in line or "barrier" in line:
            assert not guard_depths, "block barrier inside a thread-dependent guard"
        depth += line.count("{") - line.count("}")
        while guard_depths and depth <= guard_depths[-1]:
            guard_depths.pop()


def test_cross_wave_hazard_in_divergent_branch_is_refused():
    """A thread-dependent branch in which one wave writes LDS that another wave then reads
    cannot be synchronised (a barrier inside would deadlock): lowering must refuse it instead
    of emitting a silent race."""
    import pytest
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def bad(A: T.Tensor((256, ), "float32"), B: T.Tensor((256, ), "float32")):
        with T.Kernel(1, threads=256) as bx:
            S = T.alloc_shared((256, ), "float32")
            tx = T.get_thread_binding()
            if tx < 128:
                S[tx] = A[tx]
                B[tx] = S[tx + 64]  # written by another wave of the same branch
    with pytest.raises(RuntimeError, match="thread-dependent branch"):
        tilelang.lower(bad, target="hip")


def test_own_element_reuse_in_divergent_branch_is_allowed():
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def ok(A: T.Tensor((256, ), "float32"), B: T.Tensor((256, ), "float32")):
        with T.Kernel(1, threads=256) as bx:
            S = T.alloc_shared((256, ), "float32")
            tx = T.get_thread_binding()
            if tx < 128:
                S[tx] = A[tx] * 2.0
                B[tx] = S[tx] + 1.0  # the thread's own element
    src = tilelang.lower(ok, target="hip").kernel_source
    assert "sync_threads" not in src.split("if")[-1]


def test_register_set_under_thread_guard_is_not_uniform():
    """``if tid == 0: flag = 1`` makes ``flag`` per-thread: a barrier under ``if flag`` must be
    refused as divergent (it would deadlock), not taken as block-uniform."""
    import pytest
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def bad(A: T.Tensor((256, ), "float32"), B: T.Tensor((256, ), "float32")):
        with T.Kernel(1, threads=256) as bx:
            S = T.alloc_shared((256, ), "float32")
            flag = T.alloc_var("int32")
            tx = T.get_thread_binding()
            flag = 0
            if tx == 0:
                flag = 1
            if flag == 1:
                S[tx] = A[tx]
                T.sync_threads()
                B[tx] = S[255 - tx]
    with pytest.raises(RuntimeError):
        tilelang.lower(bad, target="hip")


def test_cross_thread_hazard_with_2d_threads_is_refused():
    """threads=(X, Y): the ownership proof must give tx and ty their own components of the flat
    id; with both set to the flat id, s[ty, tx] / s[ty, tx ^ 1] would look like one thread."""
    import pytest
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def bad(A: T.Tensor((8, 32), "float32"), B: T.Tensor((8, 32), "float32")):
        with T.Kernel(1, threads=(32, 8)) as bx:
            S = T.alloc_shared((8, 32), "float32")
            tx = T.get_thread_binding(0)
            ty = T.get_thread_binding(1)
            if tx < 16:
                S[ty, tx] = A[ty, tx]
                B[ty, tx] = S[ty, tx ^ 1]  # the neighbouring lane's element
    with pytest.raises(RuntimeError, match="thread-dependent branch"):
        tilelang.lower(bad, target="hip")

    @T.prim_func
    def ok(A: T.Tensor((8, 32), "float32"), B: T.Tensor((8, 32), "float32")):
        with T.Kernel(1, threads=(32, 8)) as bx:
            S = T.alloc_shared((8, 32), "float32")
            tx = T.get_thread_binding(0)
            ty = T.get_thread_binding(1)
            if tx < 16:
                S[ty, tx] = A[ty, tx] * 2.0
                B[ty, tx] = S[ty, tx] + 1.0  # own element
    tilelang.lower(ok, target="hip")


def test_lds_atomics_commute_without_barriers():
    """LDS atomics of one buffer commute: a histogram over several iterations per thread needs
    the barrier after the zero-fill and the one before the plain read, none between the atomic
    iterations (they were one barrier per unrolled iteration, each waiting on a global load)."""
    import re
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def hist(ids: T.Tensor((1024, ), "int32"), out: T.Tensor((8, ), "int32")):
        with T.Kernel(1, threads=256) as bx:
            cnt = T.alloc_shared((8, ), "int32")
            for e in T.Parallel(8):
                cnt[e] = 0
            for j in T.Parallel(1024):
                T.atomic_add(cnt[ids[j]], 1)
            for e in T.Parallel(8):
                out[e] = cnt[e]
    src = tilelang.lower(hist, target="hip").kernel_source
    body = src[src.find("__global__"):]
    assert body.count("atomic_add") == 4
    assert len(re.findall(r"sync_threads\(\)", body)) == 2
    # the barriers sit after the zero-fill and after the last atomic
    first_atomic, last_atomic = body.find("atomic_add"), body.rfind("atomic_add")
    bars = [m.start() for m in re.finditer(r"sync_threads\(\)", body)]
    assert bars[0] < first_atomic and bars[1] > last_atomic


def test_barrier_before_vector_load_addressed_through_lds():
    """Regression: a vectorised global load whose row id is read from LDS (``X[pos[r], c]``)
    reads ``pos``; the barrier between the write of ``pos`` and that load was missing when the
    load was emitted as one ``load_vec`` (its address expression was not scanned)."""
    import re
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def rows(X: T.Tensor((64, 64), "bfloat16"), order: T.Tensor((64, ), "int32"),
             out: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=128) as bx:
            pos = T.alloc_shared((16, ), "int32")
            acc = T.alloc_fragment((16, 64), "float32")
            red = T.alloc_fragment((64, ), "float32")
            T.clear(acc)
            for it in T.serial(4):
                for r in T.Parallel(16):
                    pos[r] = order[it * 16 + r]
                for r, c in T.Parallel(16, 64):
                    acc[r, c] += T.Cast("float32", X[pos[r], c])
            T.reduce_sum(acc, red, dim=0)
            T.copy(red, out)
    src = tilelang.lower(rows, target="hip", pass_configs={"tl.disable_safe_memory_legalize": True}).kernel_source
    body = src[src.find("for (int"):]
    loop = body[:body.find("reduce") if "reduce" in body else len(body)]
    assert "load_vec" in loop
    first_load = loop.find("load_vec")
    write = loop.find("&pos[")  # the staged row ids (a 16-byte copy into pos)
    assert 0 <= write < first_load
    assert re.search(r"sync_threads\(\)", loop[write:first_load]), loop[:800]


def test_cross_wave_reduction_barriers_left_to_thread_sync():
    """Two cross-wave row reductions per loop iteration (a softmax's max and sum over a tile split
    across waves) need one barrier each between the workspace stores and the partner loads; the
    barriers before the stores / after the loads are placed by ThreadSync only when a conflicting
    access since the last barrier exists (there were 3 per reduction)."""
    import re
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def two_reduce(A: T.Tensor((8, 64, 64), "float16"), B: T.Tensor((64, 64), "float16"),
                   O: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=512) as bx:
            a_s = T.alloc_shared((64, 64), "float16")
            b_s = T.alloc_shared((64, 64), "float16")
            s = T.alloc_fragment((64, 64), "float32")
            mx = T.alloc_fragment((64, ), "float32")
            sm = T.alloc_fragment((64, ), "float32")
            tot = T.alloc_fragment((64, ), "float32")
            T.copy(B, b_s)
            T.fill(tot, 0)
            for k in T.serial(8):
                T.copy(A[k, :, :], a_s)
                T.clear(s)
                T.gemm(a_s, b_s, s, policy=T.GemmWarpPolicy.Square)
                T.reduce_max(s, mx, dim=1)
                for i, j in T.Parallel(64, 64):
                    s[i, j] = s[i, j] - mx[i]
                T.reduce_sum(s, sm, dim=1)
                for i in T.Parallel(64):
                    tot[i] += sm[i]
            T.copy(tot, O)
    src = tilelang.lower(two_reduce, target="hip").kernel_source
    m = re.search(r"for \(int \w+ = 0; \w+ < 8;", src)
    loop = src[m.start():]  # the loop and the short tail after it
    assert "red_ws" in loop  # the row reductions cross waves (Square policy)
    n = len(re.findall(r"sync_threads\(\)", loop))
    # one each for: the a_s tile store -> gemm read, the max stores -> loads, the sum stores -> loads
    # (+ the loop-carried WAR / tail): with 3 barriers per reduction it would be >= 7
    assert n <= 5, (n, loop[:1500])
