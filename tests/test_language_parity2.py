"""Language parity sweep, part 2: ports of the reference's testing/python/language/
test_tilelang_language_{copy,annot,alias,frontend_v2}.py, test_tilelang_intimm.py and
test_tilelang_capture.py (see test_language_parity.py for part 1).  CPU-target numerics where
the program means the same with one thread per block, gfx950 runs under the ``gpu`` marker."""
import gc
import weakref

import pytest
import torch

import tilelang
import tilelang.language as T

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
TD = {"float16": torch.float16, "float32": torch.float32, "float": torch.float32}


def _compile(prog, dev, **kw):
    return tilelang.compile(prog, target="cpu" if dev == "cpu" else "hip", **kw)


# ---- test_tilelang_language_copy.py -------------------------------------------------------


def copy_program(M, N, bm, bn, dtype):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            for i, j in T.Parallel(bm, bn):
                B[by * bm + i, bx * bn + j] = A[by * bm + i, bx * bn + j]

    return main


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("M,N,bm,bn,dtype", [(256, 256, 128, 128, "float16"), (128, 576, 32, 576, "float16"),
                                             (128, 576, 32, 576, "float")])
def test_copy(dev, M, N, bm, bn, dtype):
    k = _compile(copy_program(M, N, bm, bn, dtype), dev, out_idx=[1])
    a = torch.randn(M, N, device=dev).to(TD[dtype])
    assert torch.equal(k(a), a)


def copy_stride_program(M, N, NN, bm, bn, dtype="float16"):

    @T.prim_func
    def main(A: T.StridedTensor((M, N), (NN, 1), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            for i, j in T.Parallel(bm, bn):
                B[by * bm + i, bx * bn + j] = A[by * bm + i, bx * bn + j]

    return main


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("dyn", [False, True])
def test_copy_with_stride(dev, dyn):
    M, N = 256, 256
    NN = T.dynamic("NN") if dyn else 512
    k = _compile(copy_stride_program(M, N, NN, 128, 128), dev, out_idx=[1])
    a = torch.randn(M, 2 * N, device=dev).half()
    assert torch.equal(k(a[:, :N]), a[:, :N])


@pytest.mark.parametrize("dev", DEVS)
def test_copy_bufferload(dev):
    n = 128

    @T.prim_func
    def main(indices: T.Tensor((n, ), "int32"), x: T.Tensor((n, ), "float16")):
        with T.Kernel(n, threads=64) as pid:
            idx = T.alloc_local([1], "int32")
            T.copy(indices[pid], idx[0])
            for z in T.Parallel(1):
                x[idx[0] + z] = x[idx[0] + z] + 1

    k = _compile(main, dev)
    perm = torch.randperm(n, device=dev).int()
    x = torch.zeros(n, device=dev).half()
    k(perm, x)
    assert torch.equal(x, torch.ones_like(x))


@pytest.mark.parametrize("dev", DEVS)
def test_copy_buffer_load_with_parallel(dev):
    M = N = 256

    @T.prim_func
    def main(A: T.Tensor((M, N), "float16"), B: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, 128), T.ceildiv(M, 128), threads=128) as (bx, by):
            for i, j in T.Parallel(128, 128):
                T.copy(A[by * 128 + i, bx * 128 + j], B[by * 128 + i, bx * 128 + j])

    k = _compile(main, dev, out_idx=[1])
    a = torch.randn(M, N, device=dev).half()
    assert torch.equal(k(a), a)


# ---- test_tilelang_language_annot.py: symbolic extents a * n + b ------------------------


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("form", ["mul", "add", "mul_add"])
def test_tensor_annot_symbolic_expr(dev, form):
    n = T.symbolic("n")
    ext = {"mul": n * 4, "add": n + 1, "mul_add": n * 3 + 1}[form]

    @T.prim_func
    def kernel(A: T.Tensor((ext, ), T.int32)):
        with T.Kernel(1) as _:
            for i in range(ext):
                A[i] = 0

    k = _compile(kernel, dev)
    A = torch.arange(16, dtype=torch.int32, device=dev)
    k(A)
    assert torch.equal(A, torch.zeros_like(A))
    if form == "mul":
        with pytest.raises(ValueError, match="not of the form"):
            k(torch.arange(15, dtype=torch.int32, device=dev))


# ---- test_tilelang_language_alias.py ------------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_alias_slices_and_let(dev):
    M = N = K = 256
    bm = bn = 128
    bk = 32

    @T.prim_func
    def main(A: T.Tensor((M, K), "float16"), B: T.Tensor((N, K), "float16"), C: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=256) as (bx, by):
            A_shared = T.alloc_shared((bm, bk), "float16")
            B_shared = T.alloc_shared((bn, bk), "float16")
            C_local = T.alloc_fragment((bm, bn), "float")
            T.clear(C_local)
            X_shared = A_shared[:bm, :bk]
            for ko in T.Pipelined(T.ceildiv(K, bk), num_stages=0):
                off = ko * bk
                T.copy(A[by * bm, off], X_shared)
                T.copy(B[bx * bn, ko * bk], B_shared[:bn, :bk])
                T.gemm(X_shared, B_shared, C_local, transpose_B=True)
            T.copy(C_local, C[by * bm, bx * bn])

    k = _compile(main, dev, out_idx=[2])
    a = torch.randn(M, K, device=dev).half()
    b = torch.randn(N, K, device=dev).half()
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float().T, rtol=1e-2, atol=1e-1)


# ---- test_tilelang_intimm.py --------------------------------------------------------------


def test_intimm_extremes():
    T.int32(0x7fffffff)
    T.int32(-0x7fffffff - 1)
    T.uint32(0xffffffff)
    T.int64(0x7fffffffffffffff)
    T.int64(-0x7fffffffffffffff - 1)
    T.uint64(0xffffffffffffffff)
    a = T.int32()
    a & 0x7fffffff
    a = T.uint32()
    a & 0xffffffff
    a = T.int64()
    a & 0x7fffffffffffffff
    a = T.uint64()
    a & T.uint64(0xffffffffffffffff)


# ---- test_tilelang_capture.py: a compiled kernel keeps no reference to call-site tensors ---


def test_kernel_does_not_capture_tensors():

    @T.prim_func
    def dummy(a: T.Tensor((1, ), T.float32)):
        with T.Kernel(1) as _:
            a[0] = 1

    a = torch.randn(1, 1024)
    ref = weakref.ref(a)
    _k = tilelang.compile(dummy, target="cpu")
    del a
    gc.collect()
    assert ref() is None


# ---- test_tilelang_language_frontend_v2.py ------------------------------------------------


def test_argument_dtypes():

    @T.prim_func
    def args(t_1: T.bool, t_2: T.short, t_3: T.int, t_4: T.long, t_5: T.half, t_6: T.float, t_8: T.int8,
             t_9: T.int16, t_10: T.int32, t_11: T.int64, t_12: T.uint8, t_13: T.uint16, t_14: T.uint32,
             t_15: T.uint64, t_21: T.float16, t_22: T.bfloat16, t_23: T.float32, t_24: T.float64):
        pass

    assert len(args.params) == 18


@pytest.mark.parametrize("dev", DEVS)
def test_annotated_var_assign(dev):

    @T.prim_func
    def main(A: T.Tensor((2, ), T.int32)):
        with T.Kernel(1) as _:
            a: T.int32 = 1
            b: T.int32 = a
            a = 2
            d: T.int32 = a
            A[0] = b
            A[1] = d

    res = _compile(main, dev, out_idx=-1)()
    assert int(res[0]) == 1 and int(res[1]) == 2


def test_macro_return():

    @T.macro
    def ret_const():
        return 0

    @T.macro
    def ret_frame(x):
        return T.alloc_var(T.float32, init=x)

    @T.macro
    def ret_expr(x):
        y = x + 1.0
        return y

    @T.macro
    def apply(x, fn):
        return fn(x)

    seen = []

    @T.prim_func
    def main():
        with T.Kernel(1) as _:
            seen.extend([ret_const(), ret_frame(3.0), ret_expr(4.0), apply(5.0, lambda x: x * 2.0)])

    assert len(seen) == 4 and all(x is not None for x in seen)


@pytest.mark.parametrize("dev", DEVS)
def test_serial_for_with_step(dev):

    @T.prim_func
    def pos(A: T.Tensor((10, ), T.int32)):
        with T.Kernel(1) as _:
            for i in range(0, 10, 2):
                A[i] = 1
            for i in range(1, 10, 2):
                A[i] = 2

    @T.prim_func
    def neg(A: T.Tensor((10, ), T.int32)):
        with T.Kernel(1) as _:
            for i in range(10, 0, -1):
                A[10 - i] = i

    r = _compile(pos, dev, out_idx=-1)().cpu()
    assert r.tolist() == [1, 2] * 5
    r = _compile(neg, dev, out_idx=-1)().cpu()
    assert r.tolist() == list(range(10, 0, -1))


@pytest.mark.parametrize("dev", DEVS)
def test_swap_logic(dev):

    @T.prim_func
    def swap_var(A: T.Tensor((2, ), T.float32)):
        with T.Kernel(1, threads=64) as _:
            a = T.alloc_var(T.float32, A[0])
            b = T.alloc_var(T.float32, A[1])
            a, b = b, a
            A[0], A[1] = a, b

    @T.prim_func
    def swap_idx(A: T.Tensor((2, ), T.float32)):
        with T.Kernel(1, threads=64) as _:
            A[0], A[1] = A[1], A[0]

    for f in (swap_var, swap_idx):
        d = torch.tensor([1.0, 2.0], device=dev)
        _compile(f, dev)(d)
        assert d.cpu().tolist() == [2.0, 1.0]


@pytest.mark.parametrize("dev", DEVS)
def test_while_loop(dev):

    @T.prim_func
    def main(A: T.Tensor((1, ), T.int32)):
        with T.Kernel(1) as _:
            i = T.alloc_var(T.int32, 0)
            s = T.alloc_var(T.int32)
            s = 0
            while i < 10:
                s += i
                i += 1
            A[0] = s

    assert int(_compile(main, dev, out_idx=-1)()[0]) == sum(range(10))
