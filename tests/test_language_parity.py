"""Language-level parity sweep: ports of the reference's testing/python/language/ files.

One section per reference file (named in each section header).  Each program runs on the CPU
target (numerics against torch) wherever the op means something with one thread per block, and
on an MI355X (``gpu`` marker) against an fp32 torch reference; code-shape checks (vector
instructions, pragmas, no bounds branches) compile for gfx950 here.  Wave-level programs use
64-lane waves (the reference's CUDA tests use 32-thread warps).
NVIDIA-only files (tma_1d) have no port.
"""
import pytest
import torch

import tilelang
import tilelang.language as T

DEVS = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
GPU = [pytest.param("cuda", marks=pytest.mark.gpu)]
TD = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16, "float64": torch.float64,
      "int32": torch.int32}


def _compile(prog, dev, **kw):
    return tilelang.compile(prog, target="cpu" if dev == "cpu" else "hip", **kw)


def _isa(prog, **kw):
    return tilelang.compile(prog, target="hip", **kw).get_assembly()


# ---- test_tilelang_language_warp_reduce.py ------------------------------------------------


def warp_reduce_program(op, dtype, n=64):

    @T.prim_func
    def main(x: T.Tensor((n, ), dtype)):
        with T.Kernel(1, threads=n):
            tx = T.get_thread_binding(0)
            lv = T.alloc_local([1], dtype)
            lv[0] = x[tx]
            rv = T.alloc_local([1], dtype)
            if op == "sum":
                rv[0] = T.warp_reduce_sum(lv[0])
            elif op == "max":
                rv[0] = T.warp_reduce_max(lv[0])
            elif op == "min":
                rv[0] = T.warp_reduce_min(lv[0])
            elif op == "bitand":
                rv[0] = T.warp_reduce_bitand(lv[0])
            else:
                rv[0] = T.warp_reduce_bitor(lv[0])
            x[tx] = rv[0]

    return main


def _warp_ref(op, a):
    w = a.view(-1, 64)
    if op == "sum":
        r = w.sum(1)
    elif op == "max":
        r = w.amax(1)
    elif op == "min":
        r = w.amin(1)
    else:
        r = w[:, 0].clone()
        for i in range(1, 64):
            r = (r & w[:, i]) if op == "bitand" else (r | w[:, i])
    return r[:, None].expand(-1, 64).reshape(-1)


@pytest.mark.parametrize("dev", GPU)
@pytest.mark.parametrize("op", ["sum", "max", "min", "bitand", "bitor"])
def test_warp_reduce(dev, op):
    dt = "int32" if op.startswith("bit") else "float32"
    k = _compile(warp_reduce_program(op, dt, 128), dev)  # two waves: each reduces its own 64 lanes
    a = (torch.randint(0, 100, (128, ), dtype=torch.int32) if dt == "int32" else torch.randn(128)).to(dev)
    ref = _warp_ref(op, a)
    k(a)
    torch.testing.assert_close(a, ref)


def test_warp_reduce_compiles_hip_and_refused_on_cpu():
    for op in ("sum", "max", "min", "bitand", "bitor"):
        dt = "int32" if op.startswith("bit") else "float32"
        isa = _isa(warp_reduce_program(op, dt))
        assert "ds_swizzle" in isa or "v_permlane" in isa or "_dpp" in isa or "ds_bpermute" in isa
    # one thread per block on the CPU target: no wave to reduce over -> a clear error, never a
    # silently wrong identity
    with pytest.raises(Exception, match="CPU target"):
        tilelang.compile(warp_reduce_program("sum", "float32"), target="cpu")


# ---- test_tilelang_language_reduce.py -----------------------------------------------------


def reduce_rr(M, N, dtype, kind, clear=True, init=None):
    fn = getattr(T, "reduce_" + kind)

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, ), dtype)):
        with T.Kernel(1, threads=128):
            A_local = T.alloc_fragment((M, N), dtype)
            B_local = T.alloc_fragment((M, ), dtype)
            T.copy(A, A_local)
            if init is not None:
                T.fill(B_local, init)
            fn(A_local, B_local, dim=1, clear=clear)
            T.copy(B_local, B)

    return main


def reduce_ss(M, N, dtype, kind):
    fn = getattr(T, "reduce_" + kind)

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, ), dtype)):
        with T.Kernel(1, threads=128):
            A_shared = T.alloc_shared((M, N), dtype)
            B_shared = T.alloc_shared((M, ), dtype)
            T.copy(A, A_shared)
            fn(A_shared, B_shared, dim=1)
            T.copy(B_shared, B)

    return main


def _reduce_ref(A, kind):
    A = A.double() if A.is_floating_point() else A
    if kind == "sum":
        return A.sum(1)
    if kind == "max":
        return A.amax(1)
    if kind == "min":
        return A.amin(1)
    if kind == "abssum":
        return A.abs().sum(1)
    if kind == "absmax":
        return A.abs().amax(1)
    r = A[:, 0].clone()
    for j in range(1, A.shape[1]):
        r = {"bitand": r & A[:, j], "bitor": r | A[:, j], "bitxor": r ^ A[:, j]}[kind]
    return r


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("M,N,dtype,kind", [(256, 256, "float32", "sum"), (128, 512, "float32", "sum"),
                                            (256, 256, "float16", "max"), (256, 256, "float32", "max"),
                                            (128, 128, "float32", "min"), (128, 128, "float32", "abssum"),
                                            (128, 128, "float32", "absmax"), (64, 64, "int32", "bitand"),
                                            (64, 64, "int32", "bitor"), (64, 64, "int32", "bitxor")])
def test_reduce_fragment(dev, M, N, dtype, kind):
    k = _compile(reduce_rr(M, N, dtype, kind), dev)
    A = (torch.randint(0, 1 << 20, (M, N), dtype=torch.int32) if dtype == "int32" else torch.randn(M, N)).to(
        TD[dtype]).to(dev)
    B = torch.zeros(M, dtype=TD[dtype], device=dev)
    k(A, B)
    ref = _reduce_ref(A, kind)
    if dtype == "int32":
        assert torch.equal(B, ref)
    else:
        torch.testing.assert_close(B.double(), ref, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("kind", ["sum", "max", "min", "abssum", "absmax"])
def test_reduce_shared(dev, kind):
    k = _compile(reduce_ss(64, 64, "float32", kind), dev)
    A = torch.randn(64, 64, device=dev)
    B = torch.zeros(64, device=dev)
    k(A, B)
    torch.testing.assert_close(B.double(), _reduce_ref(A, kind), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("dev", DEVS)
def test_reduce_no_clear(dev):
    # clear=False accumulates into the destination's current value
    k = _compile(reduce_rr(256, 256, "float32", "sum", clear=False, init=1.0), dev)
    A = torch.randn(256, 256, device=dev)
    B = torch.zeros(256, device=dev)
    k(A, B)
    torch.testing.assert_close(B, A.sum(1) + 1, atol=1e-2, rtol=1e-2)
    k = _compile(reduce_rr(256, 256, "float16", "max", clear=False, init=-T.infinity("float16")), dev)
    A = torch.randn(256, 256, device=dev).half()
    B = torch.zeros(256, device=dev).half()
    k(A, B)
    torch.testing.assert_close(B, A.amax(1))


# ---- test_tilelang_language_cumsum.py -----------------------------------------------------


def cumsum_program(M, N, bm, bn, dim, reverse, scope, threads=256, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((bm, bn), dtype)
            T.copy(A[by * bm, bx * bn], A_shared)
            if scope == "smem":
                T.cumsum(src=A_shared, dim=dim, reverse=reverse)
                T.copy(A_shared, B[by * bm, bx * bn])
            else:
                A_frag = T.alloc_fragment((bm, bn), dtype)
                T.copy(A_shared, A_frag)
                T.cumsum(src=A_frag, dim=dim, reverse=reverse)
                T.copy(A_frag, B[by * bm, bx * bn])

    return main


def cumsum_1d_program(N, bn, reverse, scope, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((N, ), dtype), B: T.Tensor((N, ), dtype)):
        with T.Kernel(T.ceildiv(N, bn), threads=bn) as bx:
            A_shared = T.alloc_shared((bn, ), dtype)
            T.copy(A[bx * bn], A_shared)
            if scope == "smem":
                T.cumsum(src=A_shared, dim=0, reverse=reverse)
                T.copy(A_shared, B[bx * bn])
            else:
                A_frag = T.alloc_fragment((bn, ), dtype)
                T.copy(A_shared, A_frag)
                T.cumsum(src=A_frag, dim=0, reverse=reverse)
                T.copy(A_frag, B[bx * bn])

    return main


def _cumsum_ref(A, bm, bn, dim, reverse):
    M, N = A.shape
    t = A.double().view(M // bm, bm, N // bn, bn)
    d = 1 if dim == 0 else 3
    if reverse:
        t = t.flip(d)
    t = t.cumsum(d)
    if reverse:
        t = t.flip(d)
    return t.reshape(M, N)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("scope", ["smem", "fragment"])
@pytest.mark.parametrize("dim,reverse", [(0, False), (1, False), (1, True), (0, True)])
def test_cumsum(dev, scope, dim, reverse):
    M = N = 256
    bm = bn = 128
    k = _compile(cumsum_program(M, N, bm, bn, dim, reverse, scope), dev)
    A = torch.randn(M, N, device=dev)
    B = torch.zeros_like(A)
    k(A, B)
    torch.testing.assert_close(B.double(), _cumsum_ref(A, bm, bn, dim, reverse), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("scope", ["smem", "fragment"])
@pytest.mark.parametrize("reverse", [False, True])
def test_cumsum_1d(dev, scope, reverse):
    N, bn = 1024, 256
    k = _compile(cumsum_1d_program(N, bn, reverse, scope), dev)
    A = torch.randn(N, device=dev)
    B = torch.zeros_like(A)
    k(A, B)
    ref = _cumsum_ref(A.view(1, N), 1, bn, 1, reverse).view(N)
    torch.testing.assert_close(B.double(), ref, atol=1e-3, rtol=1e-3)


# ---- alloc_reducer / finalize_reducer (reference language/allocate.py, op/finalize_reducer) --


def reducer_program(M, N, op, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((N, ), dtype)):
        with T.Kernel(1, threads=128):
            R = T.alloc_reducer((N, ), dtype, op=op, replication="all")
            T.fill(R, 0.0 if op == "sum" else (-T.infinity(dtype) if op == "max" else T.infinity(dtype)))
            for i, j in T.Parallel(M, N):
                if op == "sum":
                    R[j] += A[i, j]
                elif op == "max":
                    R[j] = T.max(R[j], A[i, j])
                else:
                    R[j] = T.min(R[j], A[i, j])
            T.finalize_reducer(R)
            T.copy(R, B)

    return main


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("op", ["sum", "max", "min"])
def test_alloc_reducer(dev, op):
    M, N = 64, 32
    k = _compile(reducer_program(M, N, op), dev)
    A = torch.randn(M, N, device=dev)
    B = torch.zeros(N, device=dev)
    k(A, B)
    ref = {"sum": A.sum(0), "max": A.amax(0), "min": A.amin(0)}[op]
    torch.testing.assert_close(B, ref, atol=1e-4, rtol=1e-4)


# ---- test_tilelang_language_clamp.py ------------------------------------------------------


def clamp_program(N, bn, dtype, lo, hi):

    @T.prim_func
    def main(A: T.Tensor((N, ), dtype), B: T.Tensor((N, ), dtype)):
        with T.Kernel(T.ceildiv(N, bn), threads=bn) as bx:
            A_shared = T.alloc_shared([bn], dtype)
            T.copy(A[bx * bn], A_shared)
            for i in T.Parallel(bn):
                A_shared[i] = T.clamp(A_shared[i], min_val=lo, max_val=hi)
            T.copy(A_shared, B[bx * bn])

    return main


def clamp_range_program(N, bn, dtype):

    @T.prim_func
    def main(A: T.Tensor((1, N), dtype), B: T.Tensor((1, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), threads=bn) as bx:
            A_frag = T.alloc_fragment([1, bn], dtype=dtype)
            mn = T.alloc_fragment([1], dtype=dtype)
            mx = T.alloc_fragment([1], dtype=dtype)
            T.copy(A[0, bx * bn], A_frag)
            T.reduce_min(A_frag, mn, dim=1)
            T.reduce_max(A_frag, mx, dim=1)
            for i in T.Parallel(bn):
                A_frag[0, i] = T.clamp(A_frag[0, i], mn[0] * 0.5, mx[0] * 0.5)
            T.copy(A_frag, B[0, bx * bn])

    return main


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("dtype,lo,hi", [("float16", -0.05, 0.05), ("float32", -0.06, 0.05)])
def test_clamp(dev, dtype, lo, hi):
    k = _compile(clamp_program(1024, 128, dtype, lo, hi), dev)
    A = torch.randn(1024, device=dev).to(TD[dtype])
    B = torch.zeros_like(A)
    k(A, B)
    torch.testing.assert_close(B, torch.clamp(A, lo, hi), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("dtype", ["float16", "float32"])
def test_clamp_value_range(dev, dtype):
    N, bn = 1024, 128
    k = _compile(clamp_range_program(N, bn, dtype), dev)
    A = torch.randint(-5, 5, (1, N)).to(TD[dtype]).to(dev)
    B = torch.zeros_like(A)
    k(A, B)
    ref = torch.empty_like(A)
    for b in range(N // bn):
        blk = A[:, b * bn:(b + 1) * bn]
        ref[:, b * bn:(b + 1) * bn] = torch.clamp(blk, blk.min() * 0.5, blk.max() * 0.5)
    torch.testing.assert_close(B, ref)


# ---- test_tilelang_language_var_init.py / test_tilelang_language_alloc.py ----------------


@pytest.mark.parametrize("dev", DEVS)
def test_var_assign(dev):

    @T.prim_func
    def main(A: T.Tensor((2, ), "int32")):
        with T.Kernel(1):
            a = T.alloc_var("int32", init=1)
            b = T.alloc_var("int32", init=a)  # b gets the value of a
            a = 2
            d = T.alloc_var("int32", init=a)  # d gets the new value of a
            A[0] = b
            A[1] = d

    k = _compile(main, dev, out_idx=-1)
    res = k()
    assert res[0] == 1 and res[1] == 2


def alloc_var_program(N, bn, dtype, init=None, two=False):

    @T.prim_func
    def main(A: T.Tensor((N, ), dtype), B: T.Tensor((N, ), dtype)):
        with T.Kernel(T.ceildiv(N, bn), threads=bn) as bx:
            if two:
                t0 = T.alloc_var(dtype, 1)
                t1 = T.alloc_var(dtype, 2)
                for i in T.Parallel(bn):
                    B[bx * bn + i] = A[bx * bn + i] + t0 + t1
            elif init is not None:
                tmp = T.alloc_var(dtype, init)
                for i in T.Parallel(bn):
                    B[bx * bn + i] = tmp
            else:
                A_shared = T.alloc_shared([bn], dtype)
                tmp = T.alloc_var(dtype)
                tmp = 1
                T.copy(A[bx * bn], A_shared)
                for i in T.Parallel(bn):
                    A_shared[i] = A_shared[i] + tmp
                T.copy(A_shared, B[bx * bn])

    return main


@pytest.mark.parametrize("dev", DEVS)
def test_alloc_var(dev):
    k = _compile(alloc_var_program(1024, 128, "float16"), dev, out_idx=[1])
    assert "tmp" in k.get_kernel_source()
    A = torch.randn(1024, device=dev).half()
    torch.testing.assert_close(k(A), A + 1)
    k = _compile(alloc_var_program(256, 64, "int32", init=5), dev, out_idx=[1])
    assert "= 5;" in k.get_kernel_source()
    assert torch.equal(k(torch.zeros(256, dtype=torch.int32, device=dev)).cpu(), torch.full((256, ), 5,
                                                                                          dtype=torch.int32))
    k = _compile(alloc_var_program(256, 64, "int32", two=True), dev, out_idx=[1])
    src = k.get_kernel_source()
    assert src.count("= 1;") >= 1 and src.count("= 2;") >= 1
    A = torch.arange(256, dtype=torch.int32, device=dev)
    assert torch.equal(k(A), A + 3)


# ---- test_tilelang_language_vectorized_cast.py ------------------------------------------


def cast_program(M, da, db, parallel):

    @T.prim_func
    def main(A: T.Tensor((M, ), da), B: T.Tensor((M, ), db)):
        with T.Kernel(1, threads=128):
            if parallel:
                A_local = T.alloc_fragment((M, ), da)
                B_local = T.alloc_fragment((M, ), db)
                T.copy(A, A_local)
                for i in T.Parallel(M):
                    B_local[i] = A_local[i]
                T.copy(B_local, B)
            else:
                T.copy(A, B)

    return main


_CASTS = [("float32", "float16", "v_cvt_pk_f16_f32"), ("float32", "bfloat16", "v_cvt_pk_bf16_f32"),
          ("float16", "float32", "v_cvt_f32_f16"), ("bfloat16", "float32", None),
          ("float32", "float8_e4m3fn", "v_cvt_pk_fp8_f32"), ("float32", "float8_e5m2", "v_cvt_pk_bf8_f32")]
TD8 = dict(TD, float8_e4m3fn=torch.float8_e4m3fn, float8_e5m2=torch.float8_e5m2)


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("da,db,ins", _CASTS)
@pytest.mark.parametrize("lanes", [2, 4])
def test_vectorized_cast(dev, da, db, ins, lanes):
    M = 128 * lanes
    A = torch.randn(M).to(TD8[da]).to(dev)
    for par in (False, True):
        k = _compile(cast_program(M, da, db, par), dev)
        B = torch.zeros(M, device=dev).to(TD8[db])
        k(A, B)
        torch.testing.assert_close(B.float(), A.to(TD8[db]).float())
        if dev == "cpu" and ins is not None:
            # the packed convert instruction is used (the reference checks __float22half2_rn &c.)
            assert ins in _isa(cast_program(M, da, db, par))


# ---- test_tilelang_language_view.py / test_tilelang_language_reshape.py -----------------


def view_program(N, M, dtype, new_dtype=None, bad=False):
    shape = [N // M, M + (1 if bad else 0)]
    if new_dtype:
        from tilelang.ir.dtypes import as_dtype
        shape[-1] = int(M * as_dtype(dtype).bits / as_dtype(new_dtype).bits)

    @T.prim_func
    def main(A: T.Tensor((N, ), dtype), B: T.Tensor(shape, new_dtype or dtype)):
        with T.Kernel(1):
            Av = T.view(A, shape, dtype=new_dtype)
            T.copy(Av, B)

    return main


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("N,M,dtype,new", [(1024, 32, "float32", None), (2048, 64, "float16", None),
                                           (1024, 32, "float32", "float16"), (2048, 64, "float16", "float32")])
def test_view(dev, N, M, dtype, new):
    k = _compile(view_program(N, M, dtype, new), dev, out_idx=-1)
    A = torch.randn(N, device=dev).to(TD[dtype])
    ref = A.view(N // M, M)
    if new:
        ref = ref.view(dtype=TD[new])
    out = k(A)
    assert torch.equal(out.view(torch.uint8), ref.contiguous().view(torch.uint8))


def test_view_shape_mismatch():
    with pytest.raises((AssertionError, ValueError)):
        view_program(1024, 32, "float32", bad=True)


def reshape_program(N, M, dtype, kind):

    if kind == "global":

        @T.prim_func
        def main(A: T.Tensor((N, ), dtype), B: T.Tensor((N // M, M), dtype)):
            with T.Kernel(1):
                T.copy(T.reshape(A, [N // M, M]), B)
    elif kind == "smem_1d_2d":

        @T.prim_func
        def main(A: T.Tensor((N, ), dtype), B: T.Tensor((N // M, M), dtype)):
            with T.Kernel(1):
                A_shared = T.alloc_shared((N, ), dtype)
                for i in T.Parallel(N):
                    A_shared[i] = A[i]
                T.copy(T.reshape(A_shared, [N // M, M]), B)
    elif kind == "smem_2d_1d":

        @T.prim_func
        def main(A: T.Tensor((N // M, M), dtype), B: T.Tensor((N, ), dtype)):
            with T.Kernel(1):
                A_shared = T.alloc_shared((N // M, M), dtype)
                for i, j in T.Parallel(N // M, M):
                    A_shared[i, j] = A[i, j]
                T.copy(T.reshape(A_shared, [N]), B)
    else:  # fragment

        @T.prim_func
        def main(A: T.Tensor((N // M, M), dtype), B: T.Tensor((N, ), dtype)):
            with T.Kernel(1, threads=64):
                A_shared = T.alloc_shared((N // M, M), dtype)
                A_local = T.alloc_fragment((N // M, M), dtype)
                B_shared = T.alloc_shared((N, ), dtype)
                T.copy(A, A_shared)
                T.copy(A_shared, A_local)
                T.copy(T.reshape(A_local, [N]), B_shared)
                T.copy(B_shared, B)

    return main


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("kind", ["global", "smem_1d_2d", "smem_2d_1d", "fragment"])
@pytest.mark.parametrize("N,M,dtype", [(1024, 32, "float32"), (2048, 64, "float16")])
def test_reshape(dev, kind, N, M, dtype):
    k = _compile(reshape_program(N, M, dtype, kind), dev, out_idx=-1)
    shape_in = (N, ) if kind in ("global", "smem_1d_2d") else (N // M, M)
    A = torch.randn(shape_in, device=dev).to(TD[dtype])
    out = k(A)
    assert torch.equal(out.flatten(), A.flatten())


# ---- test_tilelang_language_ceildiv.py ----------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_ceildiv(dev):
    for a, b in ((128, 32), (1, 32), (-1, 32), (-2, 32), (33, 32)):

        @T.prim_func
        def main(A: T.Tensor((1, ), "int32")):
            with T.Kernel(1, threads=64):
                A[0] = T.ceildiv(T.int32(a), T.int32(b))

        k = _compile(main, dev, out_idx=[-1])
        assert int(k()[0]) == -(-a // b), (a, b)

    @T.prim_func
    def dyn(A: T.Tensor((1, ), "int32"), a: T.int32):
        with T.Kernel(1, threads=64):
            A[0] = T.ceildiv(a, T.int32(32))

    k = _compile(dyn, dev)
    for a in (128, 1, -1, -2, 33):
        A = torch.zeros(1, dtype=torch.int32, device=dev)
        k(A, a)
        assert int(A[0]) == -(-a // 32), a


# ---- test_tilelang_language_chain_equal.py ------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_chain_equal(dev):
    N, bs = 128, 64

    @T.prim_func
    def main(A: T.Tensor((N, ), "float32"), B: T.Tensor((N, ), "float32"), C: T.Tensor((N, ), "float32")):
        with T.Kernel(T.ceildiv(N, bs), threads=bs) as bx:
            for lane in T.Parallel(bs):
                idx = bx * bs + lane
                A[idx] = B[idx] = C[idx] = 1

    k = _compile(main, dev)
    ts = [torch.zeros(N, device=dev) for _ in range(3)]
    k(*ts)
    for t in ts:
        torch.testing.assert_close(t, torch.ones_like(t))


# ---- test_tilelang_language_clear.py ------------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_clear_shared_inside_pipeline(dev):
    M = N = K = 256
    bm, bn, bk = 128, 128, 32

    @T.prim_func
    def main(A: T.Tensor((M, K), "float16"), B: T.Tensor((N, K), "float16"), C: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=256) as (bx, by):
            A_shared = T.alloc_shared((bm, bk), "float16")
            B_shared = T.alloc_shared((bn, bk), "float16")
            C_local = T.alloc_fragment((bm, bn), "float")
            T.clear(C_local)
            for ko in T.Pipelined(T.ceildiv(K, bk), num_stages=0):
                T.copy(A[by * bm, ko * bk], A_shared)
                T.clear(A_shared)
                T.copy(B[bx * bn, ko * bk], B_shared)
                T.gemm(A_shared, B_shared, C_local, transpose_B=True)
            T.copy(C_local, C[by * bm, bx * bn])

    k = _compile(main, dev, out_idx=[2])
    c = k(torch.randn(M, K, device=dev).half(), torch.randn(N, K, device=dev).half())
    assert torch.count_nonzero(c) == 0


# ---- test_tilelang_language_if_range.py / test_tilelang_language_ternary.py --------------


@pytest.mark.parametrize("dev", DEVS)
def test_if_range(dev):
    M = N = 128
    bm = bn = 32

    @T.prim_func
    def main(A: T.Tensor((M, N), "float16"), B: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            for i, j in T.Parallel(bm, bn):
                r = by * bm + i
                c = bx * bn + j
                if 16 < r < 96:
                    B[r, c] = A[r, c] * 2.0
                else:
                    B[r, c] = A[r, c] * 0.5

    k = _compile(main, dev, out_idx=[1])
    a = torch.randn(M, N, device=dev).half()
    ref = a * 0.5
    ref[17:96] = a[17:96] * 2.0
    torch.testing.assert_close(k(a), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("dev", DEVS)
def test_ternary(dev):
    M = N = 128
    bm = bn = 32

    @T.prim_func
    def main(A: T.Tensor((M, N), "float16"), B: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            for i, j in T.Parallel(bm, bn):
                B[by * bm + i, bx * bn + j] = (A[by * bm + i, bx * bn + j] if (by * bm + i) < (M // 2) else 0)

    k = _compile(main, dev, out_idx=[1])
    a = torch.randn(M, N, device=dev).half()
    ref = a.clone()
    ref[M // 2:] = 0
    torch.testing.assert_close(k(a), ref)


# ---- test_tilelang_language_infinity.py ---------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32", "float64"])
def test_infinity(dev, dtype):

    @T.prim_func
    def main(A: T.Tensor((64, ), dtype)):
        with T.Kernel(1, threads=64):
            T.fill(A, T.infinity(dtype))

    out = _compile(main, dev, out_idx=-1)()
    assert torch.all(out == torch.inf)


# ---- test_tilelang_language_int64.py ------------------------------------------------------


def fill_program(n, value, dtype="bfloat16"):
    bn = 512

    @T.prim_func
    def main(x: T.Tensor[n, dtype]):
        with T.Kernel(T.ceildiv(n, bn), threads=128) as bx:
            for i in T.Parallel(bn):
                x[bx * bn + i] = value

    return main


def test_int64_index_codegen():
    # 2^32 elements: element offsets need 64-bit arithmetic (the grid alone is 2^23 blocks)
    src = tilelang.compile(fill_program(2**32, 1.0), target="hip").get_kernel_source()
    assert "int64_t" in src or "long" in src
    n = T.symbolic("n", "int64")
    src = tilelang.compile(fill_program(n, 1.0), target="hip").get_kernel_source()
    assert "int64_t" in src or "long" in src


@pytest.mark.gpu
def test_int64_fill_gpu():
    n = 2**32 + 1024  # 8 GiB of bf16: past the 32-bit element range
    x = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    tilelang.compile(fill_program(n, 1.0), target="hip")(x)
    assert x.min() == 1.0 and x.max() == 1.0
    x.zero_()
    tilelang.compile(fill_program(T.symbolic("n", "int64"), 1.0), target="hip")(x)
    assert x.min() == 1.0 and x.max() == 1.0
    del x
    torch.cuda.empty_cache()


# ---- test_tilelang_language_let.py --------------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_let_vectorize_load(dev):

    @T.prim_func
    def main(A: T.Tensor((16, 16), "float32")):
        with T.Kernel(1, threads=64):
            b = A[0, 0:4]
            A[0, 4:8] = b

    k = _compile(main, dev)
    A = torch.randn(16, 16, device=dev)
    ref = A.clone()
    ref[0, 4:8] = A[0, 0:4]
    k(A)
    torch.testing.assert_close(A, ref)
    if dev == "cpu":
        isa = _isa(main)
        # one 16-byte load (uniform address: clang may use the scalar s_load_dwordx4) and store
        assert ("global_load_dwordx4" in isa or "s_load_dwordx4 s[0:3], s[4:5], 0x0" in isa) and \
            "global_store_dwordx4" in isa


# ---- test_tilelang_language_mask_op.py ---------------------------------------------------


def mask_program(M, N, bm, bn, kind, dtype="float16"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=256) as (bx, by):
            A_shared = T.alloc_shared((bm, bn), dtype)
            tx = T.get_thread_binding(0)
            if kind == "parallel":
                if tx < 128:
                    for i, k in T.Parallel(bm, bn):
                        A_shared[i, k] = A[by * bm + i, bx * bn + k]
            elif kind == "copy":
                if tx < 128:
                    T.copy(A[by * bm, bx * bn], A_shared)
            else:
                if tx >= 128 and tx < 256:
                    for i, k in T.Parallel(bm, bn):
                        A_shared[i, k] = A[by * bm + i, bx * bn + k]
            T.copy(A_shared, B[by * bm, bx * bn])

    return main


@pytest.mark.parametrize("dev", GPU)
@pytest.mark.parametrize("kind", ["parallel", "copy", "parallel_range"])
def test_mask_op(dev, kind):
    # a T.Parallel / T.copy under a thread-range condition is partitioned over the threads that
    # run it (the reference's thread-range-aware layout inference)
    k = _compile(mask_program(512, 512, 128, 128, kind), dev, out_idx=[1])
    a = torch.randn(512, 512, device=dev).half()
    torch.testing.assert_close(k(a), a)


def mask_dyn_program(lo, hi):
    n = T.dynamic("n")

    @T.prim_func
    def main(A: T.Tensor((n, ), "float32"), B: T.Tensor((n, ), "float32")):
        with T.Kernel(1, threads=256):
            tx = T.get_thread_binding(0)
            if tx >= lo and tx < hi:
                for i in T.Parallel(A.shape[0]):  # dynamic extent: lower_dynamic_nest
                    B[i] = A[i] * 2.0

    return main


def test_mask_op_dynamic_source():
    # the dynamic-extent nest is strided over the hi - lo threads of the condition
    src = tilelang.lower(mask_dyn_program(128, 256), target="hip").kernel_source
    assert "* 128)" in src and "- 128)" in src


@pytest.mark.parametrize("dev", GPU)
@pytest.mark.parametrize("lo,hi", [(0, 128), (64, 192)])
def test_mask_op_dynamic(dev, lo, hi):
    k = _compile(mask_dyn_program(lo, hi), dev, out_idx=[1])
    a = torch.randn(1000, device=dev)
    torch.testing.assert_close(k(a), a * 2)


# ---- test_tilelang_language_negative_index.py ---------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_negative_index(dev):

    @T.prim_func
    def main(A: T.Tensor((16, ), "float32"), B: T.Tensor((4, ), "float32")):
        with T.Kernel(1, threads=64):
            B[0] = A[-1]
            for i in T.serial(1, 4):
                B[i] = A[-i - 1]

    k = _compile(main, dev)
    A = torch.randn(16, device=dev)
    B = torch.zeros(4, device=dev)
    k(A, B)
    torch.testing.assert_close(B, A.flip(0)[:4])


# ---- test_tilelang_language_unroll.py ----------------------------------------------------


def test_unroll_step_and_factor():

    @T.prim_func
    def step(A: T.Tensor((16, 16), "float32")):
        with T.Kernel(1, threads=64):
            for i in T.unroll(0, 16, step=4):
                A[0, i] = 1.0

    @T.prim_func
    def factor(A: T.Tensor((16, 16), "float32")):
        with T.Kernel(1, threads=64):
            for i in T.unroll(0, 16, unroll_factor=4):
                A[0, i] = 1.0

    assert "#pragma unroll" in tilelang.compile(step, target="hip").get_kernel_source()
    assert "#pragma unroll 4" in tilelang.compile(factor, target="hip").get_kernel_source()
    for fn, cols in ((step, [0, 4, 8, 12]), (factor, list(range(16)))):
        A = torch.zeros(16, 16)
        tilelang.compile(fn, target="cpu")(A)
        ref = torch.zeros(16, 16)
        ref[0, cols] = 1.0
        torch.testing.assert_close(A, ref)


# ---- test_tilelang_language_vectorize.py ---------------------------------------------------


def vectorize_program(N, M, sa, sb):

    @T.prim_func
    def main(A: T.StridedTensor((N, M), (1, sa), "float32"), B: T.StridedTensor((N, M), (1, sb), "float32")):
        with T.Kernel(M // 128, threads=128) as bx:
            tx = T.get_thread_binding(0)
            col = bx * 128 + tx
            for row in T.vectorized(N):
                B[row, col] = A[row, col]

    return main


@pytest.mark.parametrize("dev", GPU)
@pytest.mark.parametrize("pad", [(0, 0), (2, 4), (4, 8), (8, 16)])
def test_vectorize_strided(dev, pad):
    N, M = 512, 256
    sa, sb = N + pad[0], N + pad[1]
    k = _compile(vectorize_program(N, M, sa, sb), dev)
    base_a = torch.randn(sa, M, device=dev)
    base_b = torch.zeros(sb, M, device=dev)
    a = torch.as_strided(base_a, (N, M), (1, sa))
    b = torch.as_strided(base_b, (N, M), (1, sb))
    k(a, b)
    torch.testing.assert_close(a, b, atol=0, rtol=0)


def test_vectorize_strided_width():
    # each access is vectorised to the width its own stride's alignment allows (the reference
    # takes the common width of both: float4 / float2); B's stride 516 keeps 16-byte stores
    # even when A's stride 514 only allows scalar loads
    for pad, ins in (((0, 0), "global_load_dwordx4"), ((4, 8), "global_load_dwordx4"),
                     ((2, 4), "global_store_dwordx4")):
        isa = _isa(vectorize_program(512, 256, 512 + pad[0], 512 + pad[1]))
        assert ins in isa, pad


# ---- test_tilelang_language_composable_index.py -------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
@pytest.mark.parametrize("M,N,bm,bn,dtype", [(256, 256, 128, 128, "float16"), (128, 576, 32, 576, "float16"),
                                             (128, 576, 32, 576, "float32")])
def test_composable_index(dev, M, N, bm, bn, dtype):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M * N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            A_local = T.alloc_fragment([bm, bn], dtype)
            B_local = T.alloc_fragment([bm * bn], dtype)
            T.copy(A[by * bm, bx * bn], A_local)
            for i, j in T.Parallel(bm, bn):
                B_local[i * bn + j] = A_local[i, j]
            for i in T.Parallel(bm * bn):
                B[by * bm * N + bx * bn + i // bn * N + i % bn] = B_local[i]

    k = _compile(main, dev, out_idx=[1])
    a = torch.randn(M, N, device=dev).to(TD[dtype])
    assert torch.equal(k(a), a.flatten())


# ---- test_tilelang_language_annotate_safe_value.py ----------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_annotate_safe_value(dev):
    M = N = 256
    bm = bn = 128
    pad = 10

    @T.prim_func
    def main(A: T.Tensor((M, N), "float16"), B: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            A_shared = T.alloc_shared((bm, bn), "float16")
            T.annotate_safe_value({A: pad})
            for i, j in T.Parallel(bm, bn):
                A_shared[i, j] = A[by * bm + i - 10, bx * bn + j]
            for i, j in T.Parallel(bm, bn):
                B[by * bm + i, bx * bn + j] = A_shared[i, j]

    k = _compile(main, dev, out_idx=[1])
    a = torch.randn(M, N, device=dev).half()
    ref = torch.full_like(a, pad)
    ref[10:] = a[:-10]
    torch.testing.assert_close(k(a), ref)


# ---- test_tilelang_language_assume.py ----------------------------------------------------


def test_assume_removes_bounds_checks():
    N = T.dynamic("N")

    @T.prim_func
    def main(A: T.Tensor((N, ), "float32"), lo: T.int32, hi: T.int32):
        with T.Kernel(1, threads=64):
            for i in T.serial(hi - lo + 1):
                T.assume(lo + i >= 0 and lo + i < N)
                A[lo + i] = 0

    assert "if (" not in tilelang.compile(main, target="hip").get_kernel_source()
    A = torch.ones(16)
    tilelang.compile(main, target="cpu")(A, 3, 6)
    ref = torch.ones(16)
    ref[3:7] = 0
    torch.testing.assert_close(A, ref)


def test_assume_enables_vectorization():
    N = T.dynamic("N")

    @T.prim_func
    def main(A: T.Tensor((128, N), "float32"), B: T.Tensor((128, N), "float32")):
        with T.Kernel(1, threads=64):
            tid = T.get_thread_binding()
            base = tid * 4
            T.assume(N % 4 == 0)
            for i in T.vectorized(4):
                T.assume(base + i < N)
                B[tid, base + i] = A[tid, base + i]

    src = tilelang.compile(main, target="hip").get_kernel_source()
    assert "if (" not in src
    isa = tilelang.compile(main, target="hip").get_assembly()
    assert "global_load_dwordx4" in isa


# ---- test_tilelang_language_get_warp_info.py ----------------------------------------------


def warp_info_program(fn, n=256):

    @T.prim_func
    def main(A: T.Tensor((n, ), "int32")):
        with T.Kernel(1, threads=n):
            tx = T.get_thread_binding()
            A[tx] = fn()

    return main


@pytest.mark.parametrize("dev", GPU)
def test_get_warp_info(dev):
    ar = torch.arange(256, dtype=torch.int32)
    cases = [(T.get_lane_idx, ar % 64), (T.get_warp_idx_sync, ar // 64), (T.get_warp_idx, ar // 64),
             (T.get_warp_group_idx, ar // 256), (lambda: T.get_lane_idx(32), ar % 32),
             (lambda: T.get_warp_idx(32), ar // 32), (lambda: T.get_warp_group_idx(64, 2), ar // 128)]
    for fn, ref in cases:
        out = _compile(warp_info_program(fn), dev, out_idx=[-1])()
        assert torch.equal(out.cpu(), ref)


# ---- test_tilelang_language_parallel.py ---------------------------------------------------


@pytest.mark.parametrize("dev", DEVS)
def test_parallel_static_and_dynamic_extent(dev):

    @T.prim_func
    def static(A: T.Tensor((256, ), "float32"), B: T.Tensor((256, ), "float32")):
        with T.Kernel(1, threads=256):
            for i in T.Parallel(256):
                B[i] = A[i] + 1.0

    k = _compile(static, dev, out_idx=[1])
    a = torch.randn(256, device=dev)
    torch.testing.assert_close(k(a), a + 1)

    @T.prim_func
    def dynamic(A: T.Tensor((512, ), "float32"), B: T.Tensor((512, ), "float32"), valid_len: T.int32):
        with T.Kernel(1, threads=256):
            for i in T.Parallel(512):
                B[i] = 0.0
            span = T.min(valid_len, 512)
            for i in T.Parallel(span):
                B[i] = A[i] - 1.0

    k = _compile(dynamic, dev, out_idx=[1])
    a = torch.randn(512, device=dev)
    for n in (0, 13, 200, 600):
        ref = torch.zeros_like(a)
        c = min(n, 512)
        ref[:c] = a[:c] - 1.0
        torch.testing.assert_close(k(a, n), ref)


# ---- device_assert (reference language/builtin.py device_assert) -------------------------


def test_device_assert():

    @T.prim_func
    def main(A: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=64):
            for i in T.Parallel(64):
                T.device_assert(A[i] >= 0, "negative input")
                A[i] = A[i] * 2

    src = tilelang.compile(main, target="hip").get_kernel_source()
    assert "negative input" in src
    k = tilelang.compile(main, target="cpu")
    A = torch.rand(64)
    ref = A * 2
    k(A)
    torch.testing.assert_close(A, ref)


# ---- cross-wave reductions without ThreadSync (tl.disable_thread_storage_sync) ------------


def softmax_rows_program(M, N):
    """Row max then row sum of exp over rows that span all 4 waves: two cross-wave exchanges
    through the reduction workspace back to back."""

    @T.prim_func
    def main(A: T.Tensor((M, N), "float32"), B: T.Tensor((M, N), "float32")):
        with T.Kernel(1, threads=256):
            S_ = T.alloc_fragment((M, N), "float32")
            mx = T.alloc_fragment((M, ), "float32")
            sm = T.alloc_fragment((M, ), "float32")
            T.copy(A, S_)
            T.reduce_max(S_, mx, dim=1)
            for i, j in T.Parallel(M, N):
                S_[i, j] = T.exp(S_[i, j] - mx[i])
            T.reduce_sum(S_, sm, dim=1)
            for i, j in T.Parallel(M, N):
                S_[i, j] = S_[i, j] / sm[i]
            T.copy(S_, B)

    return main


def test_reduction_barriers_without_thread_sync():
    cfg = {"tl.disable_thread_storage_sync": True}
    with_ts = tilelang.lower(softmax_rows_program(4, 1024), target="hip").kernel_source
    without = tilelang.lower(softmax_rows_program(4, 1024), target="hip", pass_configs=cfg).kernel_source
    # the reductions keep their leading / trailing barriers themselves when ThreadSync is off
    assert without.count("__syncthreads()") >= with_ts.count("__syncthreads()")


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{}, {"tl.disable_thread_storage_sync": True}])
def test_reduction_barriers_without_thread_sync_gpu(cfg):
    k = tilelang.compile(softmax_rows_program(4, 1024), target="hip", pass_configs=cfg)
    A = torch.randn(4, 1024, device="cuda")
    B = torch.zeros_like(A)
    k(A, B)
    torch.testing.assert_close(B, torch.softmax(A, 1), rtol=1e-4, atol=1e-6)
