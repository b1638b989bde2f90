"""Atomics: ports of the reference's testing/python/language/test_tilelang_language_atomic_add.py
(atomic_add / tile atomic_add / max / min / load+store / memory_order / different orders /
addx2 / addx4 / return_prev), plus the gfx950-specific checks: 16-bit scalar adds are one
``global_atomic_pk_add`` (no CAS loop), tile-level 16-bit atomics are pair-vectorised
(AtomicAddVectorize), and memory orders reach the ISA (release = ``buffer_wbl2`` before the op).

Every program runs on the CPU target (numerics vs torch) and compiles for gfx950; the ``gpu``
tests run the same programs on an MI355X against an fp32 torch reference.  Blocks use 64 threads
(one wave) where the reference uses 32.
"""
import re

import pytest
import torch

import tilelang
import tilelang.language as T

TH = 64
DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


def atomic_add_program(K, M, N, block_M, block_N, dtype="float32", memory_order=None):

    @T.prim_func
    def main(A: T.Tensor((K, M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), K, threads=TH) as (bx, by, bz):
            A_shared = T.alloc_shared((block_M, block_N), dtype)
            T.copy(A[bz, bx * block_M:(bx + 1) * block_M, by * block_N:(by + 1) * block_N], A_shared)
            for i, j in T.Parallel(block_M, block_N):
                T.atomic_add(B[bx * block_M + i, by * block_N + j], A_shared[i, j], memory_order=memory_order)

    return main


def tile_atomic_add_program(K, M, N, block_M, block_N, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((K, M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), K, threads=TH) as (bx, by, bz):
            A_shared = T.alloc_shared((block_M, block_N), dtype)
            T.copy(A[bz, bx * block_M:(bx + 1) * block_M, by * block_N:(by + 1) * block_N], A_shared)
            T.atomic_add(B[bx * block_M, by * block_N], A_shared)

    return main


def atomic_minmax_program(kind, K, M, N, block_M, block_N, dtype="float32"):
    fn = T.atomic_max if kind == "max" else T.atomic_min

    @T.prim_func
    def main(A: T.Tensor((K, M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), K, threads=TH) as (bx, by, bz):
            A_shared = T.alloc_shared((block_M, block_N), dtype)
            T.copy(A[bz, bx * block_M:(bx + 1) * block_M, by * block_N:(by + 1) * block_N], A_shared)
            for i, j in T.Parallel(block_M, block_N):
                fn(B[bx * block_M + i, by * block_N + j], A_shared[i, j])

    return main


def atomic_load_store_program(M, N, block_M, block_N, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), threads=TH) as (bx, by):
            for i, j in T.Parallel(block_M, block_N):
                idx_i = bx * block_M + i
                idx_j = by * block_N + j
                if idx_i < M and idx_j < N:
                    val = T.atomic_load(A[idx_i, idx_j])
                    T.atomic_store(B[idx_i, idx_j], val)

    return main


def different_orders_program(M, N, block_M, block_N, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype), C: T.Tensor((M, N), dtype),
             D: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), threads=TH) as (bx, by):
            for i, j in T.Parallel(block_M, block_N):
                idx_i = bx * block_M + i
                idx_j = by * block_N + j
                if idx_i < M and idx_j < N:
                    val = A[idx_i, idx_j]
                    T.atomic_add(B[idx_i, idx_j], val, memory_order="release")
                    T.atomic_max(C[idx_i, idx_j], val, memory_order="relaxed")
                    T.atomic_min(D[idx_i, idx_j], val, memory_order="relaxed")

    return main


def addx2_program(M, N, block_M, block_N, dtype="float16"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), threads=TH) as (bx, by):
            for i, j in T.Parallel(block_M, block_N // 2):
                idx_i = bx * block_M + i
                idx_j = by * block_N + j * 2
                T.atomic_addx2(B[idx_i, idx_j], A[idx_i, idx_j])

    return main


def addx4_program(M, N, block_M, block_N, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), threads=TH) as (bx, by):
            for i, j in T.Parallel(block_M, block_N // 4):
                idx_i = bx * block_M + i
                idx_j = by * block_N + j * 4
                T.atomic_addx4(B[idx_i, idx_j], A[idx_i, idx_j])

    return main


def return_prev_program(M, N, block_M, block_N, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype), old_vals: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), threads=TH) as (bx, by):
            for i, j in T.Parallel(block_M, block_N):
                idx_i = bx * block_M + i
                idx_j = by * block_N + j
                if idx_i < M and idx_j < N:
                    old_vals[idx_i, idx_j] = T.atomic_add(B[idx_i, idx_j], A[idx_i, idx_j], return_prev=True)

    return main


def lds_histogram_program(n, bins, dtype="float16"):
    """Shared-memory 16-bit atomics (``ds_pk_add_f16``): per-block histogram of weights."""

    @T.prim_func
    def main(Idx: T.Tensor((n, ), "int32"), W: T.Tensor((n, ), dtype), H: T.Tensor((bins, ), "float32")):
        with T.Kernel(1, threads=TH):
            hs = T.alloc_shared((bins, ), dtype)
            T.clear(hs)
            for i in T.Parallel(n):
                T.atomic_add(hs[Idx[i]], W[i])
            T.copy(hs, H)

    return main


# ---- helpers -----------------------------------------------------------------------------


def _tol(dtype):
    return dict(atol=1e-3, rtol=1e-3) if dtype == "float32" else dict(atol=2e-2, rtol=2e-2)


def _run_add(prog, dev, K=4, M=64, N=64, bm=16, bn=16, dtype="float32", **kw):
    k = tilelang.compile(prog(K, M, N, bm, bn, dtype, **kw), target="cpu" if dev == "cpu" else "hip")
    # 16-bit: small integers are exact in f16 / bf16 (sums of up to K of them), so any order of
    # the atomic adds gives the same bits
    A = (torch.randint(-4, 5, (K, M, N)).float() if dtype != "float32" else torch.randn(K, M, N)).to(DT[dtype])
    A = A.to(dev)
    B = torch.zeros(M, N, dtype=DT[dtype], device=dev)
    k(A, B)
    torch.testing.assert_close(B.float(), A.float().sum(0), **_tol(dtype))
    return k


def _isa(k):
    return k.get_assembly()


# ---- CPU target: numerics of every form -------------------------------------------------


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_atomic_add_cpu(dtype):
    _run_add(atomic_add_program, "cpu", dtype=dtype)


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_tile_atomic_add_cpu(dtype):
    _run_add(tile_atomic_add_program, "cpu", dtype=dtype)


def test_atomic_memory_order_cpu():
    _run_add(atomic_add_program, "cpu", memory_order="relaxed")
    _run_add(atomic_add_program, "cpu", memory_order="seq_cst")


@pytest.mark.parametrize("kind", ["max", "min"])
def test_atomic_max_min_cpu(kind):
    K, M, N = 4, 64, 64
    k = tilelang.compile(atomic_minmax_program(kind, K, M, N, 16, 16), target="cpu")
    A = torch.randn(K, M, N)
    B = torch.zeros(M, N) if kind == "max" else torch.full((M, N), float("inf"))
    ref = torch.maximum(B, A.amax(0)) if kind == "max" else torch.minimum(B, A.amin(0))
    k(A, B)
    torch.testing.assert_close(B, ref)


def test_atomic_load_store_cpu():
    k = tilelang.compile(atomic_load_store_program(64, 64, 16, 16), target="cpu")
    A = torch.randn(64, 64)
    B = torch.zeros(64, 64)
    k(A, B)
    torch.testing.assert_close(B, A)


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_atomic_different_memory_orders_cpu(dtype):
    _check_orders("cpu", dtype)


def _check_orders(dev, dtype):
    M = N = 32
    k = tilelang.compile(different_orders_program(M, N, 8, 8, dtype), target="cpu" if dev == "cpu" else "hip")
    t = DT[dtype]
    A = torch.randn(M, N).to(t).to(dev)
    B = torch.zeros(M, N, dtype=t, device=dev)
    C = torch.zeros(M, N, dtype=t, device=dev)
    D = torch.full((M, N), float("inf"), dtype=t, device=dev)
    k(A, B, C, D)
    torch.testing.assert_close(B, A, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(C, torch.maximum(torch.zeros_like(A), A))
    torch.testing.assert_close(D, torch.minimum(torch.full_like(A, float("inf")), A))


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_atomic_addx2_cpu(dtype):
    _check_addx(addx2_program, "cpu", dtype)


def test_atomic_addx4_cpu():
    _check_addx(addx4_program, "cpu", "float32")


def _check_addx(prog, dev, dtype):
    M, N = 32, 64
    k = tilelang.compile(prog(M, N, 8, 16, dtype), target="cpu" if dev == "cpu" else "hip")
    t = DT[dtype]
    A = torch.randn(M, N).to(t).to(dev)
    B0 = torch.randn(M, N).to(t).to(dev)
    B = B0.clone()
    k(A, B)
    # every element is added exactly once (the round-4 alias dropped the odd columns)
    torch.testing.assert_close(B.float(), (B0.float() + A.float()).to(t).float(), **_tol(dtype))


def test_atomic_return_prev_cpu():
    _check_return_prev("cpu")


def _check_return_prev(dev):
    M = N = 32
    k = tilelang.compile(return_prev_program(M, N, 8, 8), target="cpu" if dev == "cpu" else "hip")
    A = torch.ones(M, N, device=dev) * 5.0
    B = torch.ones(M, N, device=dev) * 2.0
    old = torch.zeros(M, N, device=dev)
    B0 = B.clone()
    k(A, B, old)
    torch.testing.assert_close(old, B0)
    torch.testing.assert_close(B, B0 + A)


def test_lds_histogram_cpu():
    _check_hist("cpu")


def _check_hist(dev):
    n, bins = 512, 32
    k = tilelang.compile(lds_histogram_program(n, bins), target="cpu" if dev == "cpu" else "hip")
    idx = torch.randint(0, bins, (n, ), dtype=torch.int32)
    w = torch.randint(-3, 4, (n, )).to(torch.float16)
    ref = torch.zeros(bins).index_add_(0, idx.long(), w.float())
    H = torch.zeros(bins, device=dev)
    k(idx.to(dev), w.to(dev), H)
    torch.testing.assert_close(H.cpu(), ref)


def test_bad_memory_order():
    with pytest.raises(KeyError):
        tilelang.compile(atomic_add_program(1, 16, 16, 16, 16, memory_order="strong"), target="cpu")


# ---- gfx950 code: the instructions the lowering promises ----------------------------------


def test_16bit_scalar_add_is_packed_atomic_hip():
    for dt, ins in (("float16", "global_atomic_pk_add_f16"), ("bfloat16", "global_atomic_pk_add_bf16")):
        k = tilelang.compile(atomic_add_program(4, 64, 64, 16, 16, dt), target="hip")
        isa = _isa(k)
        assert ins in isa, dt
        assert "global_atomic_cmpswap" not in isa, dt  # no CAS loop


def test_tile_atomic_vectorized_hip():
    # tile-level 16-bit atomics from an LDS tile: pairs of columns per packed atomic
    k = tilelang.compile(tile_atomic_add_program(4, 64, 64, 16, 16, "float16"), target="hip")
    src = k.get_kernel_source()
    assert "tl::atomic_addx2(" in src
    assert "tl::atomic_add(" not in src
    assert "global_atomic_pk_add_f16" in _isa(k)


def test_splitk_fp16_output_uses_pk_add_hip():
    from example_tilelang_gemm_splitk import matmul_splitk
    f = matmul_splitk.get_tir(1024, 1024, 8192, out_dtype="float16")
    k = tilelang.compile(f, target="hip")
    src = k.get_kernel_source()
    n2 = src.count("tl::atomic_addx2(")
    assert n2 > 0 and src.count("tl::atomic_add(") == 0
    isa = _isa(k)
    assert "global_atomic_pk_add_f16" in isa and "global_atomic_cmpswap" not in isa


def test_splitk_fp32_atomics_staged_hip():
    """fp32 tile atomics from an MFMA accumulator go through a row-padded LDS tile so each wave
    instruction adds 64 consecutive floats (lower_tile_op.lower_atomic_staged); a tile over the LDS
    budget keeps the per-element form."""
    from example_tilelang_gemm_splitk import matmul_splitk
    src = tilelang.lower(matmul_splitk.get_tir(1024, 1024, 8192, split_k=8), target="hip").kernel_source
    assert re.search(r"tl::atomic_add\(&C\[[^;]*\], red_ws\d+\[", src), "atomics read the LDS tile"
    assert "* 132)" in src  # 128 floats + 4 of padding per row
    big = tilelang.lower(matmul_splitk.get_tir(1024, 1024, 8192, block_M=256, block_N=256, block_K=64, threads=512,
                                               split_k=8), target="hip").kernel_source
    assert "red_ws" not in big and "tl::atomic_add(&C[" in big


def test_f32_atomic_nest_one_element_per_lane_hip():
    """An element-form f32 atomic nest maps one element per lane (no vector f32 atomic exists, so a
    4-wide mapping would only spread each wave instruction over every fourth float)."""
    src = tilelang.lower(tile_atomic_add_program(4, 64, 64, 16, 16, "float32"), target="hip").kernel_source
    adds = [ln for ln in src.splitlines() if "tl::atomic_add(" in ln]
    assert len(adds) == 16 * 16 // TH and "tl::atomic_addx" not in src
    assert all("tid_ * 4" not in ln for ln in adds)


def test_addx2_addx4_codegen_hip():
    k = tilelang.compile(addx2_program(32, 64, 8, 16, "bfloat16"), target="hip")
    assert "global_atomic_pk_add_bf16" in _isa(k)
    k = tilelang.compile(addx4_program(32, 64, 8, 16, "float32"), target="hip")
    isa = _isa(k)
    assert len(re.findall(r"global_atomic_add_f32", isa)) >= 4


def test_memory_order_reaches_isa_hip():
    rel = _isa(tilelang.compile(atomic_add_program(4, 64, 64, 16, 16, memory_order="release"), target="hip"))
    rlx = _isa(tilelang.compile(atomic_add_program(4, 64, 64, 16, 16, memory_order="relaxed"), target="hip"))
    assert "buffer_wbl2" in rel and "buffer_wbl2" not in rlx
    sc = _isa(tilelang.compile(atomic_add_program(4, 64, 64, 16, 16, "float16", memory_order="seq_cst"),
                               target="hip"))
    assert "buffer_wbl2" in sc and "buffer_inv" in sc and "global_atomic_pk_add_f16" in sc


def test_lds_16bit_atomic_is_ds_pk_add_hip():
    k = tilelang.compile(lds_histogram_program(512, 32), target="hip")
    assert "ds_pk_add_f16" in _isa(k)


# ---- on the MI355X ------------------------------------------------------------------------


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_atomic_add_gpu(dtype):
    _run_add(atomic_add_program, "cuda", K=8, M=128, N=128, bm=32, bn=32, dtype=dtype)
    _run_add(tile_atomic_add_program, "cuda", K=8, M=128, N=128, bm=32, bn=32, dtype=dtype)


@pytest.mark.gpu
def test_atomic_memory_order_gpu():
    _run_add(atomic_add_program, "cuda", memory_order="relaxed")
    _run_add(atomic_add_program, "cuda", dtype="float16", memory_order="acq_rel")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["max", "min"])
@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_atomic_max_min_gpu(kind, dtype):
    K, M, N = 4, 64, 64
    k = tilelang.compile(atomic_minmax_program(kind, K, M, N, 16, 16, dtype), target="hip")
    t = DT[dtype]
    A = torch.randn(K, M, N, device="cuda").to(t)
    B = torch.zeros(M, N, device="cuda", dtype=t) if kind == "max" else torch.full((M, N), float("inf"),
                                                                                    device="cuda", dtype=t)
    ref = torch.maximum(B, A.amax(0)) if kind == "max" else torch.minimum(B, A.amin(0))
    k(A, B)
    torch.testing.assert_close(B, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_atomic_load_store_gpu(dtype):
    k = tilelang.compile(atomic_load_store_program(64, 64, 16, 16, dtype), target="hip")
    A = torch.randn(64, 64, device="cuda").to(DT[dtype])
    B = torch.zeros(64, 64, device="cuda", dtype=DT[dtype])
    k(A, B)
    torch.testing.assert_close(B, A)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_atomic_different_memory_orders_gpu(dtype):
    _check_orders("cuda", dtype)


@pytest.mark.gpu
def test_atomic_addx2_addx4_gpu():
    _check_addx(addx2_program, "cuda", "float16")
    _check_addx(addx2_program, "cuda", "bfloat16")
    _check_addx(addx4_program, "cuda", "float32")


@pytest.mark.gpu
def test_atomic_return_prev_gpu():
    _check_return_prev("cuda")


@pytest.mark.gpu
def test_lds_histogram_gpu():
    _check_hist("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(1024, 1024), (1000, 904)])
def test_splitk_fp32_staged_atomics_gpu(M, N):
    from example_tilelang_gemm_splitk import matmul_splitk
    K = 4096
    k = matmul_splitk(M, N, K, split_k=8, block_K=64)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = torch.zeros(M, N, device="cuda")
    k(a, b, c)
    torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-3, atol=2e-2)


@pytest.mark.gpu
def test_splitk_fp16_output_gpu():
    from example_tilelang_gemm_splitk import matmul_splitk
    M, N, K = 512, 512, 4096
    k = matmul_splitk(M, N, K, split_k=4, out_dtype="float16")
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = torch.zeros(M, N, device="cuda", dtype=torch.float16)
    k(a, b, c)
    torch.testing.assert_close(c.float(), a.float() @ b.float(), rtol=2e-2, atol=1.0)
