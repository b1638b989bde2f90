"""T.gemm on the other gfx950 matrix-core forms: 32x32x16 f16/bf16, int8 (16x16x64 / 32x32x32,
int32 accumulate) and fp32 (16x16x4), against fp32 / int64 PyTorch references."""
import pytest
import torch

import tilelang
import tilelang.language as T


def gemm_kernel(M, N, K, bm, bn, bk, threads, dtype, accum, out_dtype, trans_A=False, trans_B=False,
                mfma_shape=None, stages=2):
    A_shape = (K, M) if trans_A else (M, K)
    B_shape = (N, K) if trans_B else (K, N)
    As = (bk, bm) if trans_A else (bm, bk)
    Bs = (bn, bk) if trans_B else (bk, bn)

    @T.prim_func
    def main(A: T.Tensor(A_shape, dtype), B: T.Tensor(B_shape, dtype), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=threads) as (bx, by):
            A_s = T.alloc_shared(As, dtype)
            B_s = T.alloc_shared(Bs, dtype)
            C_l = T.alloc_fragment((bm, bn), accum)
            T.clear(C_l)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=stages):
                if trans_A:
                    T.copy(A[k * bk, by * bm], A_s)
                else:
                    T.copy(A[by * bm, k * bk], A_s)
                if trans_B:
                    T.copy(B[bx * bn, k * bk], B_s)
                else:
                    T.copy(B[k * bk, bx * bn], B_s)
                T.gemm(A_s, B_s, C_l, transpose_A=trans_A, transpose_B=trans_B, mfma_shape=mfma_shape)
            T.copy(C_l, C[by * bm, bx * bn])

    return main


def _ref(a, b, ta, tb):
    a = a.t() if ta else a
    b = b.t() if tb else b
    if a.dtype == torch.int8:  # exact in float64 (|sum| < 2^53); integer matmul has no GPU kernel
        return (a.double() @ b.double()).long()
    return a.float() @ b.float()


CASES = [
    # name, dtype, accum, out, ta, tb, shape, (bm, bn, bk, threads)
    ("bf16_32x32", "bfloat16", "float32", "float32", False, False, "32x32", (128, 128, 64, 256)),
    ("f16_32x32_tb", "float16", "float32", "float32", False, True, "32x32", (128, 128, 64, 256)),
    ("bf16_32x32_ta", "bfloat16", "float32", "float32", True, False, "32x32", (128, 128, 32, 256)),
    ("i8_16x16", "int8", "int32", "int32", False, True, None, (128, 128, 64, 256)),
    ("i8_32x32", "int8", "int32", "int32", False, True, "32x32", (128, 128, 64, 256)),
    ("f32_16x16", "float32", "float32", "float32", False, False, None, (64, 64, 32, 256)),
    ("f32_16x16_tatb", "float32", "float32", "float32", True, True, None, (64, 64, 32, 256)),
    # fp8 with B [K, N] (N contiguous): ds_read_b64_tr_b8 transposed operand reads, on the scaled
    # 16x16x128 MFMA (K % 128 == 0) and on the 16x16x32 fp8 MFMA
    ("f8_trb_k128", "float8_e4m3fn", "float32", "float32", False, False, None, (64, 128, 128, 256)),
    ("f8_trb_k32", "float8_e4m3fn", "float32", "float32", False, False, None, (64, 128, 64, 256)),
    ("f8_tb_k128", "float8_e4m3fn", "float32", "float32", False, True, None, (64, 128, 128, 256)),
]


def _inputs(dtype, ta, tb, M, N, K, device):
    ash = (K, M) if ta else (M, K)
    bsh = (N, K) if tb else (K, N)
    if dtype == "int8":
        return (torch.randint(-128, 128, ash, dtype=torch.int8, device=device),
                torch.randint(-128, 128, bsh, dtype=torch.int8, device=device))
    if dtype.startswith("float8"):  # exactly representable small integers: an exact check
        return (torch.randint(-4, 5, ash, device=device).float().to(getattr(torch, dtype)),
                torch.randint(-4, 5, bsh, device=device).float().to(getattr(torch, dtype)))
    td = getattr(torch, dtype)
    return torch.randn(ash, device=device).to(td), torch.randn(bsh, device=device).to(td)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_mfma_form_cpu_and_codegen(case):
    name, dt, acc, out, ta, tb, shape, (bm, bn, bk, th) = case
    M, N, K = 128, 128, 256
    f = gemm_kernel(M, N, K, bm, bn, bk, th, dt, acc, out, ta, tb, shape)
    kh = tilelang.compile(f, target="hip")
    src = kh.get_kernel_source()
    expect = {"bf16_32x32": "gemm_ss_32", "f16_32x32_tb": "gemm_ss_32", "bf16_32x32_ta": "gemm_ss_32",
              "i8_16x16": "gemm_ss_i8<16", "i8_32x32": "gemm_ss_i8<32", "f32_16x16": "gemm_ss_f32",
              "f32_16x16_tatb": "gemm_ss_f32", "f8_trb_k128": "u, false>", "f8_trb_k32": "u, false>",
              "f8_tb_k128": "u, true>"}[name]
    assert expect in src and len(kh.code[0]) > 0
    kc = tilelang.compile(f, target="cpu")
    a, b = _inputs(dt, ta, tb, M, N, K, "cpu")
    c = torch.zeros(M, N, dtype=getattr(torch, out))
    kc(a, b, c)
    ref = _ref(a, b, ta, tb)
    if dt == "int8":
        assert torch.equal(c.long(), ref)
    else:
        torch.testing.assert_close(c, ref, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_mfma_form_gpu(case):
    name, dt, acc, out, ta, tb, shape, (bm, bn, bk, th) = case
    M, N, K = 256, 256, 512
    k = tilelang.compile(gemm_kernel(M, N, K, bm, bn, bk, th, dt, acc, out, ta, tb, shape), target="hip")
    a, b = _inputs(dt, ta, tb, M, N, K, "cuda")
    c = torch.zeros(M, N, dtype=getattr(torch, out), device="cuda")
    k(a, b, c)
    ref = _ref(a, b, ta, tb)
    if dt == "int8":
        assert torch.equal(c.long().cpu(), ref.cpu())
    elif dt == "float32":
        torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-3)
    else:
        torch.testing.assert_close(c, ref, rtol=1e-2, atol=1e-2)
