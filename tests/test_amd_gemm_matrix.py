"""The reference's AMD GEMM test matrix (testing/python/amd/test_tilelang_test_amd.py:100-125 and its
commented-out ``gemm_rs`` half) on gfx950: fp16 / bf16 inputs, fp32 or bf16 output, all four
transpose combinations, ``k_pack`` in {1, 2}, operand A from LDS (ss) or from registers (rs), on
both MFMA shapes (16x16x32 and 32x32x16).  Every case: the CPU target against fp32 torch and a gfx950
compile here; on an MI355X (``gpu`` marker) the HIP kernel against fp32 torch at 1024^3 as the
reference runs it.  Also: ragged M/N/K on the 256x256 quad-loop tile."""
import itertools

import pytest
import torch

import tilelang
import tilelang.language as T


def matmul(M, N, K, bm, bn, bk, ta, tb, in_dtype, out_dtype, accum, stages, threads, k_pack=1, rs=False,
           mfma_shape=None):
    A_shape = (K, M) if ta else (M, K)
    B_shape = (N, K) if tb else (K, N)
    As = (bk, bm) if ta else (bm, bk)
    Bs = (bn, bk) if tb else (bk, bn)
    vec = 4 * k_pack

    @T.prim_func
    def main(A: T.Tensor(A_shape, in_dtype), B: T.Tensor(B_shape, in_dtype), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=threads) as (bx, by):
            A_s = T.alloc_shared(As, in_dtype)
            B_s = T.alloc_shared(Bs, in_dtype)
            C_l = T.alloc_fragment((bm, bn), accum)
            if rs:
                A_l = T.alloc_fragment(As, in_dtype)
            T.clear(C_l)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=stages):
                if ta:
                    T.copy(A[k * bk, by * bm], A_s, coalesced_width=vec)
                else:
                    T.copy(A[by * bm, k * bk], A_s, coalesced_width=vec)
                if tb:
                    T.copy(B[bx * bn, k * bk], B_s, coalesced_width=vec)
                else:
                    T.copy(B[k * bk, bx * bn], B_s, coalesced_width=vec)
                if rs:
                    T.copy(A_s, A_l)
                    T.gemm(A_l, B_s, C_l, ta, tb, k_pack=k_pack, mfma_shape=mfma_shape)
                else:
                    T.gemm(A_s, B_s, C_l, ta, tb, k_pack=k_pack, mfma_shape=mfma_shape)
            T.copy(C_l, C[by * bm, bx * bn])

    return main


def _ref(a, b, ta, tb):
    a = a.t() if ta else a
    b = b.t() if tb else b
    return a.float() @ b.float()


# (in, out) dtype pairs of the reference's three test functions
DTYPES = [("float16", "float32"), ("bfloat16", "float32"), ("bfloat16", "bfloat16")]
TRANS = list(itertools.product([False, True], [False, True]))
CASES = []
for (ind, outd), (ta, tb), shape in itertools.product(DTYPES, TRANS, [None, "32x32"]):
    CASES.append((ind, outd, ta, tb, 1, False, shape))
for (ind, outd), shape in itertools.product(DTYPES, [None, "32x32"]):
    CASES.append((ind, outd, False, True, 2, False, shape))  # the reference's k_pack=2 row (NT)
# gemm_rs: A in registers (the reference keeps these commented out; they run here)
for (ind, outd), (ta, tb), shape in itertools.product(DTYPES[:2], TRANS, [None, "32x32"]):
    CASES.append((ind, outd, ta, tb, 1, True, shape))
CASES.append(("float16", "float32", False, True, 2, True, None))


def _id(c):
    ind, outd, ta, tb, kp, rs, shape = c
    return (f"{ind[:4]}-{outd[:4]}-{'T' if ta else 'N'}{'T' if tb else 'N'}-kp{kp}-{'rs' if rs else 'ss'}-"
            f"{shape or '16x16'}")


def _run(case, M, N, K, device):
    ind, outd, ta, tb, kp, rs, shape = case
    f = matmul(M, N, K, 128, 128, 32 * kp, ta, tb, ind, outd, "float32", 2, 128, k_pack=kp, rs=rs,
               mfma_shape=shape)
    k = tilelang.compile(f, out_idx=[2], target="cpu" if device == "cpu" else "hip")
    td = getattr(torch, ind)
    a = torch.randn((K, M) if ta else (M, K), device=device).to(td)
    b = torch.randn((N, K) if tb else (K, N), device=device).to(td)
    c = k(a, b)
    ref = _ref(a, b, ta, tb)
    tol = 2e-2 if outd == "bfloat16" else 1e-2
    torch.testing.assert_close(c.float(), ref.to(getattr(torch, outd)).float(), rtol=tol, atol=tol * 8)
    return k


@pytest.mark.parametrize("case", CASES, ids=[_id(c) for c in CASES])
def test_amd_gemm_matrix_cpu(case):
    _run(case, 128, 256, 128, "cpu")
    ind, outd, ta, tb, kp, rs, shape = case
    f = matmul(256, 256, 256, 128, 128, 32 * kp, ta, tb, ind, outd, "float32", 2, 128, k_pack=kp, rs=rs,
               mfma_shape=shape)
    kh = tilelang.compile(f, out_idx=[2], target="hip")
    assert len(kh.code[0]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[_id(c) for c in CASES])
def test_amd_gemm_matrix_gpu(case):
    _run(case, 1024, 1024, 1024, "cuda")


# ---- ragged shapes on the 256x256x64 / 512-thread tile (the quad-loop configuration) ----------

RAGGED = [(4000, 4096, 4096), (4096, 4000, 4096), (4096, 4096, 4000), (1000, 1000, 1000), (4096, 4096, 4096),
          (4000, 4000, 4000), (300, 520, 72), (257, 255, 8)]


def _quad_kernel(M, N, K, target):
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "gemm"))
    from example_gemm import matmul as mm
    f = mm.get_tir(M, N, K, 256, 256, 64, 512, 2, "float16", trans_B=True, staged_epilogue=True)
    return tilelang.compile(f, out_idx=[-1], target=target)


@pytest.mark.parametrize("M,N,K,mode", [(4096, 4096, 4096, "<half_t, false, 0>"),
                                         (4000, 4096, 4096, "<half_t, true, 0>"),
                                         (4096, 4000, 4096, "<half_t, false, 0, true, false>"),
                                         (4096, 4096, 4000, "<half_t, false, 0, false, true>"),
                                         (1000, 1000, 1000, "<half_t, true, 0, true, true>")])
def test_quad_tile_ragged_selects_quad_loop(M, N, K, mode):
    """Ragged M (range-checked A rows), N (range-checked B rows) and K (zero-filled last K tile)
    all run the tl::gemm_quad_nt_x main loop, not the generic pipeline."""
    src = _quad_kernel(M, N, K, "hip").get_kernel_source()
    assert "tl::gemm_quad_nt_x" + mode in src


@pytest.mark.parametrize("M,N,K", [(200, 264, 136), (256, 256, 200)])
def test_quad_tile_ragged_cpu(M, N, K):
    k = _quad_kernel(M, N, K, "cpu")
    a = torch.randn(M, K).half()
    b = torch.randn(N, K).half()
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float().t(), rtol=2e-2, atol=2e-1)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", RAGGED)
def test_quad_tile_ragged_gpu(M, N, K):
    k = _quad_kernel(M, N, K, "hip")
    a = torch.randn(M, K, device="cuda").half()
    b = torch.randn(N, K, device="cuda").half()
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float().t(), rtol=2e-2, atol=2e-1)
