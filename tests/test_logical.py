"""T.any_of / T.all_of over global, shared and local regions (block-sparse GEMM guard)."""
import pytest
import torch

import tilelang
import tilelang.language as T


def sparse_gemm(M, N, K, bm, bn, bk, cdim, where, op):
    pick = T.any_of if op == "any" else T.all_of

    @T.prim_func
    def main(A: T.Tensor((M, K), "float16"), B: T.Tensor((K, N), "float16"),
             Mask: T.Tensor((M // bm, N // bn, K // bk, cdim), "bool"), C: T.Tensor((M, N), "float32")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=128) as (bx, by):
            A_s = T.alloc_shared((bm, bk), "float16")
            B_s = T.alloc_shared((bk, bn), "float16")
            C_l = T.alloc_fragment((bm, bn), "float32")
            m_s = T.alloc_shared((cdim, ), "bool")
            m_l = T.alloc_local((cdim, ), "bool")
            T.clear(C_l)
            for k in T.Pipelined(K // bk, num_stages=2):
                if where == "shared":
                    for i in T.serial(cdim):
                        m_s[i] = Mask[by, bx, k, i]
                    cond = pick(m_s)
                elif where == "local":
                    for i in T.serial(cdim):
                        m_l[i] = Mask[by, bx, k, i]
                    cond = pick(m_l)
                else:
                    cond = pick(Mask[by, bx, k, :])
                if cond:
                    T.copy(A[by * bm, k * bk], A_s)
                    T.copy(B[k * bk, bx * bn], B_s)
                    T.gemm(A_s, B_s, C_l)
            T.copy(C_l, C[by * bm, bx * bn])

    return main


def _ref(a, b, mask, bm, bn, bk, op):
    M, N, K = a.shape[0], b.shape[1], a.shape[1]
    sel = mask.any(-1) if op == "any" else mask.all(-1)
    c = torch.zeros(M, N)
    for i in range(M // bm):
        for j in range(N // bn):
            for k in range(K // bk):
                if sel[i, j, k]:
                    c[i * bm:(i + 1) * bm, j * bn:(j + 1) * bn] += \
                        a[i * bm:(i + 1) * bm, k * bk:(k + 1) * bk].float() @ \
                        b[k * bk:(k + 1) * bk, j * bn:(j + 1) * bn].float()
    return c


def _run(where, op, device):
    M = N = K = 128
    bm = bn = bk = 32
    cdim = 2
    k = tilelang.compile(sparse_gemm(M, N, K, bm, bn, bk, cdim, where, op), target="cpu" if device == "cpu" else "hip")
    torch.manual_seed(0)
    a = torch.randn(M, K, dtype=torch.float16)
    b = torch.randn(K, N, dtype=torch.float16)
    mask = torch.rand(M // bm, N // bn, K // bk, cdim) > 0.6
    c = torch.zeros(M, N)
    if device == "cuda":
        a, b, mask, c = a.cuda(), b.cuda(), mask.cuda(), c.cuda()
    k(a, b, mask, c)
    torch.testing.assert_close(c.cpu(), _ref(a.cpu(), b.cpu(), mask.cpu(), bm, bn, bk, op), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("where", ["global", "shared", "local"])
@pytest.mark.parametrize("op", ["any", "all"])
def test_any_all_cpu(where, op):
    _run(where, op, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["global", "shared", "local"])
@pytest.mark.parametrize("op", ["any", "all"])
def test_any_all_gpu(where, op):
    _run(where, op, "cuda")


def test_any_of_rejects_multi_dim_region():
    buf = T.Tensor((4, 4), "bool").make_buffer("m")
    with pytest.raises(ValueError):
        T.any_of(buf)
