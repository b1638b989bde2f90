"""``tilelang.lazy_jit`` walkthrough (reference: examples/lazy_jit/lazyjit.en.ipynb, as a script).

``@tilelang.lazy_jit`` specialises a kernel from the *call's* arguments: ``T.Tensor[[dims], dtype]``
annotations give the dims (``T.dyn`` = a runtime extent, ``int`` = bound from the first call and
part of the specialisation key), ``Any`` dtypes come from the tensors, ``T.empty`` allocates the
outputs, and every new (shape, dtype) combination compiles once and is cached."""
from typing import Any

import tilelang
import tilelang.language as T


def make(target="auto"):

    @tilelang.lazy_jit(target=target)
    def gemm(A: T.Tensor[[T.dyn, int], Any], B: T.Tensor[[int, int], Any], bm: int = 64, bn: int = 64,
             bk: int = 32):
        M, K = A.shape
        K, N = B.shape
        C = T.empty(M, N, dtype=T.float32)
        with T.Kernel(T.ceildiv(M, bm), T.ceildiv(N, bn), threads=128) as (bx, by):
            A_s = T.alloc_shared((bm, bk), A.dtype)
            B_s = T.alloc_shared((bk, bn), A.dtype)
            C_l = T.alloc_fragment((bm, bn), "float32")
            T.clear(C_l)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=2):
                T.copy(A[bx * bm, k * bk], A_s)
                T.copy(B[k * bk, by * bn], B_s)
                T.gemm(A_s, B_s, C_l)
            T.copy(C_l, C[bx * bm, by * bn])
        return C

    return gemm


def main(device="cuda"):
    import torch
    gemm = make("cpu" if device == "cpu" else "auto")
    for m in (128, 256, 192):  # M is T.dyn: the same specialisation serves all three
        a = torch.randn(m, 128, device=device, dtype=torch.float16)
        b = torch.randn(128, 64, device=device, dtype=torch.float16)
        c = gemm(a, b)
        torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-2, atol=1e-1)
    print(f"lazy_jit gemm ok for M in (128, 256, 192); specialisations: {len(gemm._cache)}")


if __name__ == "__main__":
    main()
