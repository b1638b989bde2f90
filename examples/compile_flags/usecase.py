"""Extra device-compiler flags (reference: examples/compile_flags/usecase.py).

``compile_flags`` (a list or one space-separated string) are appended to the ROCm clang command
that builds the gfx950 code object (``clang++ -x hip --offload-arch=gfx950 --offload-device-only
-O3 ...``); they are part of the kernel cache key.  The reference's nvcc flags
(``--use_fast_math``, ``--expt-relaxed-constexpr``) have clang counterparts (``-ffast-math``)."""
import tilelang
import tilelang.language as T


def matmul(M, N, K, block_M, block_N, block_K, dtype="float16", accum_dtype="float"):

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=256) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.clear(C_local)
            for ko in T.Pipelined(T.ceildiv(K, block_K), num_stages=2):
                T.copy(A[by * block_M, ko * block_K], A_shared)
                T.copy(B[ko * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local)
            T.copy(C_local, C[by * block_M, bx * block_N])

    return main


def build(M=1024, N=1024, K=1024, target="hip", flags=("-O3", "-ffast-math")):
    func = matmul(M, N, K, 128, 128, 64)
    # list form; "-O3 -ffast-math" (one string) is accepted too
    return tilelang.compile(func, out_idx=[2], target=target, compile_flags=list(flags))


def main():
    import torch
    M = N = K = 1024
    jit_kernel = build(M, N, K)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = jit_kernel(a, b)
    torch.testing.assert_close(c, a @ b, rtol=1e-2, atol=1e-2)
    print("Kernel output matches PyTorch reference.")


if __name__ == "__main__":
    main()
