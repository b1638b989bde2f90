"""Static roofline analysis of a tile program (reference: examples/analyze/example_gemm_analyze.py).

``tilelang.tools.Analyzer`` walks the tile IR (grid x loop trip counts x tile ops) and reports
FLOPs, global-memory bytes and the MI355X roofline time (MFMA peak vs HBM3E bandwidth)."""
import tilelang.language as T
from tilelang.tools import Analyzer

M = N = K = 1024


def kernel(block_M=128, block_N=128, block_K=32, num_stages=3, thread_num=256, enable_rasteration=True):
    dtype, accum_dtype = "float16", "float"

    @T.prim_func
    def matmul(A: T.Tensor((M, K), dtype), B: T.Tensor((N, K), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=thread_num) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_N, block_K), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            C_shared = T.alloc_shared((block_M, block_N), dtype)
            T.use_swizzle(panel_size=10, enable=enable_rasteration)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(B[bx * block_N, k * block_K], B_shared)
                T.gemm(A_shared, B_shared, C_local, transpose_B=True)
            T.copy(C_local, C_shared)
            T.copy(C_shared, C[by * block_M, bx * block_N])

    return matmul


def main():
    result = Analyzer.analysis(kernel(), "MI355X")
    print(result)
    print(f"Analyzed FLOPs: {result.total_flops}")
    print(f"Expected FLOPs: {2 * M * N * K}")
    return result


if __name__ == "__main__":
    main()
