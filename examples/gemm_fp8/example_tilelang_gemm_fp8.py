"""FP8 GEMM (reference: examples/gemm_fp8/example_tilelang_gemm_fp8.py, example_tilelang_gemm_amd.py).

gfx950 uses OCP fp8 (float8_e4m3fn / float8_e5m2).  With block_K % 128 == 0 the tile GEMM
issues v_mfma_scale_f32_16x16x128_f8f6f4 with unit e8m0 scales — twice the bf16 MFMA rate
(~5 PFLOPS dense on MI355X); B is given K-contiguous ([N, K], transpose_B=True).
"""
import argparse

import tilelang
import tilelang.language as T
from tilelang.layout import PaddedLayout


@tilelang.jit(out_idx=[-1])
def matmul(M, N, K, block_M=256, block_N=256, block_K=128, threads=512, num_stages=2, dtype="float8_e4m3fn",
           out_dtype="bfloat16", accum_dtype="float", panel=8, staged_epilogue=False):
    """``staged_epilogue``: the C tile goes through row-padded LDS (the A/B ring's space, dead after
    the loop) and leaves as row-contiguous 16-byte stores -- the small-K shapes are store-bound."""

    @T.prim_func
    def gemm_fp8(
            A: T.Tensor((M, K), dtype),
            B: T.Tensor((N, K), dtype),
            C: T.Tensor((M, N), out_dtype),
    ):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_N, block_K), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.use_swizzle(panel_size=panel)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(B[bx * block_N, k * block_K], B_shared)
                T.gemm(A_shared, B_shared, C_local, transpose_B=True)
            if staged_epilogue:
                C_shared = T.alloc_shared((block_M, block_N), out_dtype)
                T.annotate_layout({C_shared: PaddedLayout((block_M, block_N), 8)})
                T.copy(C_local, C_shared)
                T.copy(C_shared, C[by * block_M, bx * block_N])
            else:
                T.copy(C_local, C[by * block_M, bx * block_N])

    return gemm_fp8


def calc_diff(x, y):
    x, y = x.double(), y.double()
    denom = (x * x + y * y).sum()
    return (1 - 2 * (x * y).sum() / denom).item()


def main(M=8192, N=8192, K=8192):
    import torch
    kernel = matmul(M, N, K)
    a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
    b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
    c = kernel(a, b)
    ref = a.float() @ b.float().t()
    d = calc_diff(c, ref)
    assert d < 1e-3, d
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b))
    print(f"fp8 gemm {M}x{N}x{K}: {lat:.3f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS (diff {d:.2e})")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=8192)
    p.add_argument("--n", type=int, default=8192)
    p.add_argument("--k", type=int, default=8192)
    a = p.parse_args()
    main(a.m, a.n, a.k)
