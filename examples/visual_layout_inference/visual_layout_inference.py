"""Layout visualisation (reference: examples/visual_layout_inference/visual_layout_inference.py).

With ``tl.layout_visualization_enable`` the compiler writes, after layout inference, every
fragment's (thread, register) map and every LDS tile's swizzle: a ``<kernel>.layouts.txt``
summary and per 2-D fragment the element grid (thread id / register per element) in the requested
formats (txt, svg, png, pdf), under ``$TILELANG_LAYOUT_DIR`` (default ``./tilelang_layouts``).
On gfx950 the accumulator fragment is the 16x16 MFMA C layout: lane l holds rows 4*(l//16)+v,
column l%16 of each 16x16 block."""
import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1], pass_configs={
    tilelang.PassConfigKey.TL_LAYOUT_VISUALIZATION_ENABLE: True,
    tilelang.PassConfigKey.TL_LAYOUT_VISUALIZATION_FORMATS: "txt,svg",
})
def matmul(M, N, K, block_M, block_N, block_K, dtype="float16", accum_dtype="float"):

    @T.prim_func
    def gemm(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=64) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=2):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(B[k * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local)
            T.copy(C_local, C[by * block_M, bx * block_N])

    return gemm


def main():
    import torch
    kernel = matmul(128, 128, 128, 32, 32, 32)
    a = torch.randn(128, 128).cuda().half()
    b = torch.randn(128, 128).cuda().half()
    torch.testing.assert_close(kernel(a, b), a @ b, rtol=1e-2, atol=1e-2)
    print("All check passed.")
    from tilelang.analysis.layout_visual import layout_dir
    print("layouts written to", layout_dir())


if __name__ == "__main__":
    main()
