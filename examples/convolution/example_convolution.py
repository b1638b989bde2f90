"""2-D convolution as an implicit GEMM (reference: examples/convolution/example_convolution.py).

out[N, OH, OW, F] = conv(data[N, H, W, C], kernel[KH, KW, C, F]) with stride S, dilation D,
padding P.  GEMM view: M = N*OH*OW output pixels, N = F filters, K = KH*KW*C.  Each K step the
A tile is gathered from the NHWC image with ``T.c2d_im2col`` (zero padding at the borders),
the B tile is a plain LDS-DMA copy of the flattened filter ``[KH*KW*C, F]``, and the MFMA
accumulates in registers; the output tile is written through the flattened ``[M, F]`` view.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[2])
def convolution(N, C, H, W, F, K, S, D, P, block_M=128, block_N=128, block_K=64, num_stages=2, threads=256,
                dtype="float16", accum_dtype="float", unroll=2):
    KH = KW = K
    OH = (H + 2 * P - D * (K - 1) - 1) // S + 1
    OW = (W + 2 * P - D * (K - 1) - 1) // S + 1
    assert (KH * KW * C) % block_K == 0

    @T.prim_func
    def main(data: T.Tensor((N, H, W, C), dtype), kernel: T.Tensor((KH, KW, C, F), dtype),
             out: T.Tensor((N, OH, OW, F), dtype)):
        with T.Kernel(T.ceildiv(F, block_N), T.ceildiv(N * OH * OW, block_M), threads=threads) as (bx, by):
            data_shared = T.alloc_shared((block_M, block_K), dtype)
            kernel_shared = T.alloc_shared((block_K, block_N), dtype)
            out_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            out_cast = T.alloc_fragment((block_M, block_N), dtype)
            kernel_flat = T.Tensor((KH * KW * C, F), dtype, kernel.data)
            out_flat = T.Tensor((N * OH * OW, F), dtype, out.data)
            T.clear(out_local)
            # unrolled (constant ring slots): 2.015 -> 1.962 ms at the example's shape
            for k_iter in T.Pipelined(KH * KW * C // block_K, num_stages=num_stages, unroll=unroll):
                T.c2d_im2col(data, data_shared, by, k_iter, KH, S, D, P)
                T.copy(kernel_flat[k_iter * block_K, bx * block_N], kernel_shared)
                T.gemm(data_shared, kernel_shared, out_local)
            T.copy(out_local, out_cast)
            T.copy(out_cast, out_flat[by * block_M, bx * block_N])

    return main


def ref_program(stride, padding, dilation):
    import torch

    def main(A, B):
        out = torch.conv2d(A.permute(0, 3, 1, 2).float(), B.permute(3, 2, 0, 1).float(), stride=stride,
                           padding=padding, dilation=dilation)
        return out.permute(0, 2, 3, 1).to(A.dtype)

    return main


def main(n=128, c=128, h=64, w=64, f=128, k=3, s=1, d=1, p=1):
    import torch
    kernel = convolution(n, c, h, w, f, k, s, d, p)
    a = torch.randn(n, h, w, c, device="cuda", dtype=torch.float16)
    b = torch.randn(k, k, c, f, device="cuda", dtype=torch.float16)
    out = kernel(a, b)
    torch.testing.assert_close(out.float(), ref_program(s, p, d)(a, b).float(), rtol=1e-2, atol=1e-1)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b))
    oh = (h + 2 * p - d * (k - 1) - 1) // s + 1
    ow = (w + 2 * p - d * (k - 1) - 1) // s + 1
    print(f"conv {n}x{h}x{w}x{c} -> {f} k{k}: {lat:.3f} ms, {2 * n * oh * ow * f * k * k * c / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    for name, dflt in (("n", 128), ("c", 128), ("h", 64), ("w", 64), ("f", 128), ("k", 3), ("s", 1), ("d", 1),
                       ("p", 1)):
        ap.add_argument(f"--{name}", type=int, default=dflt)
    a = ap.parse_args()
    main(a.n, a.c, a.h, a.w, a.f, a.k, a.s, a.d, a.p)
