"""DeepGEMM-style block-scaled fp8 GEMM with two-level accumulation (reference:
examples/deepseek_deepgemm/example_deepgemm_fp8_2xAcc.py:12-84).

C[m, n] = sum_kb  sa[m, kb] * sb[n // 128, kb] * (A[m, kb*128:(kb+1)*128] . B[n, kb*128:(kb+1)*128])

A is per-token (1x128) scaled, B per-block (128x128) scaled, both float8_e4m3fn (OCP fp8 on gfx950).
CDNA4 schedule: block_K equals the 128-wide scale group, so each K step is exactly one
v_mfma_scale_f32_16x16x128_f8f6f4 per 16x16 accumulator tile (unit e8m0 scales — the fp32 group
scales are not powers of two and cannot ride the MFMA's own scale operand).  The raw partial is
promoted into a second fp32 accumulator with the (row scale x column-group scale) product after
every K step — the "2xAcc" that keeps fp8 rounding error from compounding over long K.  The
per-step scales are staged through LDS with the A/B tiles by the same LDS-DMA pipeline.
"""
import argparse

import tilelang
import tilelang.language as T

GROUP = 128


@tilelang.jit
def tl_gemm(M, N, K, block_N=128, in_dtype="float8_e4m3fn", out_dtype="bfloat16", accum_dtype="float",
            block_M=128, threads=256, num_stages=2, panel=8):
    assert in_dtype in ("float8_e4m3fn", "float8_e4m3"), "block-scaled fp8 GEMM takes e4m3 operands"
    in_dtype = "float8_e4m3fn"
    assert out_dtype in ("bfloat16", "float32", "float")
    block_K = GROUP
    assert K % GROUP == 0
    KG = K // GROUP
    NG = T.ceildiv(N, GROUP)
    n_sb = max(1, block_N // GROUP)
    assert block_N % GROUP == 0 or GROUP % block_N == 0

    @T.prim_func
    def main(A: T.Tensor((M, K), in_dtype), B: T.Tensor((N, K), in_dtype), C: T.Tensor((M, N), out_dtype),
             scales_a: T.Tensor((M, KG), "float32"), scales_b: T.Tensor((NG, KG), "float32")):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, block_K), in_dtype)
            B_s = T.alloc_shared((block_N, block_K), in_dtype)
            sa_s = T.alloc_shared((block_M, ), "float32")
            sb_s = T.alloc_shared((n_sb, ), "float32")
            C_part = T.alloc_fragment((block_M, block_N), accum_dtype)
            C_acc = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.use_swizzle(panel_size=panel)
            T.clear(C_acc)
            for k in T.Pipelined(KG, num_stages=num_stages):
                T.copy(A[by * block_M, k * block_K], A_s)
                T.copy(B[bx * block_N, k * block_K], B_s)
                for i in T.Parallel(block_M):
                    sa_s[i] = scales_a[T.min(by * block_M + i, M - 1), k]
                for j in T.Parallel(n_sb):
                    sb_s[j] = scales_b[T.min((bx * block_N) // GROUP + j, NG - 1), k]
                T.gemm(A_s, B_s, C_part, transpose_B=True, clear_accum=True)
                for i, j in T.Parallel(block_M, block_N):
                    C_acc[i, j] += C_part[i, j] * (sa_s[i] * sb_s[j // GROUP])
            T.copy(C_acc, C[by * block_M, bx * block_N])

    return main


def ceildiv(a, b):
    return (a + b - 1) // b


def per_token_cast_to_fp8(x):
    import torch
    assert x.dim() == 2 and x.size(1) % GROUP == 0
    m, n = x.shape
    xv = x.view(m, -1, GROUP)
    amax = xv.abs().float().amax(dim=2).view(m, -1).clamp(1e-4)
    return (xv * (448.0 / amax.unsqueeze(2))).to(torch.float8_e4m3fn).view(m, n), (amax / 448.0).view(m, -1)


def per_block_cast_to_fp8(x):
    import torch
    m, n = x.shape
    xp = torch.zeros(ceildiv(m, GROUP) * GROUP, ceildiv(n, GROUP) * GROUP, dtype=x.dtype, device=x.device)
    xp[:m, :n] = x
    xv = xp.view(-1, GROUP, xp.size(1) // GROUP, GROUP)
    amax = xv.abs().float().amax(dim=(1, 3), keepdim=True).clamp(1e-4)
    xs = (xv * (448.0 / amax)).to(torch.float8_e4m3fn)
    return xs.view_as(xp)[:m, :n].contiguous(), (amax / 448.0).view(xv.size(0), xv.size(2))


def ref_deepgemm_fp8(A_fp8, B_fp8, A_scale, B_scale, out_dtype):
    """fp32 reference of the same block-scaled product (dequantise, then one fp32 GEMM)."""
    import torch
    a = A_fp8.float() * A_scale.repeat_interleave(GROUP, dim=1)[:, :A_fp8.shape[1]]
    sb = B_scale.repeat_interleave(GROUP, dim=0).repeat_interleave(GROUP, dim=1)
    b = B_fp8.float() * sb[:B_fp8.shape[0], :B_fp8.shape[1]]
    return (a @ b.t()).to(out_dtype)


def calc_diff(x, y):
    x, y = x.double(), y.double()
    return (1 - 2 * (x * y).sum() / (x * x + y * y).sum()).item()


def assert_tl_gemm_correctness(M, N, K, block_N, in_dtype="float8_e4m3fn", out_dtype="bfloat16", accum_dtype="float",
                               bench=True, **kw):
    import torch
    kernel = tl_gemm(M, N, K, block_N, in_dtype, out_dtype, accum_dtype, **kw)
    odt = torch.bfloat16 if out_dtype == "bfloat16" else torch.float32
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    A_fp8, A_scale = per_token_cast_to_fp8(A)
    B_fp8, B_scale = per_block_cast_to_fp8(B)
    C = torch.zeros(M, N, device="cuda", dtype=odt)
    kernel(A_fp8, B_fp8, C, A_scale, B_scale)
    diff = calc_diff(C, ref_deepgemm_fp8(A_fp8, B_fp8, A_scale, B_scale, torch.float32))
    assert diff < 1e-3, diff
    if bench:
        lat = kernel.get_profiler().do_bench(lambda: kernel(A_fp8, B_fp8, C, A_scale, B_scale))
        print(f"deepgemm fp8 2xAcc {M}x{N}x{K} block_N={block_N} {out_dtype}: {lat:.3f} ms, "
              f"{2 * M * N * K / lat * 1e-9:.1f} TFLOPS (diff {diff:.2e})")
    return diff


def main():
    assert_tl_gemm_correctness(1024, 1024, 8192, 128)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1024)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--k", type=int, default=8192)
    a = p.parse_args()
    for out_dtype in ("bfloat16", "float32"):
        for bn in (128, 256):
            assert_tl_gemm_correctness(a.m, a.n, a.k, bn, out_dtype=out_dtype)
    assert_tl_gemm_correctness(8192, 8192, 8192, 256, block_M=256, threads=512)
