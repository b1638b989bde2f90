"""BF16 x MXFP4 weight-only GEMM (reference: examples/dequantize_gemm/
example_dequant_gemm_bf16_mxfp4_hopper.py, example_dequant_gemm_fp4_hopper.py).

C[M, N] = A[M, K] (bf16) @ dequant(Bq, S)^T with Bq [N, K/2] uint8 = two OCP e2m1 codes per byte
(low nibble = even k) and S [N, K/32] uint8 e8m0 block scales (w = e2m1 * 2^(s-127)).  The
packed tile (1/4 of a bf16 tile) and its scales stream through the LDS-DMA ring; the waves
expand them into a bf16 LDS tile (the e2m1 decode is a 16-entry select, the e8m0 scale an
exponent) and run bf16 MFMAs -- weight HBM traffic is 4.25 bits/element, which is what bounds
the small-M (decode) shapes.

``mode="native"`` (the MI355X path for compute-bound, prefill-sized M): the activations are
quantised on the fly to MXFP8 (e4m3 + e8m0 per 32, ``quant_act_mxfp8``) and the GEMM runs on the
scaled matrix cores, ``v_mfma_scale_f32_16x16x128_f8f6f4`` with A in fp8 and the weights in their
stored fp4 (``T.gemm_scaled``, examples/gemm_fp8/example_tilelang_gemm_mx.py): no dequantised
tile ever exists, and the MFMA runs at the fp8 rate (2x bf16).
"""
import argparse

import tilelang
import tilelang.language as T
from tilelang.quantize import dequantize_mxfp4, e2m1_to_float, quantize_mxfp4


@tilelang.jit(out_idx=[-1])
def dequant_gemm_mxfp4(M, N, K, block_M=None, block_N=None, block_K=128, threads=None, num_stages=2,
                       dtype="bfloat16", accum_dtype="float"):
    # decode (small M): thin tiles so N/block_N workgroups fill the CUs; prefill: 128x128
    if block_M is None:  # (a 256-row tile + the 2-stage ring + the bf16 B tile exceed 160 KiB of LDS)
        block_M = 16 if M <= 16 else (64 if M <= 256 else 128)
    if block_N is None:
        block_N = 32 if M <= 16 else 128
    if threads is None:
        threads = 64 if M <= 16 else 256
    assert K % block_K == 0 and block_K % 32 == 0

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), Bq: T.Tensor((N, K // 2), "uint8"), S: T.Tensor((N, K // 32), "uint8"),
             C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            Bq_shared = T.alloc_shared((block_N, block_K // 2), "uint8")
            S_shared = T.alloc_shared((block_N, block_K // 32), "uint8")
            B_shared = T.alloc_shared((block_N, block_K), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            C_cast = T.alloc_fragment((block_M, block_N), dtype)
            T.use_swizzle(panel_size=8)
            T.clear(C_local)
            for k in T.Pipelined(K // block_K, num_stages=num_stages):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(Bq[bx * block_N, k * (block_K // 2)], Bq_shared)
                T.copy(S[bx * block_N, k * (block_K // 32)], S_shared)
                for n, kk in T.Parallel(block_N, block_K):
                    nib = T.Cast("int32", (Bq_shared[n, kk // 2] >> ((kk % 2) * 4)) & 15)
                    if dtype == "bfloat16":
                        # integer decode straight into bf16 bits: the e8m0 scale only adds to
                        # the exponent field (e2m1 e=0 is 0 or 0.5 -> exponent s-1)
                        sc = T.Cast("int32", S_shared[n, kk // 32])
                        e = (nib >> 1) & 3
                        sgn = (nib & 8) << 12
                        bits = T.if_then_else(e == 0, T.if_then_else((nib & 1) == 1, sgn | ((sc - 1) << 7), sgn),
                                              sgn | ((e + sc - 1) << 7) | ((nib & 1) << 6))
                        B_shared[n, kk] = T.reinterpret(T.Cast("uint16", bits), dtype)
                    else:
                        sc = T.exp2(T.Cast("float32", S_shared[n, kk // 32]) - 127.0)
                        B_shared[n, kk] = T.Cast(dtype, e2m1_to_float(nib) * sc)
                T.gemm(A_shared, B_shared, C_local, transpose_B=True)
            T.copy(C_local, C_cast)
            T.copy(C_cast, C[by * block_M, bx * block_N])

    return main


@tilelang.jit(out_idx=[1, 2])
def quant_act_mxfp8(M, K, block_M=64, threads=256, dtype="bfloat16"):
    """A [M, K] -> (e4m3 [M, K], e8m0 [M, K/32]) with power-of-two block scales: every lane owns
    one 32-element block (64 B read as 16-byte vectors)."""
    G = K // 32

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), Q: T.Tensor((M, K), "float8_e4m3fn"), SA: T.Tensor((M, G), "uint8")):
        with T.Kernel(T.ceildiv(M, block_M), threads=threads) as bx:
            for r, g in T.Parallel(block_M, G):
                row = bx * block_M + r
                if row < M:
                    v = T.alloc_local((32, ), "float32")
                    amax = T.alloc_var("float32")
                    amax = 1e-30
                    for j in T.unroll(32):
                        v[j] = T.Cast("float32", A[row, g * 32 + j])
                        amax = T.max(amax, T.abs(v[j]))
                    e = T.min(T.max(T.ceil(T.log2(amax / 448.0)), -127.0), 127.0)
                    inv = T.exp2(-e)
                    SA[row, g] = T.Cast("uint8", e + 127.0)
                    for j in T.unroll(32):
                        Q[row, g * 32 + j] = T.Cast("float8_e4m3fn", v[j] * inv)

    return main


@tilelang.jit(out_idx=[-1])
def mxfp4_gemv(M, N, K, block_N=None, threads=256, dtype="bfloat16", row_group=None):
    """Decode-sized (M <= 8) bf16 x MXFP4: a pure weight stream (include/tl/gemv.h): 16-byte
    non-temporal weight loads, v_cvt_scalef32_pk_f32_fp4 (two codes per instruction, the e8m0
    scale folded in), FMAs against x held in registers, one block reduction per ``row_group``
    rows.  ``block_N`` rows per block (x is re-read once per row group from L1/L2: 32 rows per
    block keep the x traffic a fraction of the weight bytes for every M)."""
    assert M <= 8 and K % 32 == 0 and dtype == "bfloat16"
    if block_N is None:  # scripts/sweep_gemv_fp4.py (profiles/r3/s3/lowp/sweep_gemv_fp4.log): 4-row blocks
        block_N = 4 if M <= 4 else 2  # M=1 16384^2: 4.69 TB/s of weights (16-row blocks 4.10)
    if row_group is None:
        # one group per block: more, smaller blocks keep more weight bytes in flight; 32-row blocks
        # in row groups cut the x re-reads but halved the M = 4 / 8 rate (1436 -> 699 GB/s at M = 4,
        # profiles/r3/s3/lowp/gemv_rowgroup_ab.log)
        row_group = block_N
    assert block_N % row_group == 0

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), Bq: T.Tensor((N, K // 2), "uint8"), S: T.Tensor((N, K // 32), "uint8"),
             C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), threads=threads) as bx:
            red = T.alloc_shared((threads // 64, row_group * M), "float32")
            T.evaluate(T.call_extern("handle", f"tl::mxfp4_gemv<{M}, {block_N}, {threads}, {row_group}>",
                                     T.address_of(A[0, 0]),
                                     T.address_of(Bq[0, 0]), T.address_of(S[0, 0]), T.address_of(C[0, 0]), N, K,
                                     bx * block_N, T.address_of(red[0, 0])))

    return main


def mxfp4_gemm_native(A, Bq, S):
    """bf16 A x MXFP4 weights on the scaled matrix cores (A quantised to MXFP8 on the fly)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gemm_fp8"))
    from example_tilelang_gemm_mx import mx_matmul
    M, K = A.shape
    N = Bq.shape[0]
    q, sa = quant_act_mxfp8(M, K)(A)
    return mx_matmul(M, N, K, a_fmt="e4m3", b_fmt="e2m1")(q, Bq, sa, S)


def ref_program(A, Bq, S):
    return (A.float() @ dequantize_mxfp4(Bq, S).t()).to(A.dtype)


def main(M=16, N=8192, K=8192, mode="dequant"):
    import torch
    if mode == "gemv":
        kernel = mxfp4_gemv(M, N, K)
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
        c = kernel(A, Bq, S)
        torch.testing.assert_close(c.float(), ref_program(A, Bq, S).float(), rtol=2e-2, atol=1.0)
        lat = kernel.get_profiler().do_bench(lambda: kernel(A, Bq, S))
        wbytes = N * K // 2 + N * K // 32
        print(f"bf16 x mxfp4 GEMV {M}x{N}x{K}: {lat * 1e3:.1f} us, {wbytes / lat * 1e-9:.2f} TB/s of weights")
        return
    if mode == "native":
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
        c = mxfp4_gemm_native(A, Bq, S)
        ref = ref_program(A, Bq, S).float()
        rel = ((c.float() - ref).norm() / ref.norm()).item()
        assert rel < 0.05, rel  # MXFP8 activations: ~2^-4 relative rounding per element
        print(f"native MX path: relative error {rel:.3e} vs bf16 x dequant(fp4)")
        from tilelang.profiler import do_bench
        lat = do_bench(lambda: mxfp4_gemm_native(A, Bq, S))
        print(f"bf16(->mxfp8) x mxfp4 GEMM {M}x{N}x{K} (quant + scaled MFMA): {lat:.4f} ms, "
              f"{2 * M * N * K / lat * 1e-9:.1f} TFLOPS")
        return
    kernel = dequant_gemm_mxfp4(M, N, K)
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
    c = kernel(A, Bq, S)
    torch.testing.assert_close(c.float(), ref_program(A, Bq, S).float(), rtol=2e-2, atol=1.0)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(A, Bq, S))
    print(f"bf16 x mxfp4 GEMM {M}x{N}x{K}: {lat:.4f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS, "
          f"{(N * K // 2 + N * K // 32 + M * K * 2) / lat * 1e-6:.1f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=16)
    p.add_argument("--n", type=int, default=8192)
    p.add_argument("--k", type=int, default=8192)
    p.add_argument("--mode", choices=["dequant", "native", "gemv"], default="dequant")
    a = p.parse_args()
    main(a.m, a.n, a.k, a.mode)
