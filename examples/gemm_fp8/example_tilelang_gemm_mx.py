"""Block-scaled MX GEMM (OCP MXFP8 / MXFP4) on the gfx950 scaled matrix cores.

``T.gemm_scaled`` lowers to ``v_mfma_scale_f32_16x16x128_f8f6f4``: the hardware multiplies every
32-element K block of each row of A and B by its e8m0 scale (2^(s-127)) inside the MFMA, so the
MX tensors are consumed as stored — no dequantisation pass.  Peak rates (dense): fp8 ~5 PF,
fp4 / fp6 ~10 PF (4x bf16).  Operands are K-contiguous: A ``[M, K]`` and B ``[N, K]`` bytes (fp8),
``[M, K/2]`` / ``[N, K/2]`` packed e2m1 pairs (low nibble = even element), or ``[M, 3K/4]`` packed
e2m3 / e3m2 (``tilelang.quantize.pack_fp6``: 4 elements per 3 bytes); scales ``[M, K/32]``,
``[N, K/32]`` read straight from global memory (a few bytes per 32 K per lane; L1/L2 resident).

The reference has no MX path (its AMD fp8 GEMM is CDNA3 fnuz, ``examples/gemm_fp8/
example_tilelang_gemm_amd.py``; its MXFP4 example dequantises to bf16,
``examples/dequantize_gemm/example_dequant_gemm_bf16_mxfp4_hopper.py``).
"""
import argparse

import tilelang
import tilelang.language as T

_DT = {"e4m3": "float8_e4m3fn", "e5m2": "float8_e5m2", "e2m1": "uint8", "e2m3": "uint8", "e3m2": "uint8"}


def _cols(k, fmt):
    """Bytes of K elements: fp8 1 each, packed fp4 1/2, packed fp6 3/4."""
    return k // 2 if fmt == "e2m1" else k * 3 // 4 if fmt in ("e2m3", "e3m2") else k


@tilelang.jit(out_idx=[-1])
def mx_matmul(M, N, K, block_M=256, block_N=None, block_K=None, threads=512, num_stages=None, a_fmt="e4m3",
              b_fmt="e4m3", out_dtype="bfloat16", accum_dtype="float", panel=8, scales_in_lds=True,
              preshuffle_scales=False):
    """``scales_in_lds``: the e8m0 scale tiles ([block, block_K/32] bytes) ride the pipeline into
    LDS with the operands, so the MFMA loop reads them with ds_read instead of waiting on a
    global load per K step.  ``preshuffle_scales``: SA / SB are 1-D, in the tile order of
    ``tilelang.quantize.preshuffle_mx_scales(s, block_M or block_N, block_K)``: one ds_read_b32 per
    four 16-row fragments instead of a byte read per fragment."""
    # tiles per format pair, measured at 8192^3 (scripts/sweep_mx.py, profiles/r3/s3/lowp/): with the
    # scale tiles on small-tile LDS-DMA the 256x256 2-stage tiles win for every pair:
    # fp4 x fp4 256x256x256 3.33 PF (256x128x256 3-stage 2.49), fp8 x fp8 256x256x128 1.86 PF
    # (256x128x128 3-stage 1.44), fp8 x fp4 256x256x128 2.26 PF
    if block_K is None:  # fp4 x fp4: 128-byte rows at block_K 256; fp6 rows would be 192 bytes
        block_K = 256 if a_fmt == b_fmt == "e2m1" else 128
    if block_N is None:
        block_N = 256
    if num_stages is None:
        num_stages = 2
    ac, bc = _cols(K, a_fmt), _cols(K, b_fmt)
    bka, bkb = _cols(block_K, a_fmt), _cols(block_K, b_fmt)
    sk = block_K // 32
    nk = K // block_K
    if preshuffle_scales:
        return _mx_matmul_ps(M, N, K, block_M, block_N, block_K, threads, num_stages, a_fmt, b_fmt, out_dtype,
                             accum_dtype, panel, ac, bc, bka, bkb, sk, nk)

    @T.prim_func
    def main(
            A: T.Tensor((M, ac), _DT[a_fmt]),
            B: T.Tensor((N, bc), _DT[b_fmt]),
            SA: T.Tensor((M, K // 32), "uint8"),
            SB: T.Tensor((N, K // 32), "uint8"),
            C: T.Tensor((M, N), out_dtype),
    ):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, bka), _DT[a_fmt])
            B_s = T.alloc_shared((block_N, bkb), _DT[b_fmt])
            C_l = T.alloc_fragment((block_M, block_N), accum_dtype)
            SA_s = T.alloc_shared((block_M, sk), "uint8")
            SB_s = T.alloc_shared((block_N, sk), "uint8")
            T.use_swizzle(panel_size=panel)
            T.clear(C_l)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A[by * block_M, k * bka], A_s)
                T.copy(B[bx * block_N, k * bkb], B_s)
                if scales_in_lds:
                    T.copy(SA[by * block_M, k * sk], SA_s)
                    T.copy(SB[bx * block_N, k * sk], SB_s)
                    T.gemm_scaled(A_s, B_s, C_l, SA_s, SB_s, transpose_B=True, a_format=a_fmt, b_format=b_fmt)
                else:
                    T.gemm_scaled(A_s, B_s, C_l, SA[by * block_M:(by + 1) * block_M, k * sk:(k + 1) * sk],
                                  SB[bx * block_N:(bx + 1) * block_N, k * sk:(k + 1) * sk], transpose_B=True,
                                  a_format=a_fmt, b_format=b_fmt)
            T.copy(C_l, C[by * block_M, bx * block_N])

    return main


_NARROW = ("e2m1", "e2m3", "e3m2")
E2M1 = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0, -0.0, -0.5, -1.0, -1.5, -2.0, -3.0, -4.0, -6.0]


def _mx_matmul_ps(M, N, K, block_M, block_N, block_K, threads, num_stages, a_fmt, b_fmt, out_dtype, accum_dtype,
                  panel, ac, bc, bka, bkb, sk, nk):
    ta, tb = block_M * sk, block_N * sk  # bytes per pre-shuffled scale tile (64-byte rows)

    @T.prim_func
    def main(
            A: T.Tensor((M, ac), _DT[a_fmt]),
            B: T.Tensor((N, bc), _DT[b_fmt]),
            SA: T.Tensor((M * K // 2048, 64), "uint8"),
            SB: T.Tensor((N * K // 2048, 64), "uint8"),
            C: T.Tensor((M, N), out_dtype),
    ):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, bka), _DT[a_fmt])
            B_s = T.alloc_shared((block_N, bkb), _DT[b_fmt])
            C_l = T.alloc_fragment((block_M, block_N), accum_dtype)
            SA_s = T.alloc_shared((ta // 64, 64), "uint8")
            SB_s = T.alloc_shared((tb // 64, 64), "uint8")
            T.use_swizzle(panel_size=panel)
            T.clear(C_l)
            for k in T.Pipelined(nk, num_stages=num_stages):
                T.copy(A[by * block_M, k * bka], A_s)
                T.copy(B[bx * block_N, k * bkb], B_s)
                T.copy(SA[(by * nk + k) * (ta // 64), 0], SA_s)
                T.copy(SB[(bx * nk + k) * (tb // 64), 0], SB_s)
                T.gemm_scaled(A_s, B_s, C_l, SA_s, SB_s, transpose_B=True, a_format=a_fmt, b_format=b_fmt,
                              scale_layout="preshuffled")
            T.copy(C_l, C[by * block_M, bx * block_N])

    return main


def quantize(x, fmt):
    """fp32 [R, K] -> (MX elements as stored, e8m0 scales [R, K/32]) with per-block power-of-2 scales."""
    import torch
    if fmt in ("e2m3", "e3m2"):
        from tilelang.quantize import quantize_mxfp6
        return quantize_mxfp6(x, fmt)
    R, K = x.shape
    blk = x.float().reshape(R, K // 32, 32)
    amax = blk.abs().amax(-1).clamp(min=1e-30)
    vmax = {"e4m3": 448.0, "e5m2": 57344.0, "e2m1": 6.0}[fmt]  # largest representable element
    e = torch.ceil(torch.log2(amax / vmax))
    s = (e + 127).clamp(0, 254).to(torch.uint8)
    q = blk / torch.exp2(s.float() - 127).unsqueeze(-1)
    q = q.reshape(R, K)
    if fmt == "e4m3":
        return q.to(torch.float8_e4m3fn), s
    if fmt == "e5m2":
        return q.to(torch.float8_e5m2), s
    lut = torch.tensor(E2M1[:8], device=x.device)
    mag = (q.abs().unsqueeze(-1) - lut).abs().argmin(-1)
    code = (mag | ((q < 0).long() << 3)).to(torch.uint8)
    return (code[:, 0::2] | (code[:, 1::2] << 4)).contiguous(), s


def dequantize(q, s, fmt):
    import torch
    if fmt in ("e2m3", "e3m2"):
        from tilelang.quantize import dequantize_mxfp6
        return dequantize_mxfp6(q, s, fmt)
    if fmt == "e2m1":
        lut = torch.tensor(E2M1, device=q.device)
        lo, hi = (q & 15).long(), (q >> 4).long()
        v = torch.stack([lut[lo], lut[hi]], -1).reshape(q.shape[0], -1)
    else:
        v = q.float()
    return v * torch.exp2(s.float() - 127).repeat_interleave(32, 1)


def ref_program(a, b, sa, sb, a_fmt, b_fmt):
    return dequantize(a, sa, a_fmt) @ dequantize(b, sb, b_fmt).t()


def main(M=8192, N=8192, K=8192, a_fmt="e4m3", b_fmt="e4m3"):
    import torch
    kernel = mx_matmul(M, N, K, a_fmt=a_fmt, b_fmt=b_fmt)
    a, sa = quantize(torch.randn(M, K, device="cuda") * 3, a_fmt)
    b, sb = quantize(torch.randn(N, K, device="cuda") * 0.2, b_fmt)
    c = kernel(a, b, sa, sb)
    ref = ref_program(a, b, sa, sb, a_fmt, b_fmt)
    torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b, sa, sb))
    print(f"MX {a_fmt}x{b_fmt} gemm {M}x{N}x{K}: {lat:.3f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")
    # the same GEMM with the scales pre-shuffled once (weights offline, activations by their quantizer)
    from tilelang.quantize import preshuffle_mx_scales
    bk = 256 if a_fmt == b_fmt == "e2m1" else 128
    kps = mx_matmul(M, N, K, a_fmt=a_fmt, b_fmt=b_fmt, preshuffle_scales=True)
    pa, pb = preshuffle_mx_scales(sa, 256, bk), preshuffle_mx_scales(sb, 256, bk)
    torch.testing.assert_close(kps(a, b, pa, pb).float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    lat = kps.get_profiler().do_bench(lambda: kps(a, b, pa, pb))
    print(f"MX {a_fmt}x{b_fmt} gemm, pre-shuffled scales: {lat:.3f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=8192)
    p.add_argument("--n", type=int, default=8192)
    p.add_argument("--k", type=int, default=8192)
    p.add_argument("--a_fmt", default="e4m3")
    p.add_argument("--b_fmt", default="e4m3")
    a = p.parse_args()
    main(a.m, a.n, a.k, a.a_fmt, a.b_fmt)
