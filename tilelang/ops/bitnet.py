"""BitNet b1.58 kernels: ternary (2-bit) weights x int8 activations on the int8 matrix cores
(reference: examples/bitnet-1.58b/kernel_benchmark/tilelang_bitnet_158_int8xint2_{decode,prefill}.py,
examples/bitnet-1.58b/utils_quant.py:16-31 ``weight_quant`` / ``activation_quant``).

* ``rms_norm_quant(x, w)``: the RMSNorm that precedes every BitLinear group fused with the per-token
  absmax int8 activation quantisation: one pass over the row in registers emits the int8 row and
  its scale (127 / absmax) — the normalised activations never reach HBM in 16-bit form.
* ``int2_gemm(xq, wq, ...)``: C = xq @ (codes(wq) - zero)^T with wq [N, K/4] uint8 holding four
  2-bit codes per byte (k = 4j + i in bits 2i..2i+1).  The packed tile (1/4 of an int8 tile)
  streams through the LDS-DMA ring, the waves expand it to an int8 LDS tile (shift, mask,
  subtract), and ``v_mfma_i32_16x16x64_i8`` accumulates exactly in int32.  Epilogue: raw int32
  (the reference kernels' output), or dequantised in place: C = acc / (s_x[m] * s_w[n]) in fp16/bf16.
  The tile is chosen from M: 16-row tiles and narrow N tiles for decode (weight streaming bound:
  0.25 byte per MAC), 128x128 for prefill.
* ``pack_int2`` / ``weight_quant_ternary`` / ``activation_quant``: host-side helpers.
"""
from __future__ import annotations

import functools

import torch

import tilelang
import tilelang.language as T

_TDT = {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}


def _tiles(M, N, K):
    bk = 128 if K % 128 == 0 else 64
    if M <= 16:
        return 16, 32, bk, 64
    if M <= 128:
        return 64, 64, bk, 256
    return 128, 128, bk, 256


@functools.lru_cache(maxsize=None)
def int2_gemm_kernel(M, N, K, zero=1, out_dtype="int32", target="hip", tiles=None):
    """out_dtype "int32": kernel(xq, wq) -> C int32; otherwise kernel(xq, wq, s_x [M] fp32, s_w [N] fp32) -> C
    (per-output-column weight scales, so fused projections — q|k|v, gate|up — keep their own)."""
    bm, bn, bk, threads = tiles or _tiles(M, N, K)
    assert K % bk == 0 and bk % 64 == 0, "K must be a multiple of 64 (int8 MFMA K step)"
    raw = out_dtype == "int32"

    @T.macro
    def body(A, B, sx, sw, C):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=threads) as (bx, by):
            A_s = T.alloc_shared((bm, bk), "int8")
            Bq_s = T.alloc_shared((bn, bk // 4), "uint8")
            B_s = T.alloc_shared((bn, bk), "int8")
            acc = T.alloc_fragment((bm, bn), "int32")
            T.use_swizzle(panel_size=8)
            T.clear(acc)
            for k in T.Pipelined(K // bk, num_stages=2):
                T.copy(A[by * bm, k * bk], A_s)
                T.copy(B[bx * bn, k * (bk // 4)], Bq_s)
                for n, kk in T.Parallel(bn, bk):
                    code = T.Cast("int32", (Bq_s[n, kk // 4] >> ((kk % 4) * 2)) & 3)
                    B_s[n, kk] = T.Cast("int8", code - zero)
                T.gemm(A_s, B_s, acc, transpose_B=True)
            if raw:
                T.copy(acc, C[by * bm, bx * bn])
            else:
                for i, j in T.Parallel(bm, bn):
                    if (by * bm + i < M) & (bx * bn + j < N):
                        C[by * bm + i, bx * bn + j] = T.Cast(
                            out_dtype, T.Cast("float32", acc[i, j]) / (sx[by * bm + i] * sw[bx * bn + j]))

    if raw:

        @T.prim_func
        def main(A: T.Tensor((M, K), "int8"), B: T.Tensor((N, K // 4), "uint8"), C: T.Tensor((M, N), "int32")):
            body(A, B, None, None, C)
    else:

        @T.prim_func
        def main(A: T.Tensor((M, K), "int8"), B: T.Tensor((N, K // 4), "uint8"), sx: T.Tensor((M, ), "float32"),
                 sw: T.Tensor((N, ), "float32"), C: T.Tensor((M, N), out_dtype)):
            body(A, B, sx, sw, C)

    return tilelang.compile(main, out_idx=[-1], target=target)


@functools.lru_cache(maxsize=None)
def int2_gemv_kernel(M, N, K, Kp, zero=1, out_dtype="float16", target="hip", block_N=16, num_stages=3):
    """Decode-sized (M <= 8) int8 x int2 product without matrix cores: the packed weight rows
    ([N, Kp/4] bytes, Kp = K rounded up to 256 codes, padding codes = ``zero``) stream through a
    3-deep LDS-DMA ring, 64 bytes (256 codes) of each of ``block_N`` rows per step (16 B per lane,
    one wave per workgroup, N / block_N workgroups), the activation rows sit in LDS for the
    whole kernel, and every lane decodes its 64 codes with shifts and masks into int32 MACs.
    kernel(xq [M, K] int8, wq [N, Kp/4] uint8, s_x [M], s_w [N]) -> C [M, N] (dequantised)."""
    assert Kp % 256 == 0 and Kp >= K
    KB = 64  # bytes per row per step

    @T.prim_func
    def main(A: T.Tensor((M, K), "int8"), B: T.Tensor((N, Kp // 4), "uint8"), sx: T.Tensor((M, ), "float32"),
             sw: T.Tensor((N, ), "float32"), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), threads=64) as bx:
            x_s = T.alloc_shared((M, Kp), "int8")
            b_s = T.alloc_shared((block_N, KB), "uint8")
            b = T.alloc_fragment((block_N, KB), "uint8")
            acc = T.alloc_fragment((M, block_N, KB), "int32")
            row = T.alloc_fragment((M, block_N), "int32")
            for m, k in T.Parallel(M, Kp):
                x_s[m, k] = T.if_then_else(k < K, A[m, T.min(k, K - 1)], T.Cast("int8", 0))
            T.clear(acc)
            for ko in T.Pipelined(Kp // 256, num_stages=num_stages):
                T.copy(B[bx * block_N, ko * KB], b_s)
                T.copy(b_s, b)
                for m, n, j in T.Parallel(M, block_N, KB):
                    w = T.Cast("int32", b[n, j])
                    base = ko * 256 + 4 * j
                    acc[m, n, j] += ((w & 3) - zero) * T.Cast("int32", x_s[m, base]) + \
                        (((w >> 2) & 3) - zero) * T.Cast("int32", x_s[m, base + 1]) + \
                        (((w >> 4) & 3) - zero) * T.Cast("int32", x_s[m, base + 2]) + \
                        (((w >> 6) & 3) - zero) * T.Cast("int32", x_s[m, base + 3])
            T.reduce_sum(acc, row, dim=2)
            for m, n in T.Parallel(M, block_N):
                if bx * block_N + n < N:
                    C[m, bx * block_N + n] = T.Cast(out_dtype, T.Cast("float32", row[m, n]) /
                                                    (sx[m] * sw[bx * block_N + n]))

    return tilelang.compile(main, out_idx=[-1], target=target)


@functools.lru_cache(maxsize=None)
def rms_norm_quant_kernel(M, N, dtype, eps, target="hip", threads=128):
    """kernel(X [M,N], W [N]) -> (Xq int8 [M,N], s [M] fp32 = 127 / absmax(rmsnorm(x) * w)).
    One row per workgroup, the row in registers padded to a multiple of 4 * threads (any N: the
    BitNet-3B widths 3200 / 8640 are not powers of two), masked loads and stores."""
    Np = -(-N // (4 * threads)) * (4 * threads)

    @T.prim_func
    def main(X: T.Tensor((M, N), dtype), Wt: T.Tensor((N, ), dtype), Q: T.Tensor((M, N), "int8"),
             S: T.Tensor((M, ), "float32")):
        with T.Kernel(M, threads=threads) as bx:
            x = T.alloc_fragment((Np, ), "float32")
            sq = T.alloc_fragment((Np, ), "float32")
            ss = T.alloc_fragment((1, ), "float32")
            mx = T.alloc_fragment((1, ), "float32")
            for j in T.Parallel(Np):
                x[j] = T.if_then_else(j < N, T.Cast("float32", X[bx, T.min(j, N - 1)]), 0.0)
                sq[j] = x[j] * x[j]
            T.reduce_sum(sq, ss, dim=0)
            for j in T.Parallel(Np):
                # the model rounds the normalised activations to its dtype before the weight multiply
                x[j] = T.Cast("float32", T.Cast(dtype, T.Cast("float32", T.Cast(dtype, x[j] * T.rsqrt(
                    ss[0] / N + eps))) * T.Cast("float32", Wt[T.min(j, N - 1)])))
                sq[j] = T.if_then_else(j < N, T.abs(x[j]), 0.0)
            T.reduce_max(sq, mx, dim=0)
            for j in T.Parallel(Np):
                if j < N:
                    Q[bx, j] = T.Cast("int8", T.max(T.min(T.nearbyint(x[j] * (127.0 / T.max(mx[0], 1e-5))), 127.0),
                                                    -128.0))
            S[bx] = 127.0 / T.max(mx[0], 1e-5)

    return tilelang.compile(main, out_idx=[-2, -1], target=target)


def _target(t: torch.Tensor) -> str:
    return "cpu" if t.device.type == "cpu" else "hip"


def rms_norm_quant(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6):
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).contiguous()
    k = rms_norm_quant_kernel(x2.shape[0], x2.shape[1], _TDT[x2.dtype], float(eps), _target(x2))
    q, s = k(x2, weight.to(x2.dtype).contiguous())
    return q.reshape(shp), s.reshape(shp[:-1])


def int2_gemm(xq: torch.Tensor, wq: torch.Tensor, s_x: torch.Tensor = None, s_w: torch.Tensor = None,
              out_dtype=torch.float16, zero: int = 1) -> torch.Tensor:
    """xq [..., K] int8, wq [N, K/4] packed codes; raw int32 when s_x is None, else dequantised."""
    shp = xq.shape
    x2 = xq.reshape(-1, shp[-1]).contiguous()
    M, K = x2.shape
    N = wq.shape[0]
    if s_x is None:
        return int2_gemm_kernel(M, N, K, zero, "int32", _target(x2))(x2, wq).reshape(*shp[:-1], N)
    sw = s_w.reshape(-1).float().expand(N).contiguous()
    Kp = wq.shape[1] * 4
    if M <= 8 and Kp % 256 == 0:  # decode: weight streaming GEMV (packed K may be padded)
        k = int2_gemv_kernel(M, N, K, Kp, zero, _TDT[out_dtype], _target(x2))
    else:
        assert Kp == K, "padded packed weights need the GEMV path (M <= 8)"
        k = int2_gemm_kernel(M, N, K, zero, _TDT[out_dtype], _target(x2))
    return k(x2, wq, s_x.reshape(-1).float().contiguous(), sw).reshape(*shp[:-1], N)


# ------------------------------------------------------------------------------------------ host helpers


def pack_int2(codes: torch.Tensor) -> torch.Tensor:
    """[N, K] codes in 0..3 -> [N, K/4] uint8 (k = 4j + i in bits 2i..2i+1)."""
    c = codes.to(torch.uint8).reshape(codes.shape[0], -1, 4)
    return (c[..., 0] | (c[..., 1] << 2) | (c[..., 2] << 4) | (c[..., 3] << 6)).contiguous()


def unpack_int2(packed: torch.Tensor) -> torch.Tensor:
    p = packed.to(torch.int32)
    return torch.stack([(p >> (2 * i)) & 3 for i in range(4)], -1).reshape(packed.shape[0], -1)


def weight_quant_ternary(w: torch.Tensor):
    """utils_quant.weight_quant: s = 1 / mean|w|, q = clamp(round(w s), -1, 1).  Returns
    (packed codes q + 1 [N, K/4] uint8, s [1] fp32)."""
    wf = w.float()
    s = 1.0 / wf.abs().mean().clamp(min=1e-5)
    q = (wf * s).round().clamp(-1, 1)
    return pack_int2((q + 1).to(torch.int32)), s.reshape(1)


def activation_quant(x: torch.Tensor, num_bits: int = 8):
    """utils_quant.activation_quant split into (int8 values, per-token scale 127/absmax)."""
    qp = 2**(num_bits - 1) - 1
    xf = x.float()
    s = qp / xf.abs().amax(-1, keepdim=True).clamp(min=1e-5)
    return (xf * s).round().clamp(-qp - 1, qp).to(torch.int8), s.squeeze(-1)
