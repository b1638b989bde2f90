"""Block-scaled fp8 linear layers (reference ``examples/deepseek_v32/inference/kernel.py:36-268``:
``act_quant`` + ``fp8_gemm``; checkpoint format of DeepSeek-V3.x: fp8 weights with one fp32 scale
per 128x128 block, activations quantised per token and 128-wide K group at run time).

``fp8_linear(x, w_fp8, w_scale)`` = dequant(act_quant(x)) @ dequant(w)^T in bf16:

    C[m, n] = sum_kb  sa[m, kb] * sw[n // 128, kb] * (A[m, kb] . W[n, kb])        (kb: 128-wide K group)

gfx950 schedule: one K step = one 128-wide scale group = one ``v_mfma_scale_f32_16x16x128_f8f6f4``
per 16x16 accumulator tile (OCP e4m3, unit e8m0 MFMA scales -- the fp32 group scales are not
powers of two), the raw partial promoted into a second fp32 accumulator with the (row scale x
column-block scale) product every step ("2xAcc", as the reference and DeepGEMM), operands and
scales staged by the LDS-DMA pipeline.  Tiles follow M: decode-sized calls (M <= 64) use a
64-row tile so the N dimension alone fills the CUs.
"""
from __future__ import annotations

import functools
from typing import Tuple

import torch

import tilelang
import tilelang.language as T

GROUP = 128
FP8_MAX = 448.0


def _tdt(dtype: torch.dtype) -> str:
    return {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[dtype]


@functools.lru_cache(maxsize=None)
def fp8_gemm_kernel(M: int, N: int, K: int, out_dtype: str = "bfloat16", target: str = "hip"):
    assert K % GROUP == 0, "fp8 block-scaled GEMM needs K % 128 == 0"
    block_M = 64 if M <= 64 else 128
    block_N = 128
    threads = 256
    KG = K // GROUP
    NG = (N + GROUP - 1) // GROUP

    @T.prim_func
    def fp8_gemm(A: T.Tensor((M, K), "float8_e4m3fn"), W: T.Tensor((N, K), "float8_e4m3fn"),
                 sa: T.Tensor((M, KG), "float32"), sw: T.Tensor((NG, KG), "float32"),
                 C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, GROUP), "float8_e4m3fn")
            W_s = T.alloc_shared((block_N, GROUP), "float8_e4m3fn")
            s_s = T.alloc_shared((block_M, ), "float32")
            part = T.alloc_fragment((block_M, block_N), "float32")
            acc = T.alloc_fragment((block_M, block_N), "float32")
            T.use_swizzle(panel_size=8)
            T.clear(acc)
            for k in T.Pipelined(KG, num_stages=2):
                T.copy(A[by * block_M, k * GROUP], A_s)
                T.copy(W[bx * block_N, k * GROUP], W_s)
                for i in T.Parallel(block_M):
                    # block_N == GROUP: one weight scale per (column block, K group)
                    s_s[i] = sa[T.min(by * block_M + i, M - 1), k] * sw[bx, k]
                T.gemm(A_s, W_s, part, transpose_B=True, clear_accum=True)
                for i, j in T.Parallel(block_M, block_N):
                    acc[i, j] += part[i, j] * s_s[i]
            T.copy(acc, C[by * block_M, bx * block_N])

    return tilelang.compile(fp8_gemm, target=target)


def weight_quant(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """[N, K] -> (fp8 e4m3 [N, K], fp32 scales [ceil(N/128), ceil(K/128)]), one scale per 128x128
    block (the DeepSeek-V3.x checkpoint format; the reference's ``convert.py`` keeps it as is)."""
    N, K = w.shape
    nb, kb = -(-N // GROUP), -(-K // GROUP)
    wp = torch.zeros(nb * GROUP, kb * GROUP, dtype=torch.float32, device=w.device)
    wp[:N, :K] = w.float()
    blocks = wp.view(nb, GROUP, kb, GROUP)
    amax = blocks.abs().amax(dim=(1, 3), keepdim=True).clamp_min(1e-4)
    q = (blocks * (FP8_MAX / amax)).to(torch.float8_e4m3fn).view(nb * GROUP, kb * GROUP)[:N, :K].contiguous()
    return q, (amax / FP8_MAX).view(nb, kb).contiguous()


def weight_dequant(w_fp8: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    N, K = w_fp8.shape
    s = scale.repeat_interleave(GROUP, 0).repeat_interleave(GROUP, 1)[:N, :K]
    return w_fp8.float() * s


def fp8_gemm(a: torch.Tensor, a_s: torch.Tensor, w: torch.Tensor, w_s: torch.Tensor,
             out_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """a [..., K] fp8 with per-(row, 128-group) scales a_s [..., K/128]; w [N, K] fp8 with
    128x128 block scales w_s -> [..., N] in ``out_dtype``."""
    K = a.shape[-1]
    a2 = a.reshape(-1, K).contiguous()
    M, N = a2.shape[0], w.shape[0]
    k = fp8_gemm_kernel(M, N, K, _tdt(out_dtype), "cpu" if a2.device.type == "cpu" else "hip")
    out = torch.empty(M, N, dtype=out_dtype, device=a2.device)
    k(a2, w, a_s.reshape(M, -1).contiguous(), w_s.contiguous(), out)
    return out.reshape(*a.shape[:-1], N)


def fp8_linear(x: torch.Tensor, w: torch.Tensor, w_s: torch.Tensor, pow2_scale: bool = False) -> torch.Tensor:
    """The reference model's ``linear`` for fp8 weights: per-token group quantisation of the
    activations (``ops.quant.act_quant``), then the block-scaled fp8 GEMM, bf16 out."""
    from .quant import act_quant
    xq, xs = act_quant(x.contiguous(), GROUP, pow2_scale)
    return fp8_gemm(xq, xs, w, w_s, x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.bfloat16)
