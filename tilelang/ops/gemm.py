"""``linear(x, w)`` = x @ w^T on MFMA (f16 / bf16: 16x16x32; fp32: the exact-f32 16x16x4 form)
(reference counterpart: examples/deepseek_v32/inference/kernel.py ``fp8_gemm`` / the model's
``linear``).  One compiled kernel per (M, N, K, dtype, target); the
tile is chosen by M so decode-sized (skinny) and prefill-sized GEMMs both fill the CUs."""
from __future__ import annotations

import functools

import torch

import tilelang
import tilelang.language as T


def _tdt(dtype: torch.dtype) -> str:
    return {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[dtype]


def _tiles(M: int, N: int, K: int, dtype: str = "float16"):
    if dtype == "float32":
        # exact-f32 MFMA (v_mfma_f32_16x16x4_f32, tl::gemm_ss_f32): fp32 tiles are twice the
        # bytes, so keep the 128x128 tile at BK=32 (2 x 16 KiB per stage)
        bm = 64 if M <= 64 else 128
        bn = 64 if N <= 256 else 128
        return bm, bn, 32, 256
    bm = 64 if M <= 64 else (128 if M <= 2048 else 256)
    bn = 64 if N <= 256 else 128 if M <= 2048 else 256
    bk = 64 if K % 64 == 0 else 32
    threads = 256 if bm * bn <= 128 * 128 else 512
    return bm, bn, bk, threads


@functools.lru_cache(maxsize=None)
def _linear_kernel(M, N, K, dtype, target):
    bm, bn, bk, threads = _tiles(M, N, K, dtype)

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), W: T.Tensor((N, K), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=threads) as (bx, by):
            A_s = T.alloc_shared((bm, bk), dtype)
            W_s = T.alloc_shared((bn, bk), dtype)
            acc = T.alloc_fragment((bm, bn), "float")
            out = T.alloc_fragment((bm, bn), dtype)
            T.use_swizzle(panel_size=8)
            T.clear(acc)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=2):
                T.copy(A[by * bm, k * bk], A_s)
                T.copy(W[bx * bn, k * bk], W_s)
                T.gemm(A_s, W_s, acc, transpose_B=True)
            T.copy(acc, out)
            T.copy(out, C[by * bm, bx * bn])

    return tilelang.compile(main, out_idx=[-1], target=target)


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [..., K] @ w[N, K]^T -> [..., N] in x's dtype (fp32 accumulation)."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).contiguous()
    M, K = x2.shape
    N = w.shape[0]
    w2 = w.contiguous()
    if w2.dtype != x2.dtype:
        raise TypeError(f"linear: x is {x2.dtype} but w is {w2.dtype}")
    if K % 32:
        # the MFMA K step is 32 (f16/bf16) / 4 (f32) and tiles are staged 16 bytes at a time:
        # zero-pad K (exact: the padded products are 0) instead of leaving the MFMA path
        pad = (-K) % 32
        x2 = torch.nn.functional.pad(x2, (0, pad))
        w2 = torch.nn.functional.pad(w2, (0, pad))
        K += pad
    k = _linear_kernel(M, N, K, _tdt(x2.dtype), "cpu" if x2.device.type == "cpu" else "hip")
    return k(x2, w2).reshape(*shp[:-1], N)


@functools.lru_cache(maxsize=None)
def _head_bmm_kernel(M, H, N, K, dtype, target):
    bm, bn, bk, threads = _tiles(M, N, K, dtype)

    @T.prim_func
    def main(A: T.Tensor((M, H, K), dtype), W: T.Tensor((H, N, K), dtype), C: T.Tensor((M, H, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), H, threads=threads) as (bx, by, h):
            A_s = T.alloc_shared((bm, bk), dtype)
            W_s = T.alloc_shared((bn, bk), dtype)
            acc = T.alloc_fragment((bm, bn), "float")
            out = T.alloc_fragment((bm, bn), dtype)
            T.clear(acc)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=2):
                T.copy(A[by * bm:(by + 1) * bm, h, k * bk:(k + 1) * bk], A_s)
                T.copy(W[h, bx * bn:(bx + 1) * bn, k * bk:(k + 1) * bk], W_s)
                T.gemm(A_s, W_s, acc, transpose_B=True)
            T.copy(acc, out)
            T.copy(out, C[by * bm:(by + 1) * bm, h, bx * bn:(bx + 1) * bn])

    return tilelang.compile(main, out_idx=[-1], target=target)


def head_bmm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Per-head GEMM: x [..., H, K] and w [H, N, K] -> [..., H, N], out[..., h, :] = x[..., h, :] @ w[h]^T
    (MFMA, fp32 accumulation).  The absorbed MLA projections (query x W_uk, latent output x W_uv:
    reference examples/deepseek_v32/inference/model.py:625-642) are this shape: one launch over
    every head instead of a per-head loop or an fp32 einsum."""
    shp = x.shape
    H, N, K = w.shape
    if shp[-2] != H or shp[-1] != K:
        raise ValueError(f"head_bmm: x {tuple(shp)} does not match w {tuple(w.shape)}")
    if w.dtype != x.dtype:
        raise TypeError(f"head_bmm: x is {x.dtype} but w is {w.dtype}")
    x3 = x.reshape(-1, H, K).contiguous()
    w3 = w.contiguous()
    if K % 32:
        pad = (-K) % 32
        x3 = torch.nn.functional.pad(x3, (0, pad))
        w3 = torch.nn.functional.pad(w3, (0, pad))
        K += pad
    k = _head_bmm_kernel(x3.shape[0], H, N, K, _tdt(x3.dtype), "cpu" if x3.device.type == "cpu" else "hip")
    return k(x3, w3).reshape(*shp[:-1], N)
