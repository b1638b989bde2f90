"""Fused RMSNorm (reference counterpart: examples/norm/rms_norm.py and the model's ``RMSNorm``)."""
from __future__ import annotations

import functools

import torch

import tilelang
import tilelang.language as T


@functools.lru_cache(maxsize=None)
def _rms_kernel_padded(M, N, dtype, eps, target, threads=128):
    """Widths that do not tile over the block (e.g. 3200): one row per workgroup, the row padded
    to a multiple of 4 * threads in registers, masked loads and stores."""
    Np = -(-N // (4 * threads)) * (4 * threads)

    @T.prim_func
    def main(X: T.Tensor((M, N), dtype), Wt: T.Tensor((N, ), dtype), Y: T.Tensor((M, N), dtype)):
        with T.Kernel(M, threads=threads) as bx:
            x = T.alloc_fragment((Np, ), "float32")
            sq = T.alloc_fragment((Np, ), "float32")
            ss = T.alloc_fragment((1, ), "float32")
            for j in T.Parallel(Np):
                x[j] = T.if_then_else(j < N, T.Cast("float32", X[bx, T.min(j, N - 1)]), 0.0)
                sq[j] = x[j] * x[j]
            T.reduce_sum(sq, ss, dim=0)
            for j in T.Parallel(Np):
                if j < N:
                    Y[bx, j] = T.Cast(dtype, x[j] * T.rsqrt(ss[0] / N + eps) * T.Cast("float32", Wt[j]))

    return tilelang.compile(main, out_idx=[-1], target=target)


@functools.lru_cache(maxsize=None)
def _rms_kernel(M, N, dtype, eps, target):
    if N % 1024:
        return _rms_kernel_padded(M, N, dtype, eps, target)
    blk_m = 4 if N <= 8192 else 1
    threads = 256

    @T.prim_func
    def main(X: T.Tensor((M, N), dtype), Wt: T.Tensor((N, ), dtype), Y: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(M, blk_m), threads=threads) as bx:
            x = T.alloc_fragment((blk_m, N), "float32")
            sq = T.alloc_fragment((blk_m, N), "float32")
            ss = T.alloc_fragment((blk_m, ), "float32")
            y = T.alloc_fragment((blk_m, N), dtype)
            T.copy(X[bx * blk_m, 0], x)
            for i, j in T.Parallel(blk_m, N):
                sq[i, j] = x[i, j] * x[i, j]
            T.reduce_sum(sq, ss, dim=1)
            for i in T.Parallel(blk_m):
                ss[i] = T.rsqrt(ss[i] / N + eps)
            for i, j in T.Parallel(blk_m, N):
                y[i, j] = x[i, j] * ss[i] * Wt[j]
            T.copy(y, Y[bx * blk_m, 0])

    return tilelang.compile(main, out_idx=[-1], target=target)


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).contiguous()
    M, N = x2.shape
    dt = {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[x2.dtype]
    k = _rms_kernel(M, N, dt, float(eps), "cpu" if x2.device.type == "cpu" else "hip")
    return k(x2, weight.to(x2.dtype).contiguous()).reshape(shp)
