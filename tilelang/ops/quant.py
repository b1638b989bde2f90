"""Per-group fp8 activation quantisation (reference: examples/deepseek_v32/inference/kernel.py ``act_quant``,
examples/cast/example_per_token_cast_to_fp8.py).  OCP e4m3 (gfx950-native), 448 max, fp32 scales."""
from __future__ import annotations

import functools

import torch

import tilelang
import tilelang.language as T

FP8_MAX = 448.0


@functools.lru_cache(maxsize=None)
def _act_quant_kernel(M, N, group, dtype, target, pow2_scale):
    blk_m = 8
    threads = 128

    @T.prim_func
    def main(X: T.Tensor((M, N), dtype), Y: T.Tensor((M, N), "float8_e4m3fn"),
             S: T.Tensor((M, N // group), "float32")):
        with T.Kernel(T.ceildiv(M, blk_m), N // group, threads=threads) as (bx, by):
            x = T.alloc_fragment((blk_m, group), "float32")
            amax = T.alloc_fragment((blk_m, ), "float32")
            sc = T.alloc_fragment((blk_m, ), "float32")
            q = T.alloc_fragment((blk_m, group), "float8_e4m3fn")
            T.copy(X[bx * blk_m, by * group], x)
            T.reduce_absmax(x, amax, dim=1)
            for i in T.Parallel(blk_m):
                if pow2_scale:
                    # ue8m0 scales (power of two), as the DeepSeek-V3.2 checkpoint format
                    sc[i] = T.exp2(T.ceil(T.log2(T.max(amax[i], 1e-4) / FP8_MAX)))
                else:
                    sc[i] = T.max(amax[i], 1e-4) / FP8_MAX
            for i, j in T.Parallel(blk_m, group):
                q[i, j] = T.clamp(x[i, j] / sc[i], -FP8_MAX, FP8_MAX)
            for i in T.Parallel(blk_m):
                S[bx * blk_m + i, by] = sc[i]
            T.copy(q, Y[bx * blk_m, by * group])

    return tilelang.compile(main, out_idx=[1, 2], target=target)


def act_quant(x: torch.Tensor, group: int = 128, pow2_scale: bool = False):
    """x [..., N] -> (fp8 [..., N], scales [..., N/group])."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).contiguous()
    M, N = x2.shape
    dt = {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[x2.dtype]
    k = _act_quant_kernel(M, N, group, dt, "cpu" if x2.device.type == "cpu" else "hip", bool(pow2_scale))
    y, s = k(x2)
    return y.reshape(shp), s.reshape(*shp[:-1], N // group)
