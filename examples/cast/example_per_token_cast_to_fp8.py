"""Per-token-group fp8 quantisation (reference: examples/cast/example_per_token_cast_to_fp8.py:8-50).

X [M, N] fp32 -> X_fp8 [M, N] OCP e4m3fn (the gfx950-native fp8, max 448) plus one fp32
scale per (row, 128-column group): ``s = max(amax, 1e-4) / 448``, ``q = clamp(x / s)``.
The group tile is read once into registers, its |x| max is a wave reduction, and the fp8
tile is written with packed conversions.
"""
import argparse

import tilelang
import tilelang.language as T

FP8_MAX = 448.0


@tilelang.jit(out_idx=[1, 2])
def per_token_cast_to_fp8(M, N, blk_m=8, group_size=128, threads=128, groups=1, nt=True):
    """``groups``: 128-column groups per block (one block reads ``blk_m x groups*128``); ``nt``: the
    input is streamed once (non-temporal loads and stores)."""
    dtype = "float32"
    gw = groups * group_size
    assert N % gw == 0

    @T.prim_func
    def per_token_cast(X: T.Tensor((M, N), dtype), X_fp8: T.Tensor((M, N), "float8_e4m3fn"),
                       X_amax: T.Tensor((M, T.ceildiv(N, group_size)), dtype)):
        with T.Kernel(T.ceildiv(M, blk_m), N // gw, threads=threads) as (bx, by):
            y = T.alloc_fragment((blk_m, groups, group_size), dtype)
            amax = T.alloc_fragment((blk_m, groups), dtype)
            scale = T.alloc_fragment((blk_m, groups), dtype)
            q = T.alloc_fragment((blk_m, groups, group_size), "float8_e4m3fn")
            if nt:
                T.annotate_nontemporal(X, X_fp8)
            for i, g, j in T.Parallel(blk_m, groups, group_size):
                y[i, g, j] = X[bx * blk_m + i, by * gw + g * group_size + j]
            T.reduce_absmax(y, amax, dim=2)
            for i, g in T.Parallel(blk_m, groups):
                scale[i, g] = T.max(amax[i, g], 1e-4) / FP8_MAX
            for i, g, j in T.Parallel(blk_m, groups, group_size):
                q[i, g, j] = T.clamp(y[i, g, j] / scale[i, g], -FP8_MAX, FP8_MAX)
            for i, g in T.Parallel(blk_m, groups):
                X_amax[bx * blk_m + i, by * groups + g] = scale[i, g]
            for i, g, j in T.Parallel(blk_m, groups, group_size):
                X_fp8[bx * blk_m + i, by * gw + g * group_size + j] = q[i, g, j]

    return per_token_cast


def ref_program(x, group_size=128):
    import torch
    m, n = x.shape
    xv = x.view(m, -1, group_size)
    amax = xv.abs().float().amax(dim=2).clamp(1e-4)
    q = (xv * (FP8_MAX / amax.unsqueeze(2))).to(torch.float8_e4m3fn).view(m, n)
    return q, amax / FP8_MAX


def main(M=8192, N=8192, blk_m=8):
    import torch
    kernel = per_token_cast_to_fp8(M, N, blk_m)
    x = torch.randn(M, N, device="cuda")
    q, s = kernel(x)
    rq, rs = ref_program(x)
    torch.testing.assert_close(q.float(), rq.float(), rtol=0.07, atol=0.01)
    torch.testing.assert_close(s, rs, rtol=1e-5, atol=1e-7)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(x))
    print(f"per-token cast {M}x{N}: {lat:.4f} ms, {M * N * 5 / lat * 1e-6:.1f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=8192)
    p.add_argument("--n", type=int, default=8192)
    a = p.parse_args()
    main(a.m, a.n)
