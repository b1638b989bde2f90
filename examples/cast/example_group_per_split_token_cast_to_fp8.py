"""Grouped per-token fp8 cast for MoE expert batches
(reference: examples/cast/example_group_per_split_token_cast_to_fp8.py:12-62).

X [M, N] bf16 holds the tokens of BG experts back to back (``batch_sizes[g]`` rows each).  The
output is padded per expert: X_fp8 [BG, M_max, N] OCP e4m3fn plus one fp32 scale per
(expert, row, 128-column group) in X_s [BG, M_max, N / 128]; rows past ``batch_sizes[g]`` are
written as zeros (scale 0), so a grouped GEMM can run over the padded batch.

One block per (row tile, 128-column group, expert).  The expert's first row is a prefix sum over
``batch_sizes`` (BG is small: a scalar loop, no extra launch).  Reads past the expert are clamped
to a valid row and masked, so the kernel never touches memory beyond X.
"""
import argparse

import tilelang
import tilelang.language as T

FP8_MAX = 448.0


@tilelang.jit(out_idx=[2, 3])
def group_per_split_token_cast_to_fp8(M, M_max, N, BG, blk_m=8, group_size=128, threads=128, dtype="bfloat16"):
    assert N % group_size == 0

    @T.prim_func
    def group_cast(X: T.Tensor((M, N), dtype), batch_sizes: T.Tensor((BG, ), "int32"),
                   X_fp8: T.Tensor((BG, M_max, N), "float8_e4m3fn"),
                   X_s: T.Tensor((BG, M_max, N // group_size), "float32")):
        with T.Kernel(T.ceildiv(M_max, blk_m), N // group_size, BG, threads=threads) as (bx, by, bz):
            y = T.alloc_fragment((blk_m, group_size), "float32")
            amax = T.alloc_fragment((blk_m, ), "float32")
            scale = T.alloc_fragment((blk_m, ), "float32")
            inv = T.alloc_fragment((blk_m, ), "float32")
            q = T.alloc_fragment((blk_m, group_size), "float8_e4m3fn")
            start = T.alloc_local((1, ), "int32")
            start[0] = 0
            for g in T.serial(bz):
                start[0] += batch_sizes[g]
            n_rows = batch_sizes[bz]
            for i, j in T.Parallel(blk_m, group_size):
                y[i, j] = T.if_then_else(bx * blk_m + i < n_rows,
                                         X[T.min(start[0] + bx * blk_m + i, M - 1), by * group_size + j], 0.0)
            T.reduce_absmax(y, amax, dim=1)
            for i in T.Parallel(blk_m):
                scale[i] = T.if_then_else(bx * blk_m + i < n_rows, T.max(amax[i], 1e-4) / FP8_MAX, 0.0)
                inv[i] = FP8_MAX / T.max(amax[i], 1e-4)
            for i, j in T.Parallel(blk_m, group_size):
                q[i, j] = T.if_then_else(bx * blk_m + i < n_rows, T.clamp(y[i, j] * inv[i], -FP8_MAX, FP8_MAX), 0.0)
            for i in T.Parallel(blk_m):
                if bx * blk_m + i < M_max:
                    X_s[bz, bx * blk_m + i, by] = scale[i]
            for i, j in T.Parallel(blk_m, group_size):
                if bx * blk_m + i < M_max:
                    X_fp8[bz, bx * blk_m + i, by * group_size + j] = q[i, j]

    return group_cast


def ref_program(x, batch_sizes, M_max, group_size=128):
    import torch
    BG, N = batch_sizes.numel(), x.shape[1]
    q = torch.zeros(BG, M_max, N, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.zeros(BG, M_max, N // group_size, dtype=torch.float32, device=x.device)
    start = 0
    for g, n in enumerate(batch_sizes.tolist()):
        xv = x[start:start + n].float().view(n, N // group_size, group_size)
        amax = xv.abs().amax(dim=2).clamp(1e-4)
        q[g, :n] = (xv * (FP8_MAX / amax.unsqueeze(2))).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).view(n, N)
        s[g, :n] = amax / FP8_MAX
        start += n
    return q, s


def main(BG=8, M_per=2048, N=7168, blk_m=8):
    import torch
    sizes = torch.randint(M_per // 2, M_per, (BG, )).tolist()
    M, M_max = sum(sizes), max(sizes)
    x = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    bs = torch.tensor(sizes, dtype=torch.int32, device="cuda")
    kernel = group_per_split_token_cast_to_fp8(M, M_max, N, BG, blk_m)
    q, s = kernel(x, bs)
    rq, rs = ref_program(x, bs, M_max)
    torch.testing.assert_close(s, rs, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(q.float(), rq.float(), rtol=0.13, atol=0.01)  # one e4m3 ulp (rounding ties)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(x, bs))
    nbytes = M * N * 2 + BG * M_max * N * (1 + 4 / 128)
    print(f"group cast BG={BG} M={M} N={N}: {lat:.4f} ms, {nbytes / lat * 1e-9:.2f} TB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--bg", type=int, default=8)
    p.add_argument("--m", type=int, default=2048)
    p.add_argument("--n", type=int, default=7168)
    a = p.parse_args()
    main(a.bg, a.m, a.n)
