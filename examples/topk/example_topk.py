"""Row top-k selection (MoE router gates; reference: examples/topk/example_topk.py:16-60).

Every block holds ``blk_m`` rows of logits in registers.  For each of the ``topk`` rounds a
row max is found with a wave reduction, the (smallest) column that holds it is found with a
second (min) reduction over candidate indices, and that entry is knocked out.  Ties resolve
to the lowest index, matching ``torch.topk`` on distinct values.
"""
import argparse
import itertools

import tilelang
import tilelang.language as T


def get_configs():
    return [dict(blk_m=m, threads=t) for m, t in itertools.product([16, 32, 64], [64, 128, 256])]


@tilelang.jit(out_idx=[1, 2])
def tl_topk(M, N, topk, blk_m=16, threads=128, dtype="float32"):

    @T.prim_func
    def topk_kernel(
            logits: T.Tensor([M, N], dtype),
            topk_gates: T.Tensor([M, topk], dtype),
            topk_indices: T.Tensor([M, topk], "int32"),
    ):
        with T.Kernel(T.ceildiv(M, blk_m), threads=threads) as bx:
            vals = T.alloc_fragment([blk_m, N], dtype)
            cand = T.alloc_fragment([blk_m, N], "int32")
            max_val = T.alloc_fragment([blk_m], dtype)
            max_idx = T.alloc_fragment([blk_m], "int32")
            T.copy(logits[bx * blk_m, 0], vals)
            for k in T.serial(topk):
                T.reduce_max(vals, max_val, dim=1)
                for i, j in T.Parallel(blk_m, N):
                    cand[i, j] = T.if_then_else(vals[i, j] == max_val[i], j, N)
                T.reduce_min(cand, max_idx, dim=1)
                for i, j in T.Parallel(blk_m, N):
                    vals[i, j] = T.if_then_else(j == max_idx[i], -T.infinity(dtype), vals[i, j])
                for i in T.Parallel(blk_m):
                    topk_gates[bx * blk_m + i, k] = max_val[i]
                    topk_indices[bx * blk_m + i, k] = max_idx[i]

    return topk_kernel


def ref_program(logits, top_k):
    import torch
    g, i = logits.topk(top_k, dim=1)
    return g, i.to(torch.int32)


def main(M=320, N=128, topk=6, blk_m=16):
    import torch
    logits = torch.rand((M, N), device="cuda", dtype=torch.float32)
    kernel = tl_topk(M, N, topk, blk_m)
    g, i = kernel(logits)
    rg, ri = ref_program(logits, topk)
    torch.testing.assert_close(g, rg)
    torch.testing.assert_close(i, ri)
    print("All checks pass.")
    print(f"topk latency: {kernel.get_profiler().do_bench(lambda: kernel(logits)):.4f} ms")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--M", type=int, default=320)
    p.add_argument("--N", type=int, default=128)
    p.add_argument("--topk", type=int, default=6)
    a = p.parse_args()
    main(a.M, a.N, a.topk)
