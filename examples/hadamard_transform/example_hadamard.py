"""Fast Walsh-Hadamard transform along the last dim (reference: examples/hadamard_transform/example_hadamard.py).

B[b, :] = A[b, :] @ H_n (Sylvester order, unnormalised), n a power of two <= 32768.  One block
per row: the row is staged in LDS (n*4 B <= 128 KiB of the 160 KiB per CU), and each of the
log2(n) butterfly stages is a ``T.Parallel`` over the n/2 disjoint pairs (every lane reads
its pair and writes both results in place; the compiler's barrier insertion separates the
stages).
"""
import argparse
import math

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[1])
def hadamard(b, n, dtype="float32", threads=256):
    assert n > 1 and n & (n - 1) == 0, "n must be a power of 2"
    logn = int(math.log2(n))
    half = n // 2

    @T.prim_func
    def main(A: T.Tensor((b, n), dtype), B: T.Tensor((b, n), dtype)):
        with T.Kernel(b, threads=threads) as bx:
            s = T.alloc_shared((n, ), "float32")
            for i in T.Parallel(n):
                s[i] = A[bx, i]
            for r in range(logn):
                h = 1 << r
                for p in T.Parallel(half):
                    lo = (p // h) * (2 * h) + p % h
                    x = s[lo]
                    y = s[lo + h]
                    s[lo] = x + y
                    s[lo + h] = x - y
            for i in T.Parallel(n):
                B[bx, i] = s[i]

    return main


def ref_program(x):
    import torch
    n = x.shape[-1]
    H = torch.ones(1, 1, dtype=torch.float64)
    while H.shape[0] < n:
        H = torch.cat([torch.cat([H, H], 1), torch.cat([H, -H], 1)], 0)
    return (x.double() @ H.to(x.device)).to(x.dtype)


def main(batch=64, dim=32768):
    import torch
    kernel = hadamard(batch, dim)
    x = torch.randn(batch, dim, device="cuda")
    torch.testing.assert_close(kernel(x), ref_program(x), rtol=1e-3, atol=1e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(x))
    print(f"hadamard {batch}x{dim}: {lat:.4f} ms")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--dim", type=int, default=32768)
    a = p.parse_args()
    main(a.batch, a.dim)
