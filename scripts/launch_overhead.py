"""Host-side launch overhead of a JITKernel call (tiny kernel, 2000 back-to-back calls) vs a
torch op, on the GPU.  python scripts/launch_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tilelang  # noqa: E402
import tilelang.language as T  # noqa: E402


@tilelang.jit(out_idx=[-1])
def add(n):
    @T.prim_func
    def main(A: T.Tensor((n, ), "float32"), B: T.Tensor((n, ), "float32"), C: T.Tensor((n, ), "float32")):
        with T.Kernel(n // 256, threads=256) as bx:
            for i in T.Parallel(256):
                C[bx * 256 + i] = A[bx * 256 + i] + B[bx * 256 + i]
    return main


def bench(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    cpu = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / n * 1e6
    return cpu, wall


a = torch.randn(4096, device="cuda")
b = torch.randn(4096, device="cuda")
k = add(4096)
c = torch.empty_like(a)
print("JITKernel (allocating output): host %.1f us/call, wall %.1f us/call" % bench(lambda: k(a, b)))
print("torch.add (allocating output): host %.1f us/call, wall %.1f us/call" % bench(lambda: torch.add(a, b)))
print("torch.add(out=):               host %.1f us/call, wall %.1f us/call" % bench(lambda: torch.add(a, b, out=c)))
