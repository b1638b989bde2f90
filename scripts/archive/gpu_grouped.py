"""Grouped GEMM: correctness sweep + MoE-shaped perf vs a per-expert hipBLASLt loop."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "grouped_gemm"))
import torch
from example_grouped_gemm_fwd import grouped_gemm, construct_inputs, torch_gmm
from tilelang.profiler import do_bench


torch.manual_seed(0)
E, T_, K, N = 8, 8192, 4096, 14336
sizes = [T_ // E] * E
sizes[0] += 100; sizes[1] -= 100
for (bm, bn, bk, st, th) in [(128, 128, 64, 2, 256), (256, 256, 64, 2, 512), (256, 128, 64, 2, 256), (128, 256, 64, 2, 256), (256, 256, 64, 3, 512), (256, 256, 32, 3, 512)]:
    try:
        k = grouped_gemm(tuple(sizes), K, N, bm, bn, bk, st, th, "float16", True)
        A, B, bs, bo, bpo = construct_inputs(sizes, K, N, True, bm)
        out = k(A, B, bs, bo, bpo)
        n2 = sizes[0] + sizes[1]
        ref = torch_gmm(A[:n2], B[:2], sizes[:2], True)
        torch.testing.assert_close(out[:n2], ref, rtol=2e-2, atol=2e-1)
        ms = do_bench(lambda: k(A, B, bs, bo, bpo), warmup=20, rep=100)
        tf = 2 * sum(sizes) * K * N / ms * 1e-9
        print(f"tilelang grouped {bm}x{bn}x{bk} s{st} t{th}: {ms:.3f} ms {tf:.1f} TF", flush=True)
    except Exception as e:
        print("cfg fail", bm, bn, bk, st, th, repr(e)[:300], flush=True)
A, B, bs, bo, bpo = construct_inputs(sizes, K, N, True, 128)
def loop():
    s = 0
    outs = []
    for i, m in enumerate(sizes):
        outs.append(A[s:s + m] @ B[i].t())
        s += m
    return outs
ms = do_bench(loop, warmup=20, rep=100)
print(f"torch per-expert loop: {ms:.3f} ms {2*sum(sizes)*K*N/ms*1e-9:.1f} TF")
