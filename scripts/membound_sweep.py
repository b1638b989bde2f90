"""Memory-bound kernels on one MI355X: configuration sweep vs a plain copy (the practical HBM
ceiling) and PyTorch, cold-cache do_bench (512 MiB flush), one process.

    python scripts/membound_sweep.py [--quick]
"""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
for d in ("elementwise", "norm", "gemv", "cast"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402


def tbs(nbytes, ms):
    return nbytes / ms * 1e-9


def bench(fn, reps=3):
    return min(do_bench(fn, warmup=10, rep=50) for _ in range(reps))


def sweep(name, nbytes, builds, ref=None, check=None):
    res = []
    for label, make in builds:
        try:
            k = make()
            if check is not None:
                check(k)
            res.append((label, bench(k)))
        except Exception as e:  # noqa: BLE001
            print(f"  {name} {label}: failed {type(e).__name__}: {str(e)[:200]}", flush=True)
    res.sort(key=lambda r: r[1])
    for label, ms in res[:5]:
        print(f"  {name} {label}: {ms:.4f} ms {tbs(nbytes, ms):.2f} TB/s", flush=True)
    if ref is not None:
        ms = bench(ref)
        print(f"  {name} torch: {ms:.4f} ms {tbs(nbytes, ms):.2f} TB/s", flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    M = N = 8192
    x = torch.randn(M, N, device="cuda")
    y = torch.randn(M, N, device="cuda")
    out = torch.empty_like(x)
    ms = bench(lambda: out.copy_(x))
    print(f"copy fp32 {M}x{N}: {ms:.4f} ms {tbs(2 * x.numel() * 4, ms):.2f} TB/s (ceiling reference)", flush=True)

    from example_elementwise_add import elementwise_add
    cfgs = [(32, 256, 256), (16, 512, 256), (64, 256, 256), (32, 512, 256), (64, 512, 512), (128, 256, 512),
            (32, 1024, 256), (64, 1024, 512), (16, 1024, 128)]
    if a.quick:
        cfgs = cfgs[:3]

    def add_k(bm, bn, t, nt=True):
        k = elementwise_add(M, N, bm, bn, t, nt=nt)
        return lambda: k(x, y)

    def add_check(fn):
        torch.testing.assert_close(fn(), x + y)

    print("elementwise add fp32 8192^2 (3 x 256 MiB)", flush=True)
    sweep("add", 3 * x.numel() * 4, [(f"{c} nt={nt}", (lambda c=c, nt=nt: add_k(*c, nt=nt))) for c in cfgs
                                     for nt in (True, False)], lambda: torch.add(x, y),
          add_check)

    from rms_norm import rms_norm
    cfgs = [(1, 256), (1, 512), (1, 1024), (2, 512), (2, 1024), (4, 1024), (4, 256), (8, 1024)]

    def rms_k(bm, t, nt=True):
        k = rms_norm(M, N, bm, t, nt=nt)
        return lambda: k(x)

    def rms_ref():
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-12)

    print("rms norm fp32 8192^2 (2 x 256 MiB)", flush=True)
    sweep("rms", 2 * x.numel() * 4, [(f"{c} nt={nt}", (lambda c=c, nt=nt: rms_k(*c, nt=nt))) for c in cfgs
                                     for nt in (True, False)], rms_ref,
          lambda fn: torch.testing.assert_close(fn(), rms_ref(), rtol=1e-4, atol=1e-4))

    from example_gemv import gemv
    NG = KG = 16384
    A = torch.randn(NG, KG, device="cuda", dtype=torch.float16)
    xv = torch.randn(KG, device="cuda", dtype=torch.float16)
    cfgs = [(8, 512, 256), (8, 1024, 256), (8, 2048, 256), (4, 2048, 256), (16, 1024, 256), (4, 4096, 256),
            (2, 4096, 256), (8, 2048, 512), (16, 2048, 512)]

    def gemv_k(bn, bk, t, nt=True):
        k = gemv(NG, KG, bn, bk, t, nt=nt)
        return lambda: k(A, xv)

    print("gemv fp16 16384^2 (512 MiB of weights)", flush=True)
    sweep("gemv", A.numel() * 2, [(f"{c} nt={nt}", (lambda c=c, nt=nt: gemv_k(*c, nt=nt))) for c in cfgs
                                  for nt in (True, False)], lambda: A @ xv,
          lambda fn: torch.testing.assert_close(fn().float(), (A.float() @ xv.float()), rtol=2e-2, atol=2e-1))

    from example_per_token_cast_to_fp8 import per_token_cast_to_fp8
    xh = torch.randn(M, N, device="cuda")
    cfgs = [(8, 128, 1), (8, 128, 4), (8, 256, 4), (16, 256, 2), (4, 256, 8), (8, 256, 8), (16, 512, 4),
            (32, 256, 1), (8, 512, 8)]

    def cast_k(bm, t, g, nt=True):
        k = per_token_cast_to_fp8(M, N, bm, 128, t, g, nt=nt)
        return lambda: k(xh)

    print("per-token(group 128) fp8 cast fp32 8192^2 (256 MiB in, 64 MiB + scales out)", flush=True)
    sweep("cast", xh.numel() * 5 + M * (N // 128) * 4, [(f"{c} nt={nt}", (lambda c=c, nt=nt: cast_k(*c, nt=nt)))
                                                         for c in cfgs for nt in (True, False)])


if __name__ == "__main__":
    main()
