"""Same-process A/B of the NT GEMM main-loop schedules of examples/gemm/example_gemm.py
(256x256x64 tile, 512 threads): ``tl::gemm_quad_nt`` (tl.gemm_quad, default) vs the K-half phased
schedule (tl.gemm_quad=False) vs hipBLASLt (torch), round-robin, cold-cache do_bench; numerics
against an fp32 torch matmul, including odd and single K-tile counts.

    python scripts/gemm_quad_ab.py [--shapes M,N,K ...] [--dtype float16|bfloat16|float8_e4m3fn] [--rounds 3]

fp8 (OCP e4m3 / e5m2): examples/gemm_fp8's 256x256x128 kernel (bf16 out) against hipBLASLt's
``torch._scaled_mm`` with unit scales.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "gemm"),
                os.path.join(HERE, "..", "examples", "gemm_fp8")]

import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_gemm import matmul  # noqa: E402
from example_tilelang_gemm_fp8 import matmul as matmul_fp8  # noqa: E402


def is_fp8(dtype):
    return dtype.startswith("float8")


def build(M, N, K, dtype, quad):
    if is_fp8(dtype):
        f = matmul_fp8.get_tir(M, N, K, dtype=dtype, staged_epilogue=True)
    else:
        f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, dtype, trans_B=True, staged_epilogue=True)
    return tilelang.compile(f, out_idx=[-1], target="hip", pass_configs={"tl.gemm_quad": quad})


def rand(shape, td):
    if td.is_floating_point and td.itemsize == 1:
        return torch.empty(shape, device="cuda").uniform_(-1, 1).to(td)
    return torch.empty(shape, device="cuda", dtype=td).uniform_(-1, 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shapes", nargs="*", default=["4096,4096,4096", "8192,8192,4096", "8192,8192,8192"])
    p.add_argument("--check", nargs="*", default=["256,256,64", "512,256,4160", "1024,512,192"])
    p.add_argument("--dtype", default="float16")
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    td = getattr(torch, a.dtype)
    for shp in a.check:
        M, N, K = map(int, shp.split(","))
        x, y = rand((M, K), td), rand((N, K), td)
        k = build(M, N, K, a.dtype, True)
        assert "gemm_quad_nt" in k.get_kernel_source(), "quad schedule not selected"
        out = k(x, y).float()
        ref = x.float() @ y.float().T
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        print(f"check {M}x{N}x{K} {a.dtype}: rel max err {err:.2e}", flush=True)
        assert err < 1e-2, err
    for shp in a.shapes:
        M, N, K = map(int, shp.split(","))
        x, y = rand((M, K), td), rand((N, K), td)
        ref = x.float() @ y.float().T
        ks = {}
        for name, quad in (("quad", True), ("khalf", False)):
            k = build(M, N, K, a.dtype, quad)
            assert ("gemm_quad_nt" in k.get_kernel_source()) == quad
            err = ((k(x, y).float() - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-2, (name, err)
            ks[name] = k
        res = {n: [] for n in list(ks) + ["hipblaslt"]}
        yt = y.T
        one = torch.ones((), device="cuda")
        if is_fp8(a.dtype):
            vendor = lambda: torch._scaled_mm(x, yt, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
        else:
            vendor = lambda: x @ yt  # noqa: E731
        for _ in range(a.rounds):
            for n, k in ks.items():
                res[n].append(do_bench(lambda: k(x, y), warmup=20, rep=100))
            res["hipblaslt"].append(do_bench(vendor, warmup=20, rep=100))
        fl = 2.0 * M * N * K
        print(f"{M}x{N}x{K} NT {a.dtype}: " + ", ".join(f"{n} {fl / min(v) * 1e-9:.0f}" for n, v in res.items()) +
              f" TF (cold, best of {a.rounds})", flush=True)


if __name__ == "__main__":
    main()
