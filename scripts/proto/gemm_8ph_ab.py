"""A/B of the 8-phase NT GEMM prototype (scripts/proto/gemm_8ph.hip) against the DSL kernel and
hipBLASLt, one process, interleaved rounds, cold-cache do_bench.  The prototype replaces the DSL
NT kernel's source through the register_hip_postproc hook (same signature, grid and block).

    python scripts/proto/gemm_8ph_ab.py [--variants "name:-DPRIO=0 ..." ...] [--shapes 4096,4096,4096 ...]
"""
import argparse
import os
import sys

os.environ["TILELANG_DISABLE_CACHE"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm"))

import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.engine import callback  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_gemm import matmul  # noqa: E402

DEFAULT = ["dsl:", "p8:-DPRIO=0", "pb:@gemm_8pb.hip"]


def parse(v):
    """name:[@source.hip] -DX=1 ..."""
    name, defs = v.split(":", 1)
    src = "gemm_8ph.hip"
    if defs.startswith("@"):
        src, _, defs = defs[1:].partition(" ")
    return name, src, defs


def build(M, N, K, defines, src_file="gemm_8ph.hip", nn=False):
    threads = 256 if src_file.startswith("gemm_4") else 512  # the 4-wave prototypes
    f = matmul.get_tir(M, N, K, 256, 256, 64, threads, 2, "float16", trans_B=not nn, staged_epilogue=True)
    if defines is None:
        callback.unregister()
        return tilelang.compile(f, out_idx=[-1], target="hip")
    src = open(os.path.join(HERE, src_file)).read()
    src = src.replace('#include "agpr_mfma.h"', open(os.path.join(HERE, "agpr_mfma.h")).read())
    head = "".join(f"#define {d[2:].replace('=', ' ', 1)}\n" for d in defines.split())
    head += f"#define GM {M}\n#define GN {N}\n#define GK {K}\n"
    callback.register_hip_postproc(lambda code, target: head + src)
    try:
        return tilelang.compile(f, out_idx=[-1], target="hip")
    finally:
        callback.unregister()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", nargs="*", default=DEFAULT)
    p.add_argument("--shapes", nargs="*", default=["4096,4096,4096", "8192,8192,4096", "8192,8192,8192"])
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--nn", action="store_true", help="B [K][N] (the bench layout) instead of [N][K]")
    a = p.parse_args()
    for shp in a.shapes:
        M, N, K = map(int, shp.split(","))
        x = torch.empty(M, K, device="cuda", dtype=torch.float16).uniform_(-1, 1)
        y = torch.empty(N, K, device="cuda", dtype=torch.float16).uniform_(-1, 1)
        if a.nn:
            y = y.T.contiguous()  # [K][N]
        yT = y.float() if a.nn else y.float().T
        ref = x.float() @ yT
        ks = {}
        for v in a.variants:
            name, src, defs = parse(v)
            if a.nn:
                defs += " -DNN=1"
            try:
                k = build(M, N, K, None if name == "dsl" else defs, src, a.nn)
                out = k(x, y)
                torch.cuda.synchronize()
                err = (out.float() - ref).abs().max().item()
                if err > 0.5:
                    print(f"{name}: WRONG (max err {err})", flush=True)
                    continue
                # a second run with different data: catches stale-LDS reads that the first hid
                x2 = torch.empty_like(x).uniform_(-1, 1)
                err2 = (k(x2, y).float() - x2.float() @ yT).abs().max().item()
                if err2 > 0.5:
                    print(f"{name}: WRONG on rerun (max err {err2})", flush=True)
                    continue
                print(f"{name}: ok (max err {err:.3g} / {err2:.3g})", flush=True)
                ks[name] = k
            except Exception as e:  # noqa: BLE001
                print(f"{name}: build/run failed: {str(e)[:600]}", flush=True)
        res = {n: [] for n in ks}
        res["hipblaslt"] = []
        yt = y if a.nn else y.T
        for _ in range(a.rounds):
            for n, k in ks.items():
                res[n].append(do_bench(lambda: k(x, y), warmup=20, rep=100))
            res["hipblaslt"].append(do_bench(lambda: x @ yt, warmup=20, rep=100))
        fl = 2.0 * M * N * K
        print(f"{M}x{N}x{K} {'NN' if a.nn else 'NT'}: " + ", ".join(f"{n} {fl / min(v) * 1e-9:.0f}" for n, v in res.items()) +
              f" TF (cold, best of {a.rounds})", flush=True)


if __name__ == "__main__":
    main()
