"""A/B of GEMM main-loop prototypes (scripts/proto/gemm_rp.hip) against the DSL kernel and
hipBLASLt, one process, interleaved rounds, cold-cache do_bench.  Each prototype replaces the
DSL kernel's source through the register_hip_postproc hook (same signature, grid and block).

    python scripts/proto/gemm_rp_ab.py [--variants "name:-DFOO=1 ..." ...] [--shapes 4096,4096,4096 ...]
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

DEFAULT = [
    "dsl:",
    "dsl_noilv:cfg tl.gemm_interleave=0",
    "dsl_noprefetch:cfg tl.gemm_prefetch=0",
    "rp2x4_ilv:-DWAVES_M=2 -DPREFETCH=1 -DILV=1",
]


def build(M, N, K, defines):
    f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, "float16", staged_epilogue=True)
    if not defines or defines.startswith("cfg "):
        # the DSL kernel; "cfg key=0 key2=1" sets boolean pass configs
        cfg = {kv.split("=")[0]: bool(int(kv.split("=")[1])) for kv in defines.split()[1:]} if defines else {}
        callback.unregister()
        return tilelang.compile(f, out_idx=[-1], target="hip", pass_configs=cfg)
    src = open(os.path.join(HERE, "gemm_rp.hip")).read()
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
    a = p.parse_args()
    for shp in a.shapes:
        M, N, K = map(int, shp.split(","))
        x = torch.empty(M, K, device="cuda", dtype=torch.float16).uniform_(-1, 1)
        y = torch.empty(K, N, device="cuda", dtype=torch.float16).uniform_(-1, 1)
        ref = x @ y
        ks = {}
        for v in a.variants:
            name, defs = v.split(":", 1)
            try:
                k = build(M, N, K, defs)
                out = k(x, y)
                err = (out.float() - ref.float()).abs().max().item()
                if err > 0.5:
                    print(f"{name}: WRONG (max err {err})", flush=True)
                    continue
                ks[name] = k
            except Exception as e:  # noqa: BLE001
                print(f"{name}: build/run failed: {str(e)[:400]}", flush=True)
        res = {n: [] for n in ks}
        res["hipblaslt"] = []
        for _ in range(a.rounds):
            for n, k in ks.items():
                res[n].append(do_bench(lambda: k(x, y), warmup=20, rep=100))
            res["hipblaslt"].append(do_bench(lambda: x @ y, warmup=20, rep=100))
        fl = 2.0 * M * N * K
        print(f"{M}x{N}x{K}: " + ", ".join(f"{n} {fl / min(v) * 1e-9:.0f}" for n, v in res.items()) + " TF (cold, best of "
              f"{a.rounds})", flush=True)


if __name__ == "__main__":
    main()
