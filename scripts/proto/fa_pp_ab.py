"""A/B of the FlashAttention forward ping-pong prototype (scripts/proto/fa_pp.hip) against the
DSL kernel of the bench (b1 h64 s4096 d128 bf16, non-causal), one process, interleaved rounds.
Each prototype replaces the DSL kernel's source through the register_hip_postproc hook.

    python scripts/proto/fa_pp_ab.py [--variants "name:-DPP=1 ..." ...] [--seq 4096]
"""
import argparse
import os
import sys

os.environ["TILELANG_DISABLE_CACHE"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "flash_attention"))

import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.engine import callback  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined as fa  # noqa: E402

DEFAULT = ["dsl:", "lockstep3:-DPP=0", "pp:-DPP=1", "pp_prio:-DPP=1 -DPRIO=1"]


def build(seq, defines):
    f = fa.get_tir(1, 64, seq, 128, False, 1, 256, 64, 512, 2, "bfloat16", True, True)
    if defines:
        src = open(os.path.join(HERE, "fa_pp.hip")).read()
        head = "".join(f"#define {d[2:].replace('=', ' ', 1)}\n" for d in defines.split())
        head += f"#define SEQ {seq}\n"
        callback.register_hip_postproc(lambda code, target: head + src)
    try:
        return tilelang.compile(f, out_idx=[3], target="hip", pass_configs=fa.pass_configs)
    finally:
        callback.unregister()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", nargs="*", default=DEFAULT)
    p.add_argument("--seq", type=int, default=4096)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    torch.manual_seed(0)
    shp = (1, a.seq, 64, 128)
    q, k, v = (torch.randn(shp, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    ref = torch.nn.functional.scaled_dot_product_attention(*(t.transpose(1, 2).float() for t in (q, k, v)))
    ref = ref.transpose(1, 2)
    ks = {}
    for var in a.variants:
        name, defs = var.split(":", 1)
        try:
            kern = build(a.seq, defs)
            out = kern(q, k, v)
            err = (out.float() - ref).abs().max().item()
            print(f"{name}: max err {err:.4f}", flush=True)
            if err > 0.05:
                print(f"{name}: WRONG", flush=True)
                continue
            ks[name] = kern
        except Exception as e:  # noqa: BLE001
            print(f"{name}: build/run failed: {str(e)[:600]}", flush=True)
    res = {n: [] for n in ks}
    for _ in range(a.rounds):
        for n, kern in ks.items():
            res[n].append(do_bench(lambda: kern(q, k, v), warmup=10, rep=50))
    fl = 4.0 * 64 * a.seq * a.seq * 128
    print(f"FA fwd b1 h64 s{a.seq} d128: " + ", ".join(f"{n} {fl / min(t) * 1e-9:.0f}" for n, t in res.items()) +
          f" TF (best of {a.rounds})", flush=True)


if __name__ == "__main__":
    main()
