"""Causal forward kernels: query-tile axis slowest in the grid (longest walks of every (batch, head)
first) vs the previous grid (tile axis in the middle: longest-first within one batch only).
Same process, round-robin; the previous kernels are loaded from copies of their sources passed
on the command line (``git show HEAD~1:<path> > <copy>``).

    python scripts/fa_fwd_lpt_ab.py OLD_PIPELINED.py OLD_SINK.py
"""
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "attention_sink"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_mha_fwd_pipelined as P  # noqa: E402
import example_gqa_sink_fwd_bhsd as SK  # noqa: E402


def load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def build(mod, B, H, S):
    import tilelang
    f = mod.flashattn_pipelined.get_tir(B, H, S, 128, True, 1, 256, 64, 512, 2, "bfloat16", True, True,
                                        sum_mfma=True, fold_max=True, young_prio=True, unroll=2)
    pc = dict(mod.flashattn_pipelined.pass_configs)
    pc["tl.gemm_rs_pipe"] = 4
    return tilelang.compile(f, out_idx=[3], pass_configs=pc)


def ab(label, kerns, args, ref, flops):
    res = {}
    for name, k in kerns.items():
        err = (k(*args).float() - ref).abs().max().item()
        res[name] = [1e9, err]
    for _ in range(3):
        for name, k in kerns.items():
            res[name][0] = min(res[name][0], do_bench(lambda: k(*args), warmup=10, rep=50))
    print(label + ": " + "  ".join(f"{n} {m * 1e3:.1f} us {flops / m * 1e-9:.0f} TF err {e:.4f}"
                                   for n, (m, e) in res.items()), flush=True)


def main():
    oldP, oldS = load(sys.argv[1], "old_pipelined"), load(sys.argv[2], "old_sink")
    torch.manual_seed(0)
    for B, H, S in ((1, 64, 4096), (4, 32, 4096), (8, 32, 2048), (16, 16, 1024)):
        q, k, v = (torch.randn(B, S, H, 128, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        ref = P.ref_program(q, k, v, True, 1).float()
        fl = 2.0 * B * H * S * S * 128
        ab(f"pipelined causal b{B} h{H} s{S} d128",
           {"old": build(oldP, B, H, S), "new": build(P, B, H, S)}, (q, k, v), ref, fl)
    for B, H, S in ((1, 64, 4096), (4, 32, 4096)):
        q = torch.randn(B, H, S, 128, device="cuda", dtype=torch.bfloat16)
        k, v = (torch.randn(B, H // 8, S, 128, device="cuda", dtype=torch.bfloat16) for _ in range(2))
        sinks = torch.randn(H, device="cuda", dtype=torch.bfloat16)
        ref = SK.ref_program(q, k, v, sinks, None).float()
        ab(f"sink causal b{B} h{H} s{S} d128 g8",
           {"old": oldS.flashattn_sink(B, H, S, S, 128, 8, None), "new": SK.flashattn_sink(B, H, S, S, 128, 8, None)},
           (q, k, v, sinks), ref, SK.flops(B, H, S, S, 128))


if __name__ == "__main__":
    main()
