"""FA forward config sweep (bench shape b1 h64 s4096 d128 bf16): warm back-to-back and cold
(do_bench, 512 MiB flush) TFLOPS per config, one process (guide rule 24), correctness checked.

    python scripts/sweep_fa.py [--quick]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "flash_attention")]
import torch  # noqa: E402

import tilelang  # noqa: E402
from example_mha_fwd import flashattn, ref_program  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

B, H, S, D = 1, 64, 4096, 128
flops = 4.0 * B * H * S * S * D
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
ref = None
CFGS = [
    # kind, block_M, block_N, threads, stages, q_in_regs, fast_math
    ("plain", 256, 64, 512, 3, True, True),
    ("staged", 256, 64, 512, 3, True, True),
    ("staged", 256, 64, 512, 2, True, True),
    ("plain", 128, 64, 256, 3, True, True),
    ("staged", 128, 64, 256, 3, True, True),
    ("staged", 256, 128, 512, 2, True, True),
]
if "--quick" in sys.argv:
    CFGS = CFGS[:4]
for kind, bm, bn, th, st, qr, fm in CFGS:
    tag = f"{kind} bm{bm} bn{bn} t{th} st{st} qregs{int(qr)} fast{int(fm)}"
    try:
        fac = flashattn if kind == "plain" else flashattn_pipelined
        f = fac.get_tir(B, H, S, D, False, 1, bm, bn, th, st, "bfloat16", True, qr)
        kern = tilelang.compile(f, out_idx=[3], target="hip",
                                pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: fm})
        o = kern(q, k, v)
        if ref is None:
            ref = ref_program(q[:, :512], k, v).float()
        err = (o[:, :512].float() - ref).abs().max().item()
        fn = lambda: kern(q, k, v)  # noqa: E731
        fn()
        cold = do_bench(fn, warmup=5, rep=30)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            fn()
        e1.record()
        torch.cuda.synchronize()
        warm = e0.elapsed_time(e1) / 30
        print(f"{tag}: err {err:.3g} | cold {flops / cold * 1e-9:.1f} TF | warm {flops / warm * 1e-9:.1f} TF", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{tag}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
