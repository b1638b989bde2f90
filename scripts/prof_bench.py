"""Run the bench.py kernels (fp16 GEMM 4096^3, FA fwd bf16 b1 h64 s4096 d128) for profiling.

    python scripts/prof_bench.py {gemm|fa|both} [reps] [--cold]

Used under ``rocprofv3 --kernel-trace --stats`` or ``--pmc``.  ``--cold`` prints the do_bench
(512 MiB flush) and back-to-back (warm) times for each kernel instead.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm"), os.path.join(ROOT, "examples", "flash_attention")]
import torch  # noqa: E402

import bench  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
reps = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 20
cold = "--cold" in sys.argv

runs = {}
if which in ("gemm", "both"):
    gemm, (A, B) = bench.build_gemm()
    runs["gemm"] = (lambda: gemm(A, B), 2.0 * 4096**3)
if which in ("fa", "both"):
    attn, (Q, K, V) = bench.build_attn()
    c = bench.ATTN_CFG
    runs["fa"] = (lambda: attn(Q, K, V), 4.0 * c["batch"] * c["heads"] * c["seq_len"]**2 * c["dim"])

if cold:
    from tilelang.profiler import do_bench
    for name, (fn, flops) in runs.items():
        fn()
        t_cold = do_bench(fn, warmup=10, rep=50)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t_warm = e0.elapsed_time(e1) / 50
        print(f"{name}: cold {t_cold * 1e3:.1f} us = {flops / t_cold * 1e-9:.1f} TF | "
              f"warm {t_warm * 1e3:.1f} us = {flops / t_warm * 1e-9:.1f} TF", flush=True)
else:
    for _ in range(reps):
        for fn, _f in runs.values():
            fn()
    torch.cuda.synchronize()
    print("done", which)
