"""A/B of device-compiler flags on the bench's FA and GEMM kernels (same process, same box).

The guide (MI355X_MICROARCH 'Per-instruction cycle constants') prices SLP-packed v_pk_*_f32 beside
MFMAs as an anti-lever; -fno-slp-vectorize keeps them scalar.  Prints cold (512 MiB flush) and warm
TFLOPS per variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm"), os.path.join(ROOT, "examples", "flash_attention")]

import torch  # noqa: E402

import bench  # noqa: E402
import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

VARIANTS = {
    "default": [],
    "no-slp": ["-fno-slp-vectorize"],
    "default2": [],
    "no-slp2": ["-fno-slp-vectorize"],
}


def warm(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    from example_mha_fwd_pipelined import flashattn_pipelined as fa
    from example_gemm import matmul
    a = bench.ATTN_CFG
    g = bench.GEMM_CFG
    fa_f = fa.get_tir(a["batch"], a["heads"], a["seq_len"], a["dim"], False, 1, a["block_M"], a["block_N"],
                      a["threads"], a["num_stages"], "bfloat16", True, True)
    gm_f = matmul.get_tir(g["M"], g["N"], g["K"], g["block_M"], g["block_N"], g["block_K"], g["threads"],
                          g["num_stages"])
    shp = (a["batch"], a["seq_len"], a["heads"], a["dim"])
    q, k, v = (torch.randn(shp, device="cuda").bfloat16() for _ in range(3))
    A = torch.randn(g["M"], g["K"], device="cuda").half()
    B = torch.randn(g["K"], g["N"], device="cuda").half()
    fa_flops = 4.0 * a["batch"] * a["heads"] * a["seq_len"]**2 * a["dim"]
    gm_flops = 2.0 * g["M"] * g["N"] * g["K"]
    fa_y = fa.get_tir(a["batch"], a["heads"], a["seq_len"], a["dim"], False, 1, a["block_M"], a["block_N"],
                      a["threads"], a["num_stages"], "bfloat16", True, True, True)
    for name, flags in (("young-prio", []), ("young-prio+no-slp", ["-fno-slp-vectorize"])):
        ky = tilelang.compile(fa_y, out_idx=[3], target="hip", pass_configs=fa.pass_configs, compile_flags=flags)
        c = do_bench(lambda: ky(q, k, v))
        w = warm(lambda: ky(q, k, v))
        print(f"fa    {name:10s} cold {fa_flops / c * 1e-9:7.1f} TF  warm {fa_flops / w * 1e-9:7.1f} TF", flush=True)
    for name, flags in VARIANTS.items():
        kf = tilelang.compile(fa_f, out_idx=[3], target="hip", pass_configs=fa.pass_configs, compile_flags=flags)
        kg = tilelang.compile(gm_f, out_idx=[-1], target="hip", compile_flags=flags)
        torch.testing.assert_close(kg(A, B).float(), (A.float() @ B.float()), rtol=2e-2, atol=1.0)
        for label, kern, args, fl in (("fa", kf, (q, k, v), fa_flops), ("gemm", kg, (A, B), gm_flops)):
            c = do_bench(lambda: kern(*args))
            w = warm(lambda: kern(*args))
            print(f"{label:5s} {name:10s} cold {fl / c * 1e-9:7.1f} TF  warm {fl / w * 1e-9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
