"""Run one bench kernel (the headline GEMM or FA) N times for a rocprofv3 --pmc pass.

    rocprofv3 --pmc <counters> -- python3 scripts/pmc_driver.py gemm|gemm_nt|hipblaslt_nt|fp8_nt|scaled_mm|fa|fa32 [iters]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "gemm"))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    which = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.manual_seed(0)
    if which == "gemm":  # B [K, N] ("NN")
        from example_gemm import matmul
        g = dict(bench.GEMM_CFG, trans_B=False)
        k = matmul(**g)
        a = torch.randn(g["M"], g["K"], device="cuda").half()
        b = torch.randn(g["K"], g["N"], device="cuda").half()
        fn = lambda: k(a, b)  # noqa: E731
    elif which == "gemm_nt":  # B given as [N, K] (K-contiguous, "NT"), the bench's tile config
        from example_gemm import matmul
        g = dict(bench.GEMM_CFG, trans_B=True)
        k = matmul(**g)
        a = torch.randn(g["M"], g["K"], device="cuda").half()
        b = torch.randn(g["N"], g["K"], device="cuda").half()
        fn = lambda: k(a, b)  # noqa: E731
    elif which == "hipblaslt_nt":  # the vendor library on the same NT problem
        g = bench.GEMM_CFG
        a = torch.randn(g["M"], g["K"], device="cuda").half()
        b = torch.randn(g["N"], g["K"], device="cuda").half()
        fn = lambda: a @ b.T  # noqa: E731
    elif which in ("fp8_nt", "scaled_mm"):  # fp8 e4m3 8192^3, B [N, K]: the quad loop / hipBLASLt
        sys.path.insert(0, os.path.join(HERE, "..", "examples", "gemm_fp8"))
        n = 8192
        a = torch.randn(n, n, device="cuda").to(torch.float8_e4m3fn)
        b = torch.randn(n, n, device="cuda").to(torch.float8_e4m3fn)
        if which == "fp8_nt":
            from example_tilelang_gemm_fp8 import matmul as mm8
            k = mm8(n, n, n, staged_epilogue=True)
            fn = lambda: k(a, b)  # noqa: E731
        else:
            one = torch.ones((), device="cuda")
            fn = lambda: torch._scaled_mm(a, b.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
    elif which == "fa":  # the bench's attention kernel, exactly as bench.py builds it
        k, (q, kk, v) = bench.build_attn("cuda")
        fn = lambda: k(q, kk, v)  # noqa: E731
    else:
        from example_mha_fwd_pipelined import flashattn_pipelined
        c = dict(bench.ATTN_CFG)
        k = flashattn_pipelined(c["batch"], c["heads"], c["seq_len"], c["dim"], False, 1, c["block_M"], c["block_N"],
                                c["threads"], c["num_stages"], mfma="32x32")
        q, kk, v = (torch.randn(c["batch"], c["seq_len"], c["heads"], c["dim"], device="cuda",
                                dtype=torch.bfloat16) for _ in range(3))
        fn = lambda: k(q, kk, v)  # noqa: E731
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print("done", which)


if __name__ == "__main__":
    main()
