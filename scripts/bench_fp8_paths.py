"""fp8 paths on one MI355X: MLA decode over an fp8 latent cache (vs the bf16-cache kernel at the
same shape), the block-scaled fp8 linear (vs bf16 hipBLASLt), the grouped per-token fp8 cast.

    python scripts/bench_fp8_paths.py [--quick]
"""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
for d in ("deepseek_mla", "cast"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402


def mla(quick):
    from example_mla_decode import mla_decode
    from example_mla_decode_kv_fp8 import flops, mla_decode_kv_fp8, quantize_kv, ref_program
    B, H, S = (64, 128, 4096) if quick else (128, 128, 8192)
    q = torch.randn(B, H, 512, device="cuda", dtype=torch.bfloat16)
    qpe = torch.randn(B, H, 64, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(B, S, 1, 512, device="cuda")
    kv8, s = quantize_kv(kv)
    kpe = torch.randn(B, S, 1, 64, device="cuda", dtype=torch.bfloat16)
    fl = flops(B, H, S, 512, 64)
    for ns in (1, 2):
        glse = torch.empty(B, H, ns, device="cuda")
        part = torch.empty(B, H, ns, 512, device="cuda")
        kb = mla_decode(B, H, 1, S, 512, 64, num_split=ns, dtype="bfloat16")
        kvb = kv.to(torch.bfloat16)
        ms = do_bench(lambda: kb(q, qpe, kvb, kpe, glse, part), warmup=10, rep=50)
        print(f"MLA bf16-cache b{B} h{H} s{S} split{ns}: {ms:.3f} ms {fl / ms * 1e-9:.1f} TFLOPS", flush=True)
        for qk_fp8, bn, st in ((True, 64, 1), (True, 32, 2), (False, 64, 1), (False, 32, 2)):
            try:
                k = mla_decode_kv_fp8(B, H, S, 512, 64, block_N=bn, num_split=ns, num_stages=st, qk_fp8=qk_fp8)
                o = k(q, qpe, kv8, kpe, s, glse, part)
                if ns == 1 and bn == 64:
                    r = ref_program(q[:8], qpe[:8], kv8[:8], s, kpe[:8], qk_fp8)
                    torch.testing.assert_close(o[:8].float(), r, rtol=2e-2, atol=2e-2)
                ms = do_bench(lambda: k(q, qpe, kv8, kpe, s, glse, part), warmup=10, rep=50)
                print(f"MLA fp8-cache qk_fp8={qk_fp8} bn{bn} st{st} split{ns}: {ms:.3f} ms "
                      f"{fl / ms * 1e-9:.1f} TFLOPS", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"MLA fp8-cache qk_fp8={qk_fp8} bn{bn} st{st} split{ns}: failed {type(e).__name__}: "
                      f"{str(e)[:200]}", flush=True)


def linear():
    from tilelang.ops import fp8_gemm as F
    for M, N, K in ((1, 7168, 2048), (64, 24576, 1536), (4096, 7168, 2048), (4096, 4096, 7168)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda") * 0.05
        wq, ws = F.weight_quant(w)
        wb = w.to(torch.bfloat16)
        from tilelang.ops.quant import act_quant
        xq, xs = act_quant(x, 128)
        ms_g = do_bench(lambda: F.fp8_gemm(xq, xs, wq, ws), warmup=10, rep=50)
        ms_l = do_bench(lambda: F.fp8_linear(x, wq, ws), warmup=10, rep=50)
        ms_b = do_bench(lambda: x @ wb.t(), warmup=10, rep=50)
        fl = 2 * M * N * K
        print(f"fp8 linear M{M} N{N} K{K}: gemm {ms_g:.4f} ms {fl / ms_g * 1e-9:.1f} TF, +act_quant {ms_l:.4f} ms; "
              f"bf16 torch {ms_b:.4f} ms {fl / ms_b * 1e-9:.1f} TF", flush=True)


def cast():
    from example_group_per_split_token_cast_to_fp8 import group_per_split_token_cast_to_fp8
    BG, N = 8, 7168
    sizes = [2048 - 97 * i for i in range(BG)]
    M, M_max = sum(sizes), max(sizes)
    x = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    bs = torch.tensor(sizes, dtype=torch.int32, device="cuda")
    for blk_m, t in ((8, 128), (16, 256), (32, 256)):
        k = group_per_split_token_cast_to_fp8(M, M_max, N, BG, blk_m, 128, t)
        ms = do_bench(lambda: k(x, bs), warmup=10, rep=50)
        nb = M * N * 2 + BG * M_max * N * (1 + 4 / 128)
        print(f"group cast BG{BG} M{M} N{N} blk_m{blk_m} t{t}: {ms:.4f} ms {nb / ms * 1e-9:.2f} TB/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    mla(a.quick)
    linear()
    cast()


if __name__ == "__main__":
    main()
