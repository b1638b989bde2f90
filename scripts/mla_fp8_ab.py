"""MLA decode (b128 h128 kv8192, d 512 + 64; BASELINE config 4) in one process, round-robin after a
pre-warm: the bf16 kernel (example_mla_decode.py, num_split 4) against the fp8-cache kernel
(example_mla_decode_kv_fp8.py) with the score GEMM and / or P V on the CDNA4 fp8 MFMA.  TFLOPS are
the same useful FLOPs for every variant; numerics against the fp32 reference over the dequantised
cache (relative norm error).

    python scripts/mla_fp8_ab.py [--splits 1,2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "deepseek_mla")]

import torch  # noqa: E402

from example_mla_decode import mla_decode, ref_program as ref16, flops  # noqa: E402
from example_mla_decode_kv_fp8 import mla_decode_kv_fp8, quantize_kv, ref_program as ref8  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--heads", type=int, default=128)
    ap.add_argument("--kv", type=int, default=8192)
    ap.add_argument("--variants", default="qk8_pv16_64_1,qk8_pv8_64_1,qk8_pv8_64_2,qk8_pv8_128_1")
    ap.add_argument("--splits", default="1")
    ap.add_argument("--bf16-variants", default="", help="extra bf16 configs block_N_stages_split[_blockH[_summfma]], e.g. 64_2_2 or 64_2_1_64_1")
    a = ap.parse_args()
    B, H, S, D, P = a.batch, a.heads, a.kv, 512, 64
    torch.manual_seed(0)
    q = torch.randn(B, H, D, device="cuda", dtype=torch.bfloat16)
    qpe = torch.randn(B, H, P, device="cuda", dtype=torch.bfloat16)
    kvf = torch.randn(B, S, 1, D, device="cuda")
    kpe = torch.randn(B, S, 1, P, device="cuda", dtype=torch.bfloat16)
    kv8, s = quantize_kv(kvf)
    runs = []
    # bf16 baseline on the same (dequantised) cache values
    kv16 = (kv8.float() * s).to(torch.bfloat16)
    k16 = mla_decode(B, H, 1, S, D, P, num_split=4, dtype="bfloat16")
    g16, p16 = torch.empty(B, H, 4, device="cuda"), torch.empty(B, H, 4, D, device="cuda")
    o = k16(q, qpe, kv16, kpe, g16, p16)
    r = ref16(q, qpe, kv16, kpe).float()
    print(f"bf16: rel err {((o.float() - r).norm() / r.norm()).item():.2e}", flush=True)
    runs.append(("bf16 (split 4)", lambda: k16(q, qpe, kv16, kpe, g16, p16)))
    for v in filter(None, a.bf16_variants.split(",")):
        parts = [int(x) for x in v.split("_")]
        bn, st, ns = parts[:3]
        bh = parts[3] if len(parts) > 3 else 64
        sm = bool(parts[4]) if len(parts) > 4 else False  # sum_mfma
        try:
            kb = mla_decode(B, H, 1, S, D, P, block_N=bn, block_H=bh, num_split=ns, num_stages=st, dtype="bfloat16",
                            sum_mfma=sm)
            gb, pb = torch.empty(B, H, ns, device="cuda"), torch.empty(B, H, ns, D, device="cuda")
            o = kb(q, qpe, kv16, kpe, gb, pb)
            print(f"bf16 {v}: rel err {((o.float() - r).norm() / r.norm()).item():.2e}", flush=True)
            runs.append((f"bf16 {v}", lambda kb=kb, gb=gb, pb=pb: kb(q, qpe, kv16, kpe, gb, pb)))
        except Exception as e:  # noqa: BLE001
            print(f"bf16 {v}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
    ref = ref8(q, qpe, kv8, s, kpe)
    for ns in (int(x) for x in a.splits.split(",")):
        for v in a.variants.split(","):
            qk, pv, bn, st, *rest = v.split("_")  # optional 5th field "nosum": reduce_sum row sums
            try:
                k = mla_decode_kv_fp8(B, H, S, D, P, block_N=int(bn), num_split=ns, num_stages=int(st),
                                      qk_fp8=qk == "qk8", pv_fp8=pv == "pv8", sum_mfma=rest != ["nosum"])
                g, pp = torch.empty(B, H, ns, device="cuda"), torch.empty(B, H, ns, D, device="cuda")
                o = k(q, qpe, kv8, kpe, s, g, pp)
                err = ((o.float() - ref).norm() / ref.norm()).item()
                print(f"{v} split {ns}: rel err {err:.2e}", flush=True)
                runs.append((f"{v} split {ns}", lambda k=k, g=g, pp=pp: k(q, qpe, kv8, kpe, s, g, pp)))
            except Exception as e:  # noqa: BLE001
                print(f"{v} split {ns}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _, f in runs:
            f()
        torch.cuda.synchronize()
    res = {n: [] for n, _ in runs}
    for _ in range(5):
        for n, f in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) / 10)
    fl = flops(B, H, S, D, P)
    base = None
    for n, _ in runs:
        ms = sorted(res[n])[2]
        tf = fl / ms * 1e-9
        base = base or tf
        print(f"MLA decode b{B} h{H} kv{S} {n}: {ms:.4f} ms, {tf:.1f} TFLOPS ({tf / base:.2f}x bf16)", flush=True)


if __name__ == "__main__":
    main()
