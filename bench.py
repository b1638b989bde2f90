#!/usr/bin/env python3
"""Headline benchmark: achieved TFLOPS of the tilelang fp16 GEMM 4096^3 + MHA fwd seqlen 4096.

BASELINE.json metric: "achieved TFLOPS: fp16 GEMM 4096^3 and MHA seqlen=4096; % of MFMA roofline".
One *step* = one fp16 GEMM (M=N=K=4096) + one FlashAttention-2 forward (bf16, batch 1, 64 heads,
seqlen 4096, head_dim 128), both compiled by tilelang from the DSL programs in examples/.
Weak scaling: every rank (one process per GPU, RCCL/torch.distributed for the barriers and the
max-over-ranks timing) runs one step's work; ``value`` is the whole-job aggregate TFLOPS.

    python bench.py --gpus N --steps K --warmup W
    (N>1 is launched by torch.distributed.run; rank/world come from the environment)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm"))
sys.path.insert(0, os.path.join(ROOT, "examples", "flash_attention"))

# reference numbers: fp16 GEMM 736 TFLOPS (H800, 8192x8192x4096);
# attention fwd bf16 hd128 seq4096 497.13 TFLOPS (H800, GQA+sink b1 h64 kvh8)
REF_GEMM_TF = 736.0
REF_ATTN_TF = 497.13
PEAK_BF16_TF = 2500.0  # MI355X dense fp16/bf16 MFMA (AMD spec, no sparsity)

GEMM_CFG = dict(M=4096, N=4096, K=4096, block_M=256, block_N=256, block_K=64, threads=512, num_stages=2)
ATTN_CFG = dict(batch=1, heads=64, seq_len=4096, dim=128, block_M=256, block_N=64, threads=512, num_stages=2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))

    from example_gemm import matmul
    from example_mha_fwd import flashattn

    g = GEMM_CFG
    gemm = matmul(g["M"], g["N"], g["K"], g["block_M"], g["block_N"], g["block_K"], g["threads"], g["num_stages"],
                  "float16")
    a_ = ATTN_CFG
    attn = flashattn(a_["batch"], a_["heads"], a_["seq_len"], a_["dim"], False, 1, a_["block_M"], a_["block_N"],
                     a_["threads"], a_["num_stages"], "bfloat16")

    torch.manual_seed(1234 + rank)
    A = torch.randn(g["M"], g["K"], device="cuda", dtype=torch.float16)
    B = torch.randn(g["K"], g["N"], device="cuda", dtype=torch.float16)
    C = torch.empty(g["M"], g["N"], device="cuda", dtype=torch.float16)
    shp = (a_["batch"], a_["seq_len"], a_["heads"], a_["dim"])
    Q = torch.randn(shp, device="cuda", dtype=torch.bfloat16)
    Kt = torch.randn(shp, device="cuda", dtype=torch.bfloat16)
    V = torch.randn(shp, device="cuda", dtype=torch.bfloat16)

    # correctness guard (cheap spot check so a broken kernel cannot post a number)
    C = gemm(A, B)
    ref = (A[:256].float() @ B.float())
    if not torch.allclose(C[:256].float(), ref, rtol=2e-2, atol=2e-1):
        raise SystemExit("GEMM result check failed")

    gemm_flops = 2.0 * g["M"] * g["N"] * g["K"]
    attn_flops = 4.0 * a_["batch"] * a_["heads"] * a_["seq_len"] ** 2 * a_["dim"]

    def step():
        gemm(A, B)
        attn(Q, Kt, V)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # per-kernel times (events) for the report, measured after the timed region
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    for _ in range(10):
        gemm(A, B)
    ev[1].record()
    for _ in range(10):
        attn(Q, Kt, V)
    ev[2].record()
    torch.cuda.synchronize()
    gemm_ms = ev[0].elapsed_time(ev[1]) / 10
    attn_ms = ev[1].elapsed_time(ev[2]) / 10

    t = torch.tensor([elapsed, gemm_ms, attn_ms], device="cuda", dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, gemm_ms, attn_ms = t.tolist()
    ms_per_step = elapsed / args.steps * 1e3
    total_flops = (gemm_flops + attn_flops) * world * args.steps
    tflops = total_flops / elapsed / 1e12
    # the reference's time for the same per-GPU work at its published rates
    ref_step_s = gemm_flops / (REF_GEMM_TF * 1e12) + attn_flops / (REF_ATTN_TF * 1e12)
    ref_tflops = (gemm_flops + attn_flops) / ref_step_s / 1e12 * world
    if rank == 0:
        out = {
            "metric": "achieved TFLOPS: fp16 GEMM 4096^3 and MHA seqlen=4096; % of MFMA roofline",
            "value": round(tflops, 2),
            "unit": "TFLOPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(tflops / ref_tflops, 4),
            "dtype": "bf16",
            "data": "synthetic (torch.randn)",
            "config": {
                "model": "fp16 GEMM 4096x4096x4096 + FlashAttention-2 fwd bf16 b1 h64 s4096 d128",
                "global_batch": world,
                "seq_len": a_["seq_len"],
                "parallelism": f"dp{world}",
            },
            "gemm_tflops": round(gemm_flops / gemm_ms / 1e9, 1),
            "attn_tflops": round(attn_flops / attn_ms / 1e9, 1),
            "pct_of_mfma_peak": round(100.0 * tflops / world / PEAK_BF16_TF, 1),
            "gemm_dtype": "float16",
            "attn_dtype": "bfloat16",
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
