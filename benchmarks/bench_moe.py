#!/usr/bin/env python3
"""MoE FFN layer throughput on the mesh (BASELINE config 5: 8 experts, 1/2/4/8 MI355X).

    python benchmarks/bench_moe.py --parallel local|ep|tp --tokens 8192 [--steps 20]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_moe.py --parallel ep

Weak scaling for ``ep`` (every rank brings --tokens tokens); ``tp`` replicates the tokens and
splits every expert's FFN width.  Prints one JSON line (rank 0) with the aggregate TFLOPS
(6 * tokens * topk * hidden * ffn per rank-batch, counting the useful expert FLOPs only).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parallel", default="ep", choices=["local", "ep", "tp"])
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=14336)
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()

    import torch
    from tilelang.models.moe import MoEConfig, MoELayer
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    mesh = None
    if world > 1 or args.parallel != "local":
        from tilelang.parallel import init_mesh
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        mesh = init_mesh(1, world)
    cfg = MoEConfig(hidden=args.hidden, ffn=args.ffn, n_experts=args.experts, topk=args.topk)
    layer = MoELayer(cfg, args.parallel, mesh=mesh, device="cuda")
    torch.manual_seed(rank if args.parallel != "tp" else 0)
    x = torch.randn(args.tokens, args.hidden, device="cuda", dtype=cfg.dtype)
    for _ in range(args.warmup):
        layer(x)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        layer(x)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / args.steps
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    flops_rank = 6.0 * args.tokens * args.topk * args.hidden * args.ffn
    total = flops_rank * (world if args.parallel != "tp" else 1)
    if rank == 0:
        print(json.dumps({"metric": "moe_ffn_tflops", "value": round(total / dt / 1e12, 2), "unit": "TFLOPS",
                          "n_gpus": world, "ms_per_step": round(dt * 1e3, 4), "parallel": args.parallel,
                          "config": {"hidden": args.hidden, "ffn": args.ffn, "experts": args.experts,
                                     "topk": args.topk, "tokens_per_rank": args.tokens, "dtype": "bf16"}}))


if __name__ == "__main__":
    main()
