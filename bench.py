#!/usr/bin/env python3
"""Headline benchmark: achieved TFLOPS of fp16 GEMM 4096^3 + MHA seqlen 4096 + the config-5 MoE.

BASELINE.json metric: "achieved TFLOPS: fp16 GEMM 4096^3 and MHA seqlen=4096; % of MFMA roofline".
One *step* on every rank (one process per GPU) =
  1. fp16 GEMM M=N=K=4096                                   (BASELINE config 2)
  2. FlashAttention-2 forward bf16, b1 h64 s4096 d128        (BASELINE config 3)
  3. MoE FFN layer, 8 SwiGLU experts, top-2, hidden 4096, expert ffn 2048, 2048 tokens/rank,
     experts sharded over the ranks (expert parallel): the routed tokens travel to their
     experts' GPU and back with two RCCL all-to-alls over xGMI (BASELINE config 5)
all three compiled by tilelang from the DSL programs in examples/ and tilelang/ops.
Weak scaling: per-rank work is fixed as N grows; ``value`` is the whole-job aggregate TFLOPS
(useful FLOPs of all N ranks / the max-over-ranks wall time of the timed steps).

    python bench.py --gpus N --steps K --warmup W
    (--gpus N>1 without a torchrun environment re-launches itself under torch.distributed.run
     as a CHILD process before touching the GPU; under torchrun WORLD_SIZE must equal N)

``vs_baseline``: the reference's time for the same per-rank work at its published rates
(736 TF fp16 GEMM; 497.13 TF attention; the MoE grouped GEMMs are priced at the
GEMM rate, the reference publishes no MoE number) divided by our time.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm"))
sys.path.insert(0, os.path.join(ROOT, "examples", "flash_attention"))

METRIC = "achieved TFLOPS: fp16 GEMM 4096^3 and MHA seqlen=4096; % of MFMA roofline"
# reference numbers: fp16 GEMM 736 TFLOPS (H800, 8192x8192x4096);
# attention fwd bf16 hd128 seq4096 497.13 TFLOPS (H800, GQA+sink b1 h64 kvh8)
REF_GEMM_TF = 736.0
REF_ATTN_TF = 497.13
PEAK_BF16_TF = 2500.0  # MI355X dense fp16/bf16 MFMA (AMD spec, no sparsity)

# staged_epilogue: C tile through LDS, row-contiguous 16-byte stores (+3-4 % cold, profiles/r2/session2/gemm_epi_ab.log)
# trans_B: B stored [N, K], the layout of the reference's benchmark/matmul/benchmark_matmul.py:163,209
# (the fp16 GEMM headline); its main loop is tl::gemm_quad_nt_x (tl/gemm_quad.h), 1179 -> 1311 TF
# over the K-half schedule at 4096^3 (profiles/r5/gemm_quad_ab1.log).  The vendor normaliser below
# runs the same layout (torch.matmul(A, B.T), hipBLASLt's NT kernel)
GEMM_CFG = dict(M=4096, N=4096, K=4096, block_M=256, block_N=256, block_K=64, threads=512, num_stages=2,
                staged_epilogue=True, trans_B=True)
# FA (scripts/sweep_fa.py, profiles/r2/fa_staged.log): 256x64 tile, 8 waves, Q in registers, 2-stage K/V
# ring, T.Pipelined(order, stage) schedule: QK^T(t) | rescale+PV(t-1) | softmax(t)
# sum_mfma: softmax row sums on the matrix cores (P x ones), +1.7-2 % (profiles/r3/s3/fa_sum_mfma_ab.log)
# fold_max: running max as the QK^T accumulator's initial value, exp(t) between the PV(t-1) MFMAs
# (+5-8 %), young_prio: waves 4-7 at issue priority 1 (+1-2 %, profiles/r4/fa_fold_ab.log; re-measured
# r5 round-robin in one process: 937.5 vs 928.4 TF sustained, profiles/r5/fa_ab_roundrobin.log)
# xcd_heads: all query tiles of a head on one XCD, K/V read through one L2 (+2-5 %, profiles/r4/fa_xcd.log)
# unroll=2: the main loop as two copies, so both LDS ring slots are compile-time offsets (no per-tile
# address VALU): 1089 -> 1094 TF, same process, round-robin (profiles/r6/fa_unroll_ab.log)
ATTN_CFG = dict(batch=1, heads=64, seq_len=4096, dim=128, block_M=256, block_N=64, threads=512, num_stages=2,
                q_in_regs=True, sum_mfma=True, fold_max=True, young_prio=True, xcd_heads=True, unroll=2,
                # P V's B fragments streamed through the MFMAs in groups of 4 (tl::gemm_rs PIPE): +1.3 %
                # non-causal and causal, same process (profiles/r6/fa_rs_pipe_ab.log)
                pass_configs={"tl.gemm_rs_pipe": 4})
MOE_CFG = dict(tokens=2048, hidden=4096, ffn=2048, experts=8, topk=2)
# expert row tiles of 256 + MOE_EXT_M rows, every expert's rows spread evenly over its tiles
# (ops/moe.py expert_gemm_sk_kernel ext_M): a random-routing expert of ~529 rows is two units, not three
MOE_EXT_M = 32
# --device cpu (CI plumbing run on the CPU target under gloo): same program, tiny shapes
TINY = dict(gemm=dict(M=128, N=128, K=128, block_M=64, block_N=64, block_K=32, threads=128, num_stages=2),
            attn=dict(batch=1, heads=2, seq_len=128, dim=64, block_M=64, block_N=32, threads=128, num_stages=2,
                      q_in_regs=True),
            moe=dict(tokens=32, hidden=64, ffn=64, experts=8, topk=2))


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(args) -> int:
    """Run this script under torch.distributed.run with one rank per GPU (child process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _target(device):
    return "cpu" if device == "cpu" else "hip"


def build_gemm(device="cuda", g=None):
    import torch
    import tilelang
    from example_gemm import matmul
    g = g or GEMM_CFG
    tb = g.get("trans_B", False)
    f = matmul.get_tir(g["M"], g["N"], g["K"], g["block_M"], g["block_N"], g["block_K"], g["threads"],
                       g["num_stages"], "float16", trans_B=tb, staged_epilogue=g.get("staged_epilogue", False))
    k = tilelang.compile(f, out_idx=[-1], target=_target(device))
    A = torch.randn(g["M"], g["K"], device=device).to(torch.float16)
    B = torch.randn(g["N"], g["K"], device=device).to(torch.float16) if tb else \
        torch.randn(g["K"], g["N"], device=device).to(torch.float16)
    return k, (A, B)


def build_attn(device="cuda", a=None):
    import torch
    import tilelang
    from example_mha_fwd_pipelined import flashattn_pipelined as flashattn
    a = a or ATTN_CFG
    f = flashattn.get_tir(a["batch"], a["heads"], a["seq_len"], a["dim"], False, 1, a["block_M"], a["block_N"],
                          a["threads"], a["num_stages"], "bfloat16", True, a.get("q_in_regs", False),
                          sum_mfma=a.get("sum_mfma", False), fold_max=a.get("fold_max", False),
                          young_prio=a.get("young_prio", False), pk_scale=a.get("pk_scale", False),
                          pingpong=a.get("pingpong", False), xcd_heads=a.get("xcd_heads", False),
                          unroll=a.get("unroll"))
    pc = dict(flashattn.pass_configs)
    pc.update(a.get("pass_configs", {}))
    k = tilelang.compile(f, out_idx=[3], target=_target(device), pass_configs=pc)
    shp = (a["batch"], a["seq_len"], a["heads"], a["dim"])
    return k, tuple(torch.randn(shp, device=device).to(torch.bfloat16) for _ in range(3))


def build_moe(mesh, device="cuda", m=None, mode=None):
    import torch
    from tilelang.models.moe import MoEConfig, MoELayer
    m = m or MOE_CFG
    dt = torch.bfloat16 if device != "cpu" else torch.float32
    bm = 256 if device != "cpu" else 16
    # expert GEMM tile: 256x256x64, 8 waves, 2-stage LDS-DMA (scripts/prof_moe.py --sweep, profiles/r2)
    gc = dict(block_N=256, block_K=64, num_stages=2, threads=512, ext_M=MOE_EXT_M) if device != "cpu" else None
    cfg = MoEConfig(hidden=m["hidden"], ffn=m["ffn"], n_experts=m["experts"], topk=m["topk"], dtype=dt, block_M=bm,
                    gemm_cfg=gc)
    layer = MoELayer(cfg, mode or ("ep" if mesh is not None else "local"), mesh=mesh, device=device)
    x = torch.randn(m["tokens"], m["hidden"], device=device).to(dt)
    return layer, x


def tp_phase(mesh, dev, m, X, dist, timed, reps, cpu):
    """Config-5 Mesh cross-GPU tiles: the same MoE layer tensor-parallel (every expert's FFN
    split over the ranks, partial outputs summed by the in-kernel two-shot T.comm all-reduce of
    the down-projection GEMM).  Checked against the fp32 definition, timed outside the headline
    step and reported next to it; any failure is reported, never fatal to the headline."""
    import torch
    try:
        layer, _ = build_moe(mesh, dev, m, mode="tp")
        torch.manual_seed(4321)  # replicated tokens: the same on every rank
        xt = torch.randn_like(X.float()).to(X.dtype)
        yt = layer(xt)
        from tilelang.models.moe import moe_reference, init_moe_weights
        from tilelang.ops.moe import route
        g_w, w1, w2 = (t.to(xt.device) for t in init_moe_weights(layer.cfg))
        rows = slice(0, 256)
        y_ref = moe_reference(xt[rows], g_w, w1, w2, layer.cfg.topk, routing=route(xt[rows], layer.gate_w,
                                                                                      layer.cfg.topk))
        if not cpu:
            from tilelang.runtime import errors
            errors.check()
        ok = bool(torch.allclose(yt[rows].float(), y_ref, rtol=3e-2, atol=3e-2 * float(y_ref.abs().max())))
        t_ = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cpu" if cpu else "cuda")
        dist.all_reduce(t_, op=dist.ReduceOp.MIN)
        if not bool(t_.item()):
            return {"error": "TP MoE result check failed"}
        ms = timed(lambda: layer(xt), reps)
        t_ = torch.tensor([ms], dtype=torch.float64, device="cpu" if cpu else "cuda")
        dist.all_reduce(t_, op=dist.ReduceOp.MAX)
        ms = float(t_.item())
        # every rank runs all tokens through 1/world of every expert's FFN
        flops = 6.0 * m["tokens"] * m["topk"] * m["hidden"] * m["ffn"] / mesh.world
        return {"ms": round(ms, 4), "tflops_per_gpu": round(flops / ms / 1e9, 1),
                "comm": "in-kernel two-shot T.comm.all_reduce over IPC (xGMI)"}
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {str(e)[:300]}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-moe", action="store_true", help="time GEMM + attention only")
    ap.add_argument("--gemm-nn", action="store_true",
                    help="B [K, N] for the GEMM phase (the layout before round 5; A/B only)")
    ap.add_argument("--prewarm-ms", type=float, default=None,
                    help="untimed, time-based pre-warm before the --warmup steps (default 300 ms on a GPU): the "
                         "MI355X clocks ramp over the first ~20 ms of dense MFMA work after idle (per-step "
                         "times below); reported as prewarm_ms, never part of the timed region")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the process group and the mesh even at world size 1 (RCCL on a GPU), so "
                         "the MoE runs expert-parallel through the mesh exchange (checked like N > 1)")
    ap.add_argument("--streams", type=int, default=1, choices=[1, 2],
                    help="2: the MoE layer runs on a second HIP stream beside GEMM + attention (the three phases "
                         "are independent; the step ends when both streams have finished)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: tiny shapes on the CPU target under gloo (CI plumbing check)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(relaunch(args))
    world = int(env_world or 1)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")

    import torch
    cpu = args.device == "cpu"
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if not cpu:
        torch.cuda.set_device(local_rank)
    dist = None
    mesh = None
    if world > 1 or args.dist:
        import torch.distributed as dist
        if env_world is None:  # --dist without torchrun: a one-rank rendezvous on this host
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                              LOCAL_RANK="0")
        if cpu:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
        world = dist.get_world_size()
        from tilelang.parallel import init_mesh
        mesh = init_mesh(1, world)
    dev = "cpu" if cpu else "cuda"
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    torch.manual_seed(1234)  # identical expert weights on every rank (EP slices them)
    g, a_, m = (TINY["gemm"], TINY["attn"], TINY["moe"]) if cpu else (GEMM_CFG, ATTN_CFG, MOE_CFG)
    if args.gemm_nn:
        g = dict(g, trans_B=False)
    gemm, (A, B) = build_gemm(dev, g)
    attn, (Q, K, V) = build_attn(dev, a_)
    moe = None
    if not args.no_moe:
        moe, X = build_moe(mesh, dev, m)
        torch.manual_seed(1234 + rank)
        X = torch.randn_like(X.float()).to(X.dtype)  # every rank brings its own tokens

    # correctness guard against the fp32 definition, so a broken kernel cannot post a number:
    # GEMM rows from every 256-row tile band (each row crosses every column tile), attention on
    # four heads spread over the head grid (bshd layout)
    C = gemm(A, B)
    step = max(1, g["M"] // 64)
    i64 = torch.arange(min(64, g["M"]), device=A.device)
    rows = i64 * step + (i64 * 37) % step  # one row per 64-row band, at a varying offset inside it
    Bkn = B.T if g.get("trans_B", False) else B  # [K, N] view
    ref = A[rows].float() @ Bkn.float()
    if not torch.allclose(C[rows].float(), ref, rtol=2e-2, atol=2e-1):
        raise SystemExit("GEMM result check failed")
    O = attn(Q, K, V)
    heads = sorted({0, a_["heads"] // 3, (2 * a_["heads"]) // 3, a_["heads"] - 1})
    q1, k1, v1 = (t[:, :, heads].float().transpose(1, 2) for t in (Q, K, V))
    o_ref = torch.softmax(q1 @ k1.transpose(-1, -2) / q1.shape[-1]**0.5, -1) @ v1
    if not torch.allclose(O[:, :, heads].float().transpose(1, 2), o_ref, rtol=3e-2, atol=3e-2):
        raise SystemExit("attention result check failed")
    ep_note = None
    if moe is not None:
        # MoE layer vs the fp32 definition with the kernel's own routing (exact 16-bit logit ties
        # may pick either expert: models.moe.routing_equivalent).  At N > 1 every rank checks its
        # own tokens after they went through the expert-parallel exchange; a failure of the
        # device exchange (tl/ep.h) falls back to the host all-to-all path instead of posting.
        def moe_ok():
            from tilelang.models.moe import moe_reference, init_moe_weights
            from tilelang.ops.moe import route
            xs = X if mesh is not None else X[:256]  # EP: the whole per-rank batch (fixed layer shape)
            g_w, w1, w2 = (t.to(xs.device) for t in init_moe_weights(moe.cfg))
            ys = moe(xs)
            if not cpu:
                from tilelang.runtime import errors
                errors.check()
            rows = slice(0, 256)
            y_ref = moe_reference(xs[rows], g_w, w1, w2, moe.cfg.topk,
                                  routing=route(xs[rows], moe.gate_w, moe.cfg.topk))
            return bool(torch.allclose(ys[rows].float(), y_ref, rtol=3e-2, atol=3e-2 * float(y_ref.abs().max())))

        def all_ranks(flag):
            if dist is None:
                return flag
            t_ = torch.tensor([1 if flag else 0], dtype=torch.int32, device="cpu" if cpu else "cuda")
            dist.all_reduce(t_, op=dist.ReduceOp.MIN)
            return bool(t_.item())

        try:
            ok = moe_ok()
        except Exception as e:  # noqa: BLE001  (device exchange error: fall back, never post a wrong number)
            ok, ep_note = False, f"{type(e).__name__}: {str(e)[:200]}"
        ok = all_ranks(ok)
        if not ok and mesh is not None and moe._device_ep():
            ep_note = ep_note or "device EP exchange failed the result check"
            moe.ep_mode = "host"
            ok = all_ranks(moe_ok())
        if not ok:
            raise SystemExit("MoE result check failed")

    gemm_flops = 2.0 * g["M"] * g["N"] * g["K"]
    attn_flops = 4.0 * a_["batch"] * a_["heads"] * a_["seq_len"]**2 * a_["dim"]
    moe_flops = 0.0 if moe is None else 6.0 * m["tokens"] * m["topk"] * m["hidden"] * m["ffn"]

    side = torch.cuda.Stream() if (args.streams == 2 and not cpu and moe is not None) else None

    def step():
        if side is not None:
            # fork: the MoE layer on the side stream, GEMM + attention on the main one; join before
            # the step's end event, so the step still covers all three phases' work
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                moe(X)
            gemm(A, B)
            attn(Q, K, V)
            torch.cuda.current_stream().wait_stream(side)
            return
        gemm(A, B)
        attn(Q, K, V)
        if moe is not None:
            moe(X)

    # disclosed pre-warm (the reference's do_bench convention: run for a fixed time before
    # timing, tilelang/profiler/bench.py:63-135): whole steps until prewarm_ms of wall time
    prewarm_ms = (0.0 if cpu else 300.0) if args.prewarm_ms is None else args.prewarm_ms
    prewarm_steps = 0
    # per-step device timestamps (events created before the warm-up: nothing between the last
    # warm-up step and the first timed one but the required sync / barrier)
    evs = None if cpu else [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    step()  # the first full-size step: the MoE's first call at 2048 tokens compiles its kernels
    sync()
    tp0 = time.perf_counter()
    while (time.perf_counter() - tp0) * 1e3 < prewarm_ms:
        for _ in range(4):
            step()
            prewarm_steps += 1
        sync()
    prewarm_ms = (time.perf_counter() - tp0) * 1e3
    for _ in range(args.warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if evs is not None:
            evs[i].record()
        step()
    if evs is not None:
        evs[-1].record()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0

    # per-phase times, measured after the timed region (MoE includes its all-to-alls).  On a GPU
    # each phase is timed on the device: two attention calls ahead of the first event keep the
    # queue busy while the host enqueues the n calls, so the span between the events is the
    # phase's device time, as inside the step (the kernel trace of a step shows the same span);
    # the host's enqueue cost of one call is reported on its own (host_ms_per_call)
    host_ms = {}

    def timed(fn, n, name=None):
        sync()
        if dist is not None:
            dist.barrier()
        if cpu or dist is not None:  # collectives inside: wall time
            t = time.perf_counter()
            for _ in range(n):
                fn()
            sync()
            return (time.perf_counter() - t) / n * 1e3
        for _ in range(2):
            attn(Q, K, V)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        if name:
            host_ms[name] = round((time.perf_counter() - t) / n * 1e3, 4)
        e1.record()
        sync()
        return e0.elapsed_time(e1) / n

    step_ms = [] if evs is None else [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    reps = 2 if cpu else 10
    gemm_ms = timed(lambda: gemm(A, B), reps, "gemm")
    attn_ms = timed(lambda: attn(Q, K, V), reps, "attn")
    moe_ms = timed(lambda: moe(X), reps, "moe") if moe is not None else 0.0
    moe_comm_ms = 0.0
    if moe is not None and mesh is not None:
        if moe._device_ep():
            # the device exchange alone: dispatch + receive wait, return + wait (FFN skipped)
            from tilelang.ops import moe as KM
            ids_, _ = KM.route(X, moe.gate_w, m["topk"])
            xc = moe._exchange[1]
            y0 = torch.zeros(xc.W * xc.cap, m["hidden"], device=dev, dtype=X.dtype)
            yd = torch.arange(xc.W * xc.cap, device=dev, dtype=torch.int32)

            def exch():
                _, _, rc, _ = xc.dispatch(X, ids_)
                xc.combine_rows(y0, yd, rc)

            moe_comm_ms = timed(exch, reps)
        else:
            # the two all-to-alls alone (same byte counts as the layer's dispatch + return)
            from tilelang.parallel import collectives as Cl
            rows = X.shape[0] * m["topk"]
            per = [rows // world] * world
            per[-1] += rows - sum(per)
            payload = torch.randn(rows, m["hidden"], device=dev).to(X.dtype)
            moe_comm_ms = timed(lambda: (Cl.all_to_all_v(payload, per), Cl.all_to_all_v(payload, per)), reps)
    tp = tp_phase(mesh, dev, m, X, dist, timed, reps, cpu) if (moe is not None and mesh is not None) else None
    # box-speed normaliser: the vendor library (hipBLASLt via torch.matmul) on the same fp16 GEMM,
    # same process, same clocks; the driver-vs-builder gap of a run can be read against it
    for _ in range(3):  # hipBLASLt loads and selects its kernel on the first calls
        torch.matmul(A, Bkn)
    vendor_ms = timed(lambda: torch.matmul(A, Bkn), reps)
    # the same normaliser for attention: PyTorch's fused SDPA (the ROCm flash-attention backend)
    # on the bench shape, bf16, non-causal, same process
    attn_vendor_ms = None
    if not cpu:
        try:
            qs, ks_, vs_ = (t.transpose(1, 2) for t in (Q, K, V))
            sdpa = torch.nn.functional.scaled_dot_product_attention
            for _ in range(3):
                sdpa(qs, ks_, vs_)
            attn_vendor_ms = timed(lambda: sdpa(qs, ks_, vs_), reps)
        except Exception:  # noqa: BLE001  (a normaliser only: never fatal)
            attn_vendor_ms = None
    dev_id = -1 if cpu else torch.cuda.current_device()
    bus = "cpu" if cpu else str(getattr(torch.cuda.get_device_properties(dev_id), "pci_bus_id", dev_id))
    ids = [None] * world
    if dist is not None:
        dist.all_gather_object(ids, (rank, local_rank, dev_id, bus))
    else:
        ids = [(rank, local_rank, dev_id, bus)]

    t = torch.tensor([elapsed, gemm_ms, attn_ms, moe_ms, moe_comm_ms, vendor_ms], dtype=torch.float64,
                     device="cpu" if cpu else "cuda")
    # per-rank phase times (ms) and the world size the backend itself reports: a one-element
    # all_reduce of ones over RCCL (nccl) / gloo
    per_rank = [t.tolist()]
    world_seen = 1
    if dist is not None:
        g_ = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g_, t)
        per_rank = [x.tolist() for x in g_]
        one = torch.ones(1, dtype=torch.int32, device="cpu" if cpu else "cuda")
        dist.all_reduce(one)
        world_seen = int(one.item())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, gemm_ms, attn_ms, moe_ms, moe_comm_ms, vendor_ms = t.tolist()
    ms_per_step = elapsed / args.steps * 1e3
    step_flops = gemm_flops + attn_flops + moe_flops
    tflops = step_flops * world * args.steps / elapsed / 1e12
    # the reference's time for the same per-rank work at its published rates
    ref_step_s = (gemm_flops + moe_flops) / (REF_GEMM_TF * 1e12) + attn_flops / (REF_ATTN_TF * 1e12)
    ref_tflops = step_flops / ref_step_s / 1e12 * world
    if rank == 0:
        out = {
            "metric": METRIC,
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
            "data": "synthetic (torch.randn inputs, random-init expert weights)",
            "config": {
                "model": (f"fp16 GEMM {g['M']}x{g['N']}x{g['K']} + FlashAttention-2 fwd bf16 b{a_['batch']} "
                          f"h{a_['heads']} s{a_['seq_len']} d{a_['dim']}"
                          + ("" if moe is None else f" + MoE FFN {m['experts']} experts top-{m['topk']} "
                             f"h{m['hidden']} f{m['ffn']} {m['tokens']} tok/rank"
                             + (" (EP)" if mesh is not None else " (all experts local)"))),
                "global_batch": world,
                "seq_len": a_["seq_len"],
                "parallelism": (f"dp{world}" if moe is None or mesh is None else f"dp{world}+ep{world}"),
            },
            "gemm_tflops": round(gemm_flops / gemm_ms / 1e9, 1),
            "gemm_vendor_tflops": round(gemm_flops / vendor_ms / 1e9, 1),
            "attn_tflops": round(attn_flops / attn_ms / 1e9, 1),
            "attn_vendor_tflops": (round(attn_flops / attn_vendor_ms / 1e9, 1) if attn_vendor_ms else None),
            "moe_tflops_per_gpu": round(moe_flops / moe_ms / 1e9, 1) if moe is not None else None,
            "moe_comm_fraction": round(moe_comm_ms / moe_ms, 3) if moe is not None and moe_ms > 0 else None,
            "streams": args.streams if side is not None else 1,
            "phase_timing": ("wall, 1 call per rep" if (cpu or dist is not None) else
                             "device time (events behind a queue-filling blocker), 10 calls"),
            "host_ms_per_call": host_ms or None,
            "ep_exchange": (None if mesh is None or moe is None else
                            (("device (tl/ep_cpu.h protocol over /dev/shm, no host sync)" if cpu else
                              "device (tl/ep.h, IPC over xGMI, no host sync)") if moe._device_ep() else
                             f"host ({'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} "
                             "all_to_all_v)")),
            "ep_fallback_reason": ep_note,
            "tp_moe": tp,
            "pct_of_mfma_peak": round(100.0 * tflops / world / PEAK_BF16_TF, 1),
            "prewarm_ms": round(prewarm_ms, 1),
            "prewarm_steps": prewarm_steps,
            "step_ms_first": round(step_ms[0], 4) if step_ms else None,
            "step_ms_median": round(sorted(step_ms)[len(step_ms) // 2], 4) if step_ms else None,
            "step_ms_last": round(step_ms[-1], 4) if step_ms else None,
            "step_ms_min": round(min(step_ms), 4) if step_ms else None,
            "step_ms_rank0": [round(x, 3) for x in step_ms],
            "gemm_dtype": "float16",
            "gemm_layout": "NT (B [N, K])" if g.get("trans_B", False) else "NN (B [K, N])",
            "attn_dtype": "bfloat16",
            "moe_dtype": "bfloat16",
            "device": args.device,
            "world_size": (dist.get_world_size() if dist is not None else 1),
            "dist_world_observed": world_seen,
            "per_rank_ms": [{"rank": r, "steps_total": round(v[0] * 1e3, 3), "gemm": round(v[1], 4),
                             "attn": round(v[2], 4), "moe": round(v[3], 4), "moe_comm": round(v[4], 4)}
                            for r, v in enumerate(per_rank)],
            "backend": (dist.get_backend() if dist is not None else None),
            "ranks": [{"rank": r, "local_rank": lr, "device": d, "pci_bus": b} for r, lr, d, b in ids],
        }
        print(json.dumps(out), flush=True)
    if mesh is not None:
        from tilelang.parallel import shutdown_mesh
        shutdown_mesh()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
