"""MoE FFN (grouped-GEMM experts) — local, expert-parallel (all-to-all) and tensor-parallel
(in-kernel mesh tile all-reduce) on the CPU target, checked against the fp32 PyTorch definition."""
import pytest
import torch

from tilelang.models.moe import MoEConfig, MoELayer, init_moe_weights, moe_reference, routing_equivalent
from tilelang.ops.moe import pack_by_expert, max_padded_rows
from tilelang.parallel import VirtualMesh

CFG = MoEConfig(hidden=64, ffn=128, n_experts=4, topk=2, dtype=torch.float32, block_M=16)


def test_pack_by_expert():
    ids = torch.tensor([2, 0, 2, 3, 0, 2, 2])
    mr = max_padded_rows(7, 4, 4)
    dest, te, counts = pack_by_expert(ids, 4, 4, mr)
    assert counts.tolist() == [2, 0, 4, 1]
    # full tiles first (expert 2's four rows), then one partial tile per expert (0, then 3)
    assert dest.tolist() == [0, 4, 1, 8, 5, 2, 3]
    assert te.tolist()[:3] == [2, 0, 3] and all(t == -1 for t in te.tolist()[3:])


def test_moe_local_cpu():
    torch.manual_seed(0)
    x = torch.randn(37, CFG.hidden)
    layer = MoELayer(CFG, "local", device="cpu")
    g, w1, w2 = init_moe_weights(CFG)
    torch.testing.assert_close(layer(x), moe_reference(x, g, w1, w2, CFG.topk), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("mode", ["ep", "tp"])
def test_moe_mesh_cpu(mode):
    vm = VirtualMesh(1, 2, "cpu", workspace_bytes=64 << 20)
    torch.manual_seed(1)
    xs = [torch.randn(29, CFG.hidden) for _ in range(2)]
    if mode == "tp":
        xs[1] = xs[0].clone()  # tensor parallel: replicated tokens
    g, w1, w2 = init_moe_weights(CFG)

    def fn(ctx):
        layer = MoELayer(CFG, mode, mesh=ctx, device="cpu")
        return layer(xs[ctx.rank])

    outs = vm.run(fn)
    vm.check()
    for r in range(2):
        torch.testing.assert_close(outs[r], moe_reference(xs[r], g, w1, w2, CFG.topk), rtol=1e-4, atol=1e-4)


def test_router_and_align_match_reference():
    """Device router top-k == torch softmax/topk/renorm; the dispatch plan places every
    assignment in its expert's padded row block (stable and atomic variants)."""
    from tilelang.ops import moe as K
    from tilelang.models.moe import route
    torch.manual_seed(3)
    x = torch.randn(300, 64)
    g = torch.randn(8, 64)
    ids, w = K.route(x, g, 2)
    rid, rw = route(x, g, 2)
    assert (ids.long() == rid).all()
    torch.testing.assert_close(w, rw)
    for stable in (True, False):
        mr = K.max_padded_rows(600, 8, 16)
        dest, row_src, te, counts, trows = K.dispatch_plan(ids, 8, 16, mr, div=2, stable=stable)
        flat = ids.reshape(-1).long()
        assert counts.tolist() == torch.bincount(flat, minlength=8).tolist()
        d = dest.long()
        assert len(set(d.tolist())) == flat.numel()
        assert (te[d // 16].long() == flat).all()
        assert (row_src[d].long() == torch.arange(600) // 2).all()
        ends = torch.zeros(mr // 16, dtype=torch.long)  # valid rows of every tile: a prefix
        for r in d.tolist():
            ends[r // 16] = max(int(ends[r // 16]), r % 16 + 1)
        assert trows.long().tolist() == ends.tolist()
        if stable:  # assignment order kept inside every expert
            for e in range(8):
                de = d[flat == e]
                assert (de[1:] > de[:-1]).all()


@pytest.mark.gpu
def test_moe_layer_gpu():
    cfg = MoEConfig(hidden=512, ffn=256, n_experts=8, topk=2, dtype=torch.bfloat16, block_M=128)
    torch.manual_seed(0)
    x = torch.randn(1000, cfg.hidden, device="cuda").to(cfg.dtype)
    layer = MoELayer(cfg, "local", device="cuda")
    out = layer(x).float()
    g, w1, w2 = (t.to("cuda") for t in init_moe_weights(cfg))
    from tilelang.ops import moe as K
    from tilelang.models.moe import routing_equivalent
    ids, w = K.route(x, g, cfg.topk)  # fused MFMA router + top-k
    assert routing_equivalent(x, g, cfg.topk, ids, w)
    ref = moe_reference(x, g, w1, w2, cfg.topk, routing=(ids, w))
    torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2 * ref.abs().max().item())


def test_tp_expert_gemm_workspace_and_grid():
    """The tensor-parallel expert GEMM (all-reduce inside the kernel) runs a persistent grid and
    two-shot all-reduces: its mesh workspace is >= 10x smaller than one slot per (tile block, rank)
    of whole fp32 tiles."""
    from tilelang.ops.moe import expert_gemm_kernel
    from tilelang.parallel import device_mesh_config
    max_rows, K, N, E, bm, bn = 4352, 256, 4096, 8, 128, 128
    with device_mesh_config(1, 8):
        k = expert_gemm_kernel(max_rows, K, N, E, "bfloat16", "cpu", bm, bn, reduce_mesh="all", mesh_shape=(1, 8))
    meta = k.artifact.kernels[0].mesh
    tiles = (max_rows // bm) * (N // bn)
    one_shot_per_tile = tiles * 8 * bm * bn * 4
    assert meta["nblocks"] == 256 and meta["slot_bytes"] == bm * bn * 4 // 8
    assert meta["ws_bytes"] * 10 <= one_shot_per_tile, (meta, one_shot_per_tile)


@pytest.mark.parametrize("ext", [0, 16])
@pytest.mark.parametrize("n_cu", [3, 5, 8])
def test_moe_tail_balanced_cpu(n_cu, ext):
    """Tail-balanced expert GEMMs: whole leading units, the trailing partial round as narrow tiles
    (n_cu chosen so the tail has 1-2 rounds of narrow tiles, or is empty); ``ext``: row-tile slots
    of block_M + ext rows with every expert's rows spread evenly over its slots."""
    cfg = MoEConfig(hidden=64, ffn=64, n_experts=4, topk=2, dtype=torch.float32, block_M=16,
                    gemm_cfg=dict(block_N=64, block_K=32, num_stages=2, threads=128, stream_k=True, n_cu=n_cu,
                                  tail_split=2, ext_M=ext))
    layer = MoELayer(cfg, "local", device="cpu")
    x = torch.randn(50, 64)
    out = layer(x).float()
    g, w1, w2 = init_moe_weights(cfg)
    ref = moe_reference(x, g, w1, w2, cfg.topk)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_moe_tail_balanced_gpu():
    """The bench's MoE layer shape with the tail-balanced grid on vs off."""
    cfg = MoEConfig(hidden=1024, ffn=512, n_experts=8, topk=2, dtype=torch.bfloat16, block_M=256,
                    gemm_cfg=dict(block_N=256, block_K=64, num_stages=2, threads=512))
    torch.manual_seed(0)
    x = torch.randn(2048, cfg.hidden, device="cuda").to(cfg.dtype)
    layer = MoELayer(cfg, "local", device="cuda")
    g, w1, w2 = (t.to("cuda") for t in init_moe_weights(cfg))
    from tilelang.ops import moe as K
    ref = moe_reference(x, g, w1, w2, cfg.topk, routing=K.route(x, g, cfg.topk))
    for sk, ph, skip, ext, quad in ((True, False, True, 0, True), (False, False, True, 0, True),
                                    (True, True, True, 0, False), (True, True, False, 0, False),
                                    (True, False, True, 32, True), (True, False, True, 32, False),
                                    (True, False, False, 32, True)):
        # phased: K-half ring with register-prefetched fragments; skip: padding waves skip
        # their reads and MFMAs (T.gemm(valid_m=)) inside the prefetched schedule too; ext: 288-row
        # slots (256 + a 32-row extension GEMM on the same W tile), rows spread evenly per expert;
        # quad: the whole-tile loop as tl::gemm_quad_nt_x (gather + extension + valid_m)
        layer.cfg.gemm_cfg = dict(block_N=256, block_K=64, num_stages=2, threads=512, stream_k=sk, phased=ph,
                                  skip_padding=skip, ext_M=ext, quad=quad)
        out = layer(x).float()
        torch.testing.assert_close(out, ref, rtol=3e-2, atol=3e-2 * ref.abs().max().item())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_fused_router_cpu(dt):
    """MFMA router GEMM + top-k in one kernel (16-bit activations): a valid top-k of the
    reference probabilities (exact 16-bit logit ties may break the other way)."""
    from tilelang.ops import moe as K
    torch.manual_seed(0)
    x = torch.randn(100, 512).to(dt)
    g = (torch.randn(8, 512) * 0.05).to(dt)
    ids, w = K.route(x, g, 2)
    assert routing_equivalent(x, g, 2, ids, w)


def _mesh_moe_worker(rank, world, port, mode, q):
    """One rank of a 2- or 4-process mesh sharing GPU 0 (or its own GPU on a multi-GPU box): the EP
    (device exchange, tl/ep.h) or TP (in-kernel all-reduce) MoE layer vs the fp32 definition."""
    import os
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tilelang.parallel import init_mesh, shutdown_mesh
        from tilelang.runtime import errors
        from tilelang.ops import moe as K
        dev = f"cuda:{rank % torch.cuda.device_count()}"
        torch.cuda.set_device(dev)
        mesh = init_mesh(1, world, device=dev)
        gcfg = None
        if mode.endswith("_ext"):  # the bench's expert GEMM config: 256 + 32-row slots (ext_M)
            mode = mode[:-4]
            gcfg = dict(block_N=256, block_K=64, num_stages=2, threads=512, ext_M=32)
        cfg = MoEConfig(hidden=512, ffn=256, n_experts=8, topk=2, dtype=torch.bfloat16,
                        block_M=256 if gcfg else 128, gemm_cfg=gcfg)
        layer = MoELayer(cfg, mode, mesh=mesh, device=dev)
        g, w1, w2 = (t.to(dev) for t in init_moe_weights(cfg))
        for step in range(4):  # several steps: both buffer parities, flag reuse across steps
            torch.manual_seed(100 + step + (0 if mode == "tp" else rank))  # TP: replicated tokens
            x = torch.randn(300 + 17 * step, cfg.hidden, device=dev).to(cfg.dtype)
            out = layer(x).float()
            errors.check()
            ids, w = K.route(x, g, cfg.topk)
            ref = moe_reference(x, g, w1, w2, cfg.topk, routing=(ids, w))
            err = (out - ref).abs().max().item()
            if not err <= 3e-2 * ref.abs().max().item():
                raise AssertionError(f"rank {rank} step {step}: max err {err} vs {ref.abs().max().item()}")
        mesh.check()
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("mode,world", [("ep", 2), ("tp", 2), ("ep_ext", 2), ("ep", 4), ("tp", 4)])
def test_moe_mesh_processes_gpu(mode, world):
    """2 and 4 processes sharing the box's GPU (distinct GPUs on a multi-GPU box)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mesh_moe_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=400) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(world)}, res


def test_ep_kernels_compile():
    """The device EP exchange (tl/ep.h) builds for gfx950 at the bench shape (8 ranks)."""
    from tilelang.ops import ep
    W, n_tok, H, topk, E = 8, 2048, 4096, 2, 8
    cap = n_tok * min(topk, E // W)
    for k in (ep.dispatch_kernel(n_tok, H, topk, W, E // W, cap, "bfloat16"), ep.recv_wait_kernel(W, cap, H * 2),
              ep.ret_kernel(W * cap + 256, H, W, cap, "bfloat16"), ep.ret_wait_kernel(W)):
        assert len(k.code[0]) > 0
    eids, recv, ret, total = ep.layout_bytes(W, cap, H * 2)
    assert recv % 4096 == 0 and total == ret + 2 * W * cap * H * 2


def _tail_ksplit_check(device, S):
    """K-split tail of the tail-balanced expert GEMM (last arriver sums the partials and runs the
    SwiGLU / store epilogue) against the narrow-tile tail, same routing."""
    from tilelang.ops import moe as K
    g = torch.Generator().manual_seed(0)
    T_, H, F, E, TOP = (96, 128, 64, 4, 2) if device == "cpu" else (2048, 1024, 512, 8, 2)
    BM = 16 if device == "cpu" else 256
    x = torch.randn(T_, H, generator=g).to(device)
    w1 = (torch.randn(E, 2 * F, H, generator=g) * 0.1).to(device)
    w2 = (torch.randn(E, H, F, generator=g) * 0.1).to(device)
    if device != "cpu":
        x, w1, w2 = x.bfloat16(), w1.bfloat16(), w2.bfloat16()
    ids = torch.randint(0, E, (T_ * TOP, ), generator=g, dtype=torch.int32).to(device)
    base = dict(n_cu=4, block_N=32, block_K=32, threads=128) if device == "cpu" else dict(block_N=256, block_K=64)
    ys = []
    for extra in (dict(tail_split=1), dict(tail_ksplit=S)):
        y, dest = K.expert_ffn_padded(x, ids, TOP, w1, w2, BM, cfg=dict(base, stream_k=True, **extra),
                                      w1_interleaved=True)
        ys.append(y[dest.long()].float())
    torch.testing.assert_close(ys[1], ys[0], rtol=2e-2, atol=2e-2 * float(ys[0].abs().max()))


def test_moe_tail_ksplit_cpu():
    _tail_ksplit_check("cpu", 2)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [2, 4])
def test_moe_tail_ksplit_gpu(S):
    _tail_ksplit_check("cuda", S)


def _dead_peer_worker(rank, world, port, q, device="cuda"):
    """Rank 1 skips the expert-parallel layer of step 1 (a dead or diverged peer): rank 0's
    device exchange must raise MeshError within ONE wait budget (TL_EP_TIMEOUT_S = 2 s; every
    later wait of the step gives up at once), then both ranks fall back to the host all-to-all
    (bench.py's fallback) and post a result checked against the fp32 definition."""
    import os
    import time
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TL_EP_TIMEOUT_S="2")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tilelang.parallel import init_mesh, shutdown_mesh
        from tilelang.parallel.mesh import MeshError
        from tilelang.runtime import errors
        from tilelang.ops import moe as K
        if device == "cpu":  # the CPU build of the exchange (tl/ep_cpu.h) over /dev/shm
            dev = "cpu"
            cfg = MoEConfig(hidden=64, ffn=128, n_experts=8, topk=2, dtype=torch.float32, block_M=16)
        else:
            dev = f"cuda:{rank % torch.cuda.device_count()}"
            torch.cuda.set_device(dev)
            cfg = MoEConfig(hidden=512, ffn=256, n_experts=8, topk=2, dtype=torch.bfloat16, block_M=128)
        mesh = init_mesh(1, world, device=dev)
        layer = MoELayer(cfg, "ep", mesh=mesh, device=dev)
        g, w1, w2 = (t.to(dev) for t in init_moe_weights(cfg))
        torch.manual_seed(7 + rank)
        x = torch.randn(256, cfg.hidden, device=dev).to(cfg.dtype)
        layer(x)
        if dev != "cpu":
            errors.check()  # step 0: both ranks healthy
        dist.barrier()
        elapsed, raised = None, None
        if rank == 0:
            t0 = time.time()
            try:
                layer(x)
                if dev != "cpu":
                    errors.check()
                mesh.check()
            except MeshError as e:
                raised = str(e)
            elapsed = time.time() - t0
        dist.barrier()
        if rank == 0:
            if raised is None:
                raise AssertionError("no MeshError although the peer skipped its dispatch")
            # one 2 s budget (plus launch/compile slack), not one per wait: W waits x 4 kernels
            # would be >= 16 s with serialised budgets
            if elapsed > 8.0:
                raise AssertionError(f"MeshError after {elapsed:.1f} s: waits were serialised ({raised})")
        mesh.err.zero_()
        layer.ep_mode = "host"  # bench.py's fallback: RCCL/gloo all_to_all_v
        out = layer(x).float()
        ids, w = K.route(x, g, cfg.topk)
        ref = moe_reference(x, g, w1, w2, cfg.topk, routing=(ids, w))
        err = (out - ref).abs().max().item()
        if not err <= 3e-2 * ref.abs().max().item():
            raise AssertionError(f"rank {rank}: host fallback max err {err}")
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok" if rank else f"ok {elapsed:.2f}s"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("device", [pytest.param("cuda", marks=pytest.mark.gpu), "cpu"])
def test_ep_dead_peer_fails_fast(device):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dead_peer_worker, args=(r, 2, port, q, device)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    assert res[1] == "ok" and res[0].startswith("ok"), res
    print("dead peer detected after", res[0])


def test_router_k_split_matches_fused(monkeypatch):
    """K-split router (partial logits by plain stores, summed + rounded in the top-k kernel) picks
    the same experts with the same weights as the fused one-pass router."""
    from tilelang.ops import moe as K
    torch.manual_seed(0)
    x = torch.randn(256, 1024).to(torch.bfloat16)
    g = (torch.randn(8, 1024) * 0.05).to(torch.bfloat16)
    ids0, w0 = K.route(x, g, 2)
    monkeypatch.setattr(K, "ROUTER_SPLITS", 4)
    ids1, w1 = K.route(x, g, 2)
    assert torch.equal(ids0, ids1)
    torch.testing.assert_close(w0, w1)


@pytest.mark.gpu
def test_router_wide_matches_fused(monkeypatch):
    """router_wide_kernel (K chunks side by side in one tile GEMM, the default on gfx950) picks the
    same experts with the same weights as the fused one-wave router."""
    from tilelang.ops import moe as K
    torch.manual_seed(0)
    x = torch.randn(512, 2048, device="cuda").to(torch.bfloat16)
    g = (torch.randn(8, 2048, device="cuda") * 0.05).to(torch.bfloat16)
    ids0, w0 = K.route(x, g, 2)
    monkeypatch.setattr(K, "ROUTER_WIDE", False)
    ids1, w1 = K.route(x, g, 2)
    assert torch.equal(ids0, ids1)
    torch.testing.assert_close(w0, w1)
