"""The bench's world-8 configuration, rehearsed on the CPU tier: 8 gloo processes, one per rank,
exchanging through /dev/shm workspaces with the same device protocols as the GPUs (tl/mesh_cpu.h
for T.comm, tl/ep_cpu.h for the expert-parallel exchange of tl/ep.h).

  * T.comm broadcast / all_gather / one-shot all_reduce / two-shot all_reduce_tile on 1x8 and 2x4
    process meshes (the MoE TP and the bench's 1x8 mesh);
  * the MoE layer expert-parallel through the device exchange at the bench's structure: 8
    experts, one per rank, several steps (both buffer parities and the slot-reuse handshakes);
  * the MoE layer tensor-parallel at the bench's slice: ffn 2048 over 8 ranks = 256 per rank,
    partial outputs summed by the in-kernel two-shot all-reduce.
Every rank checks against the fp32 definition (reference counterpart:
examples/deepseek_v32/inference/model.py:787-850, generate.py:100-108)."""
import os
import socket

import pytest
import torch

WORLD = 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, args, world=WORLD, timeout=600):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + tuple(args)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=timeout) for _ in range(world))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res == {r: "ok" for r in range(world)}, res


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _comm_worker(rank, world, port, q, nrow, ncol):
    try:
        dist = _init(rank, world, port)
        import tilelang
        import tilelang.language as T
        from tilelang.parallel import init_mesh, shutdown_mesh, device_mesh_config
        ctx = init_mesh(nrow, ncol, device="cpu")
        M, N, blocks = 32, 64, 2
        with device_mesh_config(nrow, ncol):

            @T.prim_func
            def main(A: T.Tensor((M * blocks, N), "float32"), B: T.Tensor((M * blocks, N), "float32"),
                     G: T.Tensor((world, M * blocks, N), "float32"), R: T.Tensor((M * blocks, ), "float32"),
                     S_: T.Tensor((M * blocks, N), "float32"), H_: T.Tensor((M * blocks, N), "float32")):
                with T.Kernel(blocks, threads=128) as bx:
                    a = T.alloc_fragment((M, N), "float32")
                    b = T.alloc_fragment((M, N), "float32")
                    g = T.alloc_shared((world, M, N), "float32")
                    r = T.alloc_fragment((M, ), "float32")
                    s = T.alloc_fragment((M, N), "float32")
                    h = T.alloc_fragment((M, N), "float32")
                    T.copy(A[bx * M, 0], a)
                    T.comm.broadcast(a, b, (0, ncol - 1), direction="all")
                    T.copy(b, B[bx * M, 0])
                    T.comm.all_gather(a, g, direction="all")
                    T.copy(g, G[0:world, bx * M:(bx + 1) * M, 0:N])
                    T.comm.all_reduce(a, r, "sum", "all", dim=1)             # one-shot, row sums
                    T.copy(r, R[bx * M])
                    T.comm.all_reduce_tile(a, s, "sum", "all")               # two-shot (8 members)
                    T.copy(s, S_[bx * M, 0])
                    T.comm.all_reduce_tile(a, h, "max", "h")                 # row group
                    T.copy(h, H_[bx * M, 0])

            k = tilelang.compile(main, target="cpu")
        torch.manual_seed(rank)
        A = torch.randn(M * blocks, N)
        outs = (torch.zeros_like(A), torch.zeros(world, M * blocks, N), torch.zeros(M * blocks), torch.zeros_like(A),
                torch.zeros_like(A))
        for _ in range(3):  # epochs advance, no workspace reset
            k(A, *outs)
        ctx.check()
        As = [torch.zeros_like(A) for _ in range(world)]
        dist.all_gather(As, A)
        B, G, R, S_, H_ = outs
        torch.testing.assert_close(B, As[ncol - 1])
        torch.testing.assert_close(G, torch.stack(As))
        torch.testing.assert_close(R, sum(a.sum(1) for a in As), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(S_, sum(As), rtol=1e-5, atol=1e-4)
        row = [As[(rank // ncol) * ncol + c] for c in range(ncol)]
        torch.testing.assert_close(H_, torch.stack(row).amax(0))
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("nrow,ncol", [(1, 8), (2, 4)])
def test_comm_world8_process_mesh_cpu(nrow, ncol):
    _spawn(_comm_worker, (nrow, ncol))


def _moe_worker(rank, world, port, q, mode):
    try:
        dist = _init(rank, world, port)
        from tilelang.parallel import init_mesh, shutdown_mesh
        from tilelang.models.moe import MoEConfig, MoELayer, init_moe_weights, moe_reference
        from tilelang.ops import moe as K
        mesh = init_mesh(1, world, device="cpu")
        # the bench's structure: 8 experts over 8 ranks (one each), top-2; ffn 2048 -> a TP slice of
        # 256 per rank; hidden and tokens small for the CPU target
        cfg = MoEConfig(hidden=64, ffn=2048, n_experts=8, topk=2, dtype=torch.float32, block_M=16)
        layer = MoELayer(cfg, mode, mesh=mesh, device="cpu")
        if mode == "ep":
            assert layer._device_ep(), "the CPU process mesh must take the device exchange"
        g, w1, w2 = init_moe_weights(cfg)
        for step in range(4):  # both parities, RFREE / TFREE reuse across steps
            torch.manual_seed(100 + step + (0 if mode == "tp" else rank))  # TP: replicated tokens
            x = torch.randn(32, cfg.hidden)  # one layer shape: one exchange, epochs 1..4
            out = layer(x)
            ids, w = K.route(x, g, cfg.topk)
            ref = moe_reference(x, g, w1, w2, cfg.topk, routing=(ids, w))
            torch.testing.assert_close(out.float(), ref, rtol=2e-4, atol=2e-4 * float(ref.abs().max()))
        mesh.check()
        if mode == "ep":
            xc = layer._exchange[1]
            assert xc.target == "cpu" and xc.W == world and xc.epoch == 4
        shutdown_mesh()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("mode", ["ep", "tp"])
def test_moe_world8_process_mesh_cpu(mode):
    _spawn(_moe_worker, (mode, ))


def _bench_worker(rank, world, port, q):
    try:
        import json
        import subprocess
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        if rank:
            q.put((rank, "ok"))
            return
        env = dict(os.environ, OMP_NUM_THREADS="1")
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--device", "cpu",
                            "--steps", "1", "--warmup", "1"], capture_output=True, text=True, env=env, timeout=900)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert r.returncode == 0 and line, r.stderr[-2000:]
        out = json.loads(line[-1])
        assert out["n_gpus"] == 8 and out["world_size"] == 8
        assert out["ep_exchange"].startswith("device"), out["ep_exchange"]
        assert out["tp_moe"] and "error" not in out["tp_moe"], out["tp_moe"]
        assert out["dist_world_observed"] == 8
        q.put((rank, "ok"))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def test_bench_world8_cpu():
    """bench.py --gpus 8 --device cpu: the driver's N=8 launch path (torch.distributed.run, one rank
    per 'GPU'), EP through the device exchange protocol, TP through the in-kernel all-reduce."""
    _spawn(_bench_worker, (), world=1, timeout=1000)
