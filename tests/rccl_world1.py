"""RCCL (``nccl`` backend) at world size 1 on one MI355X -- run under torchrun by
tests/test_gpu_rccl.py (SURVEY §7.5 "RCCL world size 1 (loopback)").

Covers every multi-GPU code path one GPU can execute:
  * ``init_mesh`` over the nccl process group: ProcessMesh with its row / column groups
  * host collectives over RCCL: all_reduce, broadcast, all_gather, reduce_scatter, all_to_all,
    all_to_all_v, put, barrier
  * a ``T.comm`` kernel (broadcast / all_gather / all_reduce / all_reduce_tile) on the IPC
    workspace of fine-grained memory (world 1: the rank's own buffer)
  * the MoE layer in expert-parallel mode: the device exchange (tl/ep.h over the symmetric
    buffer) and the host fallback (RCCL all_to_all_v), both against the fp32 definition
  * the tensor-parallel MoE layer (in-kernel T.comm all-reduce of the down projection)
Prints one ``RCCL_WORLD1_OK`` line on success; any failure raises (non-zero exit).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from tilelang.parallel import init_mesh, shutdown_mesh
    from tilelang.parallel import collectives as C
    from tilelang.runtime import errors

    mesh = init_mesh(1, 1, backend="nccl")
    assert dist.get_backend() == "nccl", dist.get_backend()
    assert dist.get_world_size() == 1 and mesh.world == 1
    assert mesh.device.type == "cuda"
    assert len(mesh.row_groups) == 1 and len(mesh.col_groups) == 1
    dev = mesh.device
    torch.manual_seed(0)

    # ---- host collectives over RCCL (world 1: identities, but every call goes through RCCL) --
    for d in ("all", "h", "v"):
        assert dist.get_backend(mesh.group(d)) == "nccl"
    x = torch.randn(64, 128, device=dev)
    y = x.clone()
    C.all_reduce(y, "sum")
    torch.testing.assert_close(y, x)
    C.all_reduce(y, "max", direction="h")
    torch.testing.assert_close(y, x)
    g = C.all_gather(x, direction="v")
    assert g.shape == (1, 64, 128)
    torch.testing.assert_close(g[0], x)
    b = x.clone()
    C.broadcast(b, 0)
    torch.testing.assert_close(b, x)
    rs = C.reduce_scatter(x.clone(), "sum")
    torch.testing.assert_close(rs, x)
    a2a = C.all_to_all(x.clone())
    torch.testing.assert_close(a2a, x)
    out, rc = C.all_to_all_v(x.clone(), [64])
    assert rc == [64]
    torch.testing.assert_close(out, x)
    C.put(x.clone(), 0, 0)
    C.barrier()

    # ---- T.comm kernel on the mesh workspace ------------------------------------------------
    import tilelang
    import tilelang.language as T
    from tilelang.parallel import device_mesh_config
    M, N = 64, 128
    with device_mesh_config(1, 1):

        @T.prim_func
        def comm(A: T.Tensor((M, N), "float16"), B: T.Tensor((M, N), "float16"), G: T.Tensor((1, M, N), "float16"),
                 R: T.Tensor((M, ), "float32"), S_: T.Tensor((M, N), "float32")):
            with T.Kernel(1, threads=256):
                a = T.alloc_fragment((M, N), "float16")
                bb = T.alloc_fragment((M, N), "float16")
                f = T.alloc_fragment((M, N), "float32")
                f2 = T.alloc_fragment((M, N), "float32")
                gs = T.alloc_shared((1, M, N), "float16")
                r = T.alloc_fragment((M, ), "float32")
                T.copy(A, a)
                T.comm.broadcast(a, bb, (0, 0), direction="all")
                T.copy(bb, B)
                T.comm.all_gather(a, gs, direction="all")
                T.copy(gs, G)
                for i, j in T.Parallel(M, N):
                    f[i, j] = a[i, j]
                T.comm.all_reduce(f, r, "sum", "all", dim=1)
                T.copy(r, R)
                T.comm.all_reduce_tile(f, f2, "sum", "all")
                T.copy(f2, S_)

        k = tilelang.compile(comm, target="hip")
    A = torch.randn(M, N, device=dev).half()
    B = torch.zeros_like(A)
    G = torch.zeros(1, M, N, device=dev, dtype=torch.float16)
    R = torch.zeros(M, device=dev)
    S_ = torch.zeros(M, N, device=dev)
    k(A, B, G, R, S_)
    errors.check()
    torch.testing.assert_close(B, A)
    torch.testing.assert_close(G[0], A)
    torch.testing.assert_close(R, A.float().sum(1), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(S_, A.float())

    # ---- MoE: expert parallel (device exchange + host RCCL fallback) and tensor parallel ------
    from tilelang.models.moe import MoEConfig, MoELayer, moe_reference, init_moe_weights
    from tilelang.ops.moe import route
    cfg = MoEConfig(hidden=512, ffn=256, n_experts=8, topk=2, dtype=torch.bfloat16, block_M=256,
                    gemm_cfg=dict(block_N=256, block_K=64, num_stages=2, threads=512))
    xs = torch.randn(512, 512, device=dev).bfloat16()
    g_w, w1, w2 = (t.to(dev) for t in init_moe_weights(cfg))
    for mode, ep_mode in (("ep", "device"), ("ep", "host"), ("tp", None)):
        layer = MoELayer(cfg, mode, mesh=mesh, device="cuda")
        if ep_mode is not None:
            layer.ep_mode = ep_mode
            assert layer._device_ep() == (ep_mode == "device")
        ys = layer(xs)
        errors.check()
        ref = moe_reference(xs, g_w, w1, w2, cfg.topk, routing=route(xs, layer.gate_w, cfg.topk))
        torch.testing.assert_close(ys.float(), ref, rtol=3e-2, atol=3e-2 * float(ref.abs().max()))
        ys2 = layer(xs)  # second step: the exchange buffers flip parity
        errors.check()
        torch.testing.assert_close(ys2.float(), ys.float(), rtol=1e-2, atol=1e-2 * float(ref.abs().max()))

    shutdown_mesh()
    dist.destroy_process_group()
    print("RCCL_WORLD1_OK", flush=True)


if __name__ == "__main__":
    main()
