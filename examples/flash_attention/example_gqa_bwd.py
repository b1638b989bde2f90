"""Grouped-query FlashAttention forward + backward with different Q/K and V head dims
(reference: examples/flash_attention/example_gqa_bwd.py, defaults d_qk=192, d_v=128 as in
DeepSeek-style heads).

Kernels are the ones of ``example_mha_bwd.py`` with ``dim_v``: the forward writes O [.., d_v] and
the base-2 LSE; the backward is the dK/dV kernel (one workgroup per KV head and key tile walks
the Q/dO tiles of ALL its query heads in one pipelined loop, so the group's dK/dV accumulate in
registers: no atomics) plus the atomic-free dQ kernel.
"""
import argparse

from example_mha_bwd import attention, ref_program


def main(BATCH=1, H=32, N_CTX=256, D_HEAD_QK=192, D_HEAD_V=128, groups=16, causal=False):
    import torch
    from tilelang.profiler import do_bench
    HKV = H // groups
    Q = torch.randn(BATCH, N_CTX, H, D_HEAD_QK, dtype=torch.half, device="cuda").requires_grad_()
    K = torch.randn(BATCH, N_CTX, HKV, D_HEAD_QK, dtype=torch.half, device="cuda").requires_grad_()
    V = torch.randn(BATCH, N_CTX, HKV, D_HEAD_V, dtype=torch.half, device="cuda").requires_grad_()
    dO = torch.randn(BATCH, N_CTX, H, D_HEAD_V, dtype=torch.half, device="cuda")
    O = attention(Q, K, V, causal)
    O.backward(dO)
    grads = [t.grad.clone() for t in (Q, K, V)]
    for t in (Q, K, V):
        t.grad = None
    O_ref = ref_program(Q, K, V, causal)
    O_ref.backward(dO)
    torch.testing.assert_close(O, O_ref, rtol=2e-2, atol=2e-2)
    for g, t in zip(grads, (Q, K, V)):
        torch.testing.assert_close(g, t.grad, rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    # fwd: QK^T (d_qk) + PV (d_v); bwd: QK^T, dP = dO V^T, dV, dK, dQ + the dQ kernel's QK^T / dP recompute
    per_pair = 2.0 * BATCH * H * N_CTX * N_CTX * (0.5 if causal else 1.0)
    fwd_flops = per_pair * (D_HEAD_QK + D_HEAD_V)
    bwd_flops = per_pair * (3 * D_HEAD_QK + 2 * D_HEAD_V)
    O = attention(Q, K, V, causal)
    lat_f = do_bench(lambda: attention(Q, K, V, causal))
    lat_b = do_bench(lambda: O.backward(dO, retain_graph=True))
    print(f"gqa fwd: {lat_f:.3f} ms, {fwd_flops / lat_f * 1e-9:.1f} TFLOPS")
    print(f"gqa bwd: {lat_b:.3f} ms, {bwd_flops / lat_b * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--h", type=int, default=32)
    p.add_argument("--n_ctx", type=int, default=1024)
    p.add_argument("--d_head_qk", type=int, default=192)
    p.add_argument("--d_head_v", type=int, default=128)
    p.add_argument("--groups", type=int, default=16)
    p.add_argument("--causal", action="store_true")
    a = p.parse_args()
    main(a.batch, a.h, a.n_ctx, a.d_head_qk, a.d_head_v, a.groups, a.causal)
