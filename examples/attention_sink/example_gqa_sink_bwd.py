"""GQA attention with a learned per-head sink: forward + backward wired into autograd
(reference: examples/attention_sink/example_{gqa,mha}_sink_bwd_bhsd.py), causal, bshd layout.

out_h = softmax([s_h1 .. s_hn, sink_h]) restricted to the keys, i.e. the sink only enlarges the
softmax denominator.  So the sink forward is the plain FlashAttention forward plus a per-row fixup
    lse' = log2(2^lse + 2^(sink*log2 e)),   o' = o * 2^(lse - lse')
and the backward is the plain FlashAttention backward run with lse' (P' = exp2(s*scale - lse'),
Delta' = rowsum(o' dO')) plus the sink gradient
    dsink_h = -sum_{b, rows} 2^(sink_h log2 e - lse'_row) * Delta'_row.
All kernels are tilelang: the FA fwd/bwd of example_mha_bwd.py (GQA dK/dV without atomics,
atomic-free dQ) plus two small kernels here (row fixup, per-head dsink reduction).
"""
import argparse
import os
import sys

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flash_attention"))
import example_mha_bwd as fa  # noqa: E402

LOG2E = 1.44269504


@tilelang.jit(out_idx=[3, 4], pass_configs=FAST_MATH)
def sink_fixup(B, S, H, D, block=64, dtype="bfloat16"):
    """(o, lse, sinks) -> (o', lse') for the sink-enlarged denominator."""

    @T.prim_func
    def main(O: T.Tensor([B, S, H, D], dtype), Lse: T.Tensor([B, H, S], "float32"), Sinks: T.Tensor([H], "float32"),
             O2: T.Tensor([B, S, H, D], dtype), Lse2: T.Tensor([B, H, S], "float32")):
        with T.Kernel(T.ceildiv(S, block), H, B, threads=256) as (bx, by, bz):
            o = T.alloc_fragment([block, D], "float32")
            l2 = T.alloc_fragment([block], "float32")
            T.copy(O[bz, bx * block:(bx + 1) * block, by, :], o)
            for i in T.Parallel(block):
                lse = Lse[bz, by, bx * block + i]
                m = T.max(lse, Sinks[by] * LOG2E)
                l2[i] = m + T.log2(T.exp2(lse - m) + T.exp2(Sinks[by] * LOG2E - m))
            for i, j in T.Parallel(block, D):
                o[i, j] = o[i, j] * T.exp2(Lse[bz, by, bx * block + i] - l2[i])
            T.copy(o, O2[bz, bx * block:(bx + 1) * block, by, :])
            T.copy(l2, Lse2[bz, by, bx * block:(bx + 1) * block])

    return main


@tilelang.jit(out_idx=[3], pass_configs=FAST_MATH)
def sink_grad(B, S, H, threads=256):
    """dsink[h] = -sum_{b, s} 2^(sink_h log2 e - lse'[b, h, s]) * Delta[b, h, s]."""
    n = B * S

    @T.prim_func
    def main(Lse2: T.Tensor([B, H, S], "float32"), Delta: T.Tensor([B, H, S], "float32"),
             Sinks: T.Tensor([H], "float32"), dSinks: T.Tensor([H], "float32")):
        with T.Kernel(H, threads=threads) as h:
            part = T.alloc_fragment([threads], "float32")
            tot = T.alloc_fragment([1], "float32")
            T.clear(part)
            for it in T.serial(T.ceildiv(n, threads)):
                for t in T.Parallel(threads):
                    k = it * threads + t
                    if k < n:
                        part[t] += T.exp2(Sinks[h] * LOG2E - Lse2[k // S, h, k % S]) * Delta[k // S, h, k % S]
            T.reduce_sum(part, tot, dim=0)
            for z in T.Parallel(1):
                dSinks[h] = -tot[z]

    return main


class _SinkAttn:
    fn = None

    @classmethod
    def get(cls):
        if cls.fn is None:
            import torch

            class SinkAttn(torch.autograd.Function):

                @staticmethod
                def forward(ctx, q, k, v, sinks):
                    B, S, H, D = q.shape
                    G = H // k.shape[2]
                    dt = "bfloat16" if q.dtype == torch.bfloat16 else "float16"
                    o, lse = fa.flashattn_fwd(B, H, S, D, True, dtype=dt, groups=G)(q, k, v)
                    o2, lse2 = sink_fixup(B, S, H, D, dtype=dt)(o, lse, sinks.float().contiguous())
                    ctx.save_for_backward(q, k, v, o2, lse2, sinks)
                    return o2

                @staticmethod
                def backward(ctx, do):
                    q, k, v, o, lse, sinks = ctx.saved_tensors
                    B, S, H, D = q.shape
                    G = H // k.shape[2]
                    dt = "bfloat16" if q.dtype == torch.bfloat16 else "float16"
                    do = do.contiguous()
                    # Delta' = rowsum(o' dO) inside the dQ kernel (fuse_delta), which runs first
                    delta = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
                    dq = fa.flashattn_bwd_dq(B, H, S, D, True, dtype=dt, groups=G, fuse_delta=True)(q, k, v, do, lse,
                                                                                                   delta, o)
                    dk, dv = torch.empty_like(k), torch.empty_like(v)
                    fa.flashattn_bwd(B, H, S, D, True, dtype=dt, dq_mode="none", groups=G)(q, k, v, do, lse, delta,
                                                                                            dk, dv)
                    ds = sink_grad(B, S, H)(lse, delta, sinks.float().contiguous())
                    return dq, dk, dv, ds.to(sinks.dtype)

            cls.fn = SinkAttn
        return cls.fn


def attention_sink(q, k, v, sinks):
    """Causal GQA attention with per-head sinks; q [B,S,H,D], k/v [B,S,H/G,D], sinks [H]."""
    return _SinkAttn.get().apply(q, k, v, sinks)


def ref_program(q, k, v, sinks):
    import torch
    B, S, H, D = q.shape
    G = H // k.shape[2]
    kf, vf = k.float().repeat_interleave(G, 2), v.float().repeat_interleave(G, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), kf) * D**-0.5
    s = s.masked_fill(~torch.ones(S, S, dtype=torch.bool, device=q.device).tril(), float("-inf"))
    s = torch.cat([s, sinks.float().view(1, H, 1, 1).expand(B, H, S, 1)], -1)
    p = torch.softmax(s, -1)[..., :-1]
    return torch.einsum("bhqk,bkhd->bqhd", p, vf).to(q.dtype)


def main(B=1, S=4096, H=64, G=8, D=128):
    import torch
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    k = torch.randn(B, S, H // G, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    v = torch.randn(B, S, H // G, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    sinks = torch.randn(H, device="cuda", dtype=torch.float32).requires_grad_()
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    o = attention_sink(q, k, v, sinks)
    o.backward(do, retain_graph=True)
    grads = [t.grad.clone() for t in (q, k, v, sinks)]
    for t in (q, k, v, sinks):
        t.grad = None
    Ss = 512  # reference on a prefix (causal: the first rows only depend on the first keys)
    qs, ks, vs = (t[:, :Ss].detach().clone().requires_grad_() for t in (q, k, v))
    ss = sinks.detach().clone().requires_grad_()
    o_ref = ref_program(qs, ks, vs, ss)
    torch.testing.assert_close(o[:, :Ss].float(), o_ref.float(), rtol=3e-2, atol=3e-2)
    print("forward matches")
    lat_f = tilelang.profiler.do_bench(lambda: attention_sink(q, k, v, sinks))
    lat = tilelang.profiler.do_bench(lambda: o.backward(do, retain_graph=True))
    flops = 2 * 2.0 * B * H * S * S * D * 0.5
    print(f"sink attention fwd {lat_f:.3f} ms ({flops / lat_f * 1e-9:.1f} TF), bwd {lat:.3f} ms "
          f"({2.5 * flops / lat * 1e-9:.1f} TF)")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--seq", type=int, default=4096)
    a = p.parse_args()
    main(S=a.seq)
