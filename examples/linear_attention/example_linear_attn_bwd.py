"""Chunked causal linear attention backward (reference: examples/linear_attention/example_linear_attn_bwd.py).

Forward (example_linear_attn_fwd.py): o_t = scale * sum_{s<=t} (q_t . k_s) v_s.  With the
running state H_c = sum_{c'<c} K_c'^T V_c' and the reverse state dH_c = sum_{c'>c} Q_c'^T dO_c':

    dQ_c = scale * ( tril(dO_c V_c^T) K_c + dO_c H_c^T )
    dK_c = scale * ( triu(V_c dO_c^T) Q_c + V_c dH_c^T )
    dV_c = scale * ( triu(K_c Q_c^T) dO_c + K_c dH_c )

MI355X schedule: one block per (batch, head) owns the whole DK x DV state in fp32 registers
(128 x 128 over 256 threads = 64 VGPRs per lane), walks the chunks forward for dQ and backward
for dK / dV, and writes every gradient once — no fp32 atomics and no zero-initialised gradient
buffers (the reference splits DK/DV across blocks and atomically accumulates fp32 gradients).
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[4, 5, 6])
def linear_attn_bwd(B, S, H, DK, DV, chunk_size=64, threads=256, dtype="float16", scale=None):
    if scale is None:
        scale = DK**-0.5
    accum_dtype = "float"
    C = chunk_size
    assert S % C == 0
    NT = S // C

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, DK], dtype), K: T.Tensor([B, S, H, DK], dtype), V: T.Tensor([B, S, H, DV], dtype),
             dO: T.Tensor([B, S, H, DV], dtype), dQ: T.Tensor([B, S, H, DK], dtype),
             dK: T.Tensor([B, S, H, DK], dtype), dV: T.Tensor([B, S, H, DV], dtype)):
        with T.Kernel(B * H, threads=threads) as (i_bh):
            i_b = i_bh // H
            i_h = i_bh % H
            q = T.alloc_shared([C, DK], dtype)
            k = T.alloc_shared([C, DK], dtype)
            v = T.alloc_shared([C, DV], dtype)
            do = T.alloc_shared([C, DV], dtype)
            st_shared = T.alloc_shared([DK, DV], dtype)
            st = T.alloc_fragment([DK, DV], accum_dtype)
            s = T.alloc_fragment([C, C], accum_dtype)
            s_cast = T.alloc_fragment([C, C], dtype)
            gq = T.alloc_fragment([C, DK], accum_dtype)
            gv = T.alloc_fragment([C, DV], accum_dtype)

            # dQ: forward over chunks, st = H_c
            T.clear(st)
            for c in T.Pipelined(NT, num_stages=2):
                T.copy(K[i_b, c * C:(c + 1) * C, i_h, :], k)
                T.copy(V[i_b, c * C:(c + 1) * C, i_h, :], v)
                T.copy(dO[i_b, c * C:(c + 1) * C, i_h, :], do)
                T.clear(s)
                T.gemm(do, v, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(C, C):
                    s_cast[i, j] = T.if_then_else(i >= j, s[i, j], 0)
                T.copy(st, st_shared)
                T.clear(gq)
                T.gemm(s_cast, k, gq, policy=T.GemmWarpPolicy.FullRow)
                T.gemm(do, st_shared, gq, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(C, DK):
                    gq[i, j] *= scale
                T.copy(gq, dQ[i_b, c * C:(c + 1) * C, i_h, :])
                T.gemm(k, v, st, transpose_A=True)

            # dK, dV: backward over chunks, st = dH_c (Q pre-scaled)
            T.clear(st)
            for r in T.Pipelined(NT, num_stages=2):
                c = NT - 1 - r
                T.copy(Q[i_b, c * C:(c + 1) * C, i_h, :], q)
                T.copy(K[i_b, c * C:(c + 1) * C, i_h, :], k)
                T.copy(V[i_b, c * C:(c + 1) * C, i_h, :], v)
                T.copy(dO[i_b, c * C:(c + 1) * C, i_h, :], do)
                for i, j in T.Parallel(DK, DV):
                    st_shared[i, j] = st[i, j] * scale
                # dK = triu(V dO^T) Q + V dH^T
                T.clear(s)
                T.gemm(v, do, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(C, C):
                    s_cast[i, j] = T.if_then_else(i <= j, s[i, j] * scale, 0)
                T.clear(gq)
                T.gemm(s_cast, q, gq, policy=T.GemmWarpPolicy.FullRow)
                T.gemm(v, st_shared, gq, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(gq, dK[i_b, c * C:(c + 1) * C, i_h, :])
                # dV = triu(K Q^T) dO + K dH
                T.clear(s)
                T.gemm(k, q, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(C, C):
                    s_cast[i, j] = T.if_then_else(i <= j, s[i, j] * scale, 0)
                T.clear(gv)
                T.gemm(s_cast, do, gv, policy=T.GemmWarpPolicy.FullRow)
                T.gemm(k, st_shared, gv, policy=T.GemmWarpPolicy.FullRow)
                T.copy(gv, dV[i_b, c * C:(c + 1) * C, i_h, :])
                # dH += scale Q^T dO
                T.gemm(q, do, st, transpose_A=True)

    return main


class LinearAttention:
    """``torch.autograd.Function`` pairing the forward and backward kernels."""

    @staticmethod
    def apply(q, k, v, scale=None):
        import torch
        from example_linear_attn_fwd import linear_attn_fwd

        class _Fn(torch.autograd.Function):

            @staticmethod
            def forward(ctx, q, k, v):
                B, S, H, D = q.shape
                fwd = linear_attn_fwd(B, S, H, D, v.shape[-1], dtype=_dt(q), scale=scale)
                o, _ = fwd(q, k, v)
                ctx.save_for_backward(q, k, v)
                return o

            @staticmethod
            def backward(ctx, do):
                q, k, v = ctx.saved_tensors
                B, S, H, D = q.shape
                bwd = linear_attn_bwd(B, S, H, D, v.shape[-1], dtype=_dt(q), scale=scale)
                return bwd(q, k, v, do.contiguous().to(q.dtype))

        return _Fn.apply(q, k, v)


def _dt(t):
    return str(t.dtype).replace("torch.", "")


def ref_program(q, k, v, scale=None):
    """fp32 causal linear attention (the definition)."""
    import torch
    q, k, v = q.float(), k.float(), v.float()
    if scale is None:
        scale = q.shape[-1]**-0.5
    S = q.shape[1]
    qs, ks, vs = (x.permute(0, 2, 1, 3) for x in (q, k, v))
    att = (qs @ ks.transpose(-1, -2) * scale).masked_fill(
        torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), 1), 0)
    return (att @ vs).permute(0, 2, 1, 3)


def check(B, S, H, D, device):
    import torch
    torch.manual_seed(0)
    mk = lambda: torch.nn.functional.normalize(torch.randn(B, S, H, D, device=device), dim=-1)  # noqa: E731
    q, k = mk().half(), mk().half()
    v = torch.randn(B, S, H, D, device=device).half()
    do = torch.randn(B, S, H, D, device=device).half()
    kern = linear_attn_bwd(B, S, H, D, D)
    dq, dk, dv = kern(q, k, v, do)
    qr, kr, vr = (x.float().requires_grad_(True) for x in (q, k, v))
    ref_program(qr, kr, vr).backward(do.float())
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        torch.testing.assert_close(got.float(), want, rtol=2e-2, atol=2e-2, msg=lambda m: f"{name}: {m}")
    return kern, (q, k, v, do)


def main(B=8, S=1024, H=32, D=128):
    kern, args = check(B, S, H, D, "cuda")
    print("dq/dk/dv match the fp32 autograd reference")
    lat = kern.get_profiler().do_bench(lambda: kern(*args))
    flops = B * H * (S // 64) * 2 * (3 * 64 * 64 * D + 5 * 64 * D * D + 64 * 64 * D)
    print(f"linear attention bwd b{B} s{S} h{H} d{D}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--B", type=int, default=8)
    p.add_argument("--S", type=int, default=1024)
    p.add_argument("--H", type=int, default=32)
    p.add_argument("--D", type=int, default=128)
    a = p.parse_args()
    main(a.B, a.S, a.H, a.D)
