"""Chunked causal linear attention forward (reference: examples/linear_attention/example_linear_attn_fwd.py).

O_t = sum_{s<=t} (q_t . k_s) v_s, computed chunk by chunk with a running state
H = sum K_c^T V_c.  MI355X schedule: one block per (value tile, batch*head) walks the chunks
in order, keeping the full-DK state tile H [DK, BV] in fp32 registers (DK=128, BV=64 is 32
VGPRs per lane at 256 threads), so no cross-block reduction or atomics are needed:

    S   = (Q_c * scale) K_c^T          (ss MFMA, FullRow -> whole rows per wave)
    O_c = tril(S) V_c                  (register-A MFMA straight from the accumulator)
        + scale * Q_c H                (H staged to LDS as fp16 once per chunk)
    H  += K_c^T V_c                    (transposed-A MFMA: ds_read_b64_tr_b16 on K_c)
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[3, 4])
def linear_attn_fwd(B, S, H, DK, DV, chunk_size=64, BV=None, threads=256, dtype="float16", scale=None):
    """``BV`` (default: 64, or 32 when the 64-wide value tiles give fewer than 256 workgroups): the
    value columns of the state each workgroup carries through the sequential chunk walk; small grids
    trade MFMA width for workgroups (b1 h16 s4096 0.142 -> 0.117 ms; b8 h32 keeps 64: 32 would be
    0.323 -> 0.426 ms; profiles/r6/linear_attn_bv_sweep.log)."""
    if BV is None:
        BV = 32 if (DV // 64) * B * H < 256 and DV % 32 == 0 else 64
    if scale is None:
        scale = DK**-0.5
    accum_dtype = "float"
    assert S % chunk_size == 0 and DV % BV == 0
    NT = S // chunk_size

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, DK], dtype), K: T.Tensor([B, S, H, DK], dtype), V: T.Tensor([B, S, H, DV], dtype),
             O: T.Tensor([B, S, H, DV], dtype), final_state: T.Tensor([B, H, DK, DV], accum_dtype)):
        with T.Kernel(DV // BV, B * H, threads=threads) as (i_v, i_bh):
            i_b = i_bh // H
            i_h = i_bh % H
            q = T.alloc_shared([chunk_size, DK], dtype)
            k = T.alloc_shared([chunk_size, DK], dtype)
            v = T.alloc_shared([chunk_size, BV], dtype)
            h_shared = T.alloc_shared([DK, BV], dtype)
            h = T.alloc_fragment([DK, BV], accum_dtype)
            s = T.alloc_fragment([chunk_size, chunk_size], accum_dtype)
            s_cast = T.alloc_fragment([chunk_size, chunk_size], dtype)
            o = T.alloc_fragment([chunk_size, BV], accum_dtype)
            o_inter = T.alloc_fragment([chunk_size, BV], accum_dtype)
            o_cast = T.alloc_fragment([chunk_size, BV], dtype)
            T.clear(h)
            for c in T.Pipelined(NT, num_stages=2):
                T.copy(Q[i_b, c * chunk_size:(c + 1) * chunk_size, i_h, :], q)
                T.copy(K[i_b, c * chunk_size:(c + 1) * chunk_size, i_h, :], k)
                T.copy(V[i_b, c * chunk_size:(c + 1) * chunk_size, i_h, i_v * BV:(i_v + 1) * BV], v)
                T.clear(s)
                T.gemm(q, k, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(chunk_size, chunk_size):
                    s_cast[i, j] = T.if_then_else(i >= j, s[i, j] * scale, 0)
                T.clear(o)
                T.gemm(s_cast, v, o, policy=T.GemmWarpPolicy.FullRow)
                T.copy(h, h_shared)
                T.clear(o_inter)
                T.gemm(q, h_shared, o_inter, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(chunk_size, BV):
                    o_cast[i, j] = o[i, j] + o_inter[i, j] * scale
                T.copy(o_cast, O[i_b, c * chunk_size:(c + 1) * chunk_size, i_h, i_v * BV:(i_v + 1) * BV])
                T.gemm(k, v, h, transpose_A=True)
            T.copy(h, final_state[i_b, i_h, :, i_v * BV:(i_v + 1) * BV])

    return main


def ref_program(q, k, v, scale=None, chunk_size=64):
    import torch
    q, k, v = q.float(), k.float(), v.float()
    if scale is None:
        scale = q.shape[-1]**-0.5
    S = q.shape[1]
    qs = (q * scale).permute(0, 2, 1, 3)  # b h s d
    ks, vs = k.permute(0, 2, 1, 3), v.permute(0, 2, 1, 3)
    att = (qs @ ks.transpose(-1, -2)).masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), 1), 0)
    o = (att @ vs).permute(0, 2, 1, 3)
    h = ks.transpose(-1, -2) @ vs
    return o, h


def main(B=1, S=4096, H=16, D=128):
    import torch
    kernel = linear_attn_fwd(B, S, H, D, D)
    q = torch.nn.functional.normalize(torch.randn(B, S, H, D, device="cuda"), dim=-1).half()
    k = torch.nn.functional.normalize(torch.randn(B, S, H, D, device="cuda"), dim=-1).half()
    v = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16)
    o, h = kernel(q, k, v)
    ro, rh = ref_program(q, k, v)
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(h, rh, rtol=1e-2, atol=1e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v))
    flops = B * H * (S // 64) * (2 * 64 * 64 * D * 2 + 2 * 64 * D * D * 2)
    print(f"linear attention fwd b{B} s{S} h{H} d{D}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--B", type=int, default=1)
    p.add_argument("--S", type=int, default=4096)
    p.add_argument("--H", type=int, default=16)
    p.add_argument("--D", type=int, default=128)
    a = p.parse_args()
    main(a.B, a.S, a.H, a.D)
