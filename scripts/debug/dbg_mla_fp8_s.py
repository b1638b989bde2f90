"""Dump the fp8-score MLA decode's first S tile (after the row scaling) and compare with torch."""
import torch

import tilelang
import tilelang.language as T

FP8 = "float8_e4m3fn"
B, H, S, D, P, BN, BH = 2, 64, 64, 512, 64, 64, 64


@tilelang.jit(out_idx=[5, 6, 7], pass_configs={"tl.enable_fast_math": True})
def dbg(fast_div=True):

    @T.prim_func
    def main(Q: T.Tensor([B, H, D], "bfloat16"), Q_pe: T.Tensor([B, H, P], "bfloat16"),
             KV: T.Tensor([B, S, 1, D], FP8), K_pe: T.Tensor([B, S, 1, P], "bfloat16"), kv_scale: T.float32,
             Sd: T.Tensor([B, H, BN], "float32"), Q8d: T.Tensor([B, H, D], FP8), QSd: T.Tensor([B, H], "float32")):
        with T.Kernel(B, 1, threads=512) as (bx, by):
            Q_f = T.alloc_fragment([BH, D], "float")
            q_amax = T.alloc_fragment([BH], "float")
            Q8_shared = T.alloc_shared([BH, D], FP8)
            qs_shared = T.alloc_shared([BH], "float")
            Q_pe_local = T.alloc_fragment([BH, P], "bfloat16")
            KV8_shared = T.alloc_shared([BN, D], FP8)
            K_pe_shared = T.alloc_shared([BN, P], "bfloat16")
            acc_s = T.alloc_fragment([BH, BN], "float")
            T.copy(Q[bx, 0:BH, :], Q_f)
            T.reduce_absmax(Q_f, q_amax, dim=1)
            for i in T.Parallel(BH):
                q_amax[i] = T.max(q_amax[i], 1e-6) / 448.0
            for i, j in T.Parallel(BH, D):
                Q8_shared[i, j] = T.clamp(Q_f[i, j] / q_amax[i], -448.0, 448.0)
            for i in T.Parallel(BH):
                qs_shared[i] = q_amax[i] * kv_scale
            T.copy(Q_pe[bx, 0:BH, :], Q_pe_local)
            T.copy(KV[bx, 0:BN, 0, :], KV8_shared)
            T.copy(K_pe[bx, 0:BN, 0, :], K_pe_shared)
            T.gemm(Q8_shared, KV8_shared, acc_s, transpose_B=True, clear_accum=True, policy=T.GemmWarpPolicy.Square)
            for i, j in T.Parallel(BH, BN):
                acc_s[i, j] *= qs_shared[i]
            T.gemm(Q_pe_local, K_pe_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.Square)
            T.copy(acc_s, Sd[bx, 0:BH, :])
            T.copy(Q8_shared, Q8d[bx, 0:BH, :])
            for i in T.Parallel(BH):
                QSd[bx, i] = qs_shared[i]

    return main


torch.manual_seed(0)
k = dbg()
q = torch.randn(B, H, D, device="cuda", dtype=torch.bfloat16)
qpe = torch.randn(B, H, P, device="cuda", dtype=torch.bfloat16)
kv = torch.randn(B, S, 1, D, device="cuda") * 3
s = float(kv.abs().amax()) / 448
kv8 = (kv / s).clamp(-448, 448).to(torch.float8_e4m3fn)
kpe = torch.randn(B, S, 1, P, device="cuda", dtype=torch.bfloat16)
out, q8k, qsk = k(q, qpe, kv8, kpe, s)
qs = q.float().abs().amax(-1, keepdim=True).clamp_min(1e-6) / 448
q8 = (q.float() / qs).clamp(-448, 448).to(torch.float8_e4m3fn)
raw = torch.einsum("bhd,bsd->bhs", q8.float(), kv8[:, :, 0].float())
ref = raw * qs * s + torch.einsum("bhd,bsd->bhs", qpe.float(), kpe[:, :, 0].float())
err = (out - ref).abs()
print("max abs err", float(err.max()), "max |S|", float(ref.abs().max()))
rows = err.amax(-1)
print("rows with err > 1e-2:", (rows > 1e-2).nonzero().tolist()[:20])
b, h = divmod(int(rows.flatten().argmax()), H)
print("worst row", b, h, "kernel", out[b, h, :6].tolist(), "ref", ref[b, h, :6].tolist())
# is the kernel row a scaled version of the reference row (wrong row scale)?
ratio = (out[b, h] - (ref[b, h] - raw[b, h] * qs[b, h] * s)) / (raw[b, h] * s)
print("implied row scale", ratio[:6].tolist(), "true qs", float(qs[b, h]), "other rows' qs", qs[b, :8, 0].tolist())

bad = (q8k.view(torch.uint8) != q8.view(torch.uint8))
print("Q8 bytes differing:", int(bad.sum()), "rows", sorted({(b_, h_) for b_, h_, _ in bad.nonzero().tolist()})[:10])
for b_, h_, d_ in bad.nonzero().tolist()[:8]:
    print(f"  ({b_},{h_},{d_}) q={q[b_, h_, d_].item():.5g} kernel {q8k[b_, h_, d_].float().item()} torch "
          f"{q8[b_, h_, d_].float().item()} x={q[b_, h_, d_].float().item() / qs[b_, h_, 0].item():.6g}")
print("qs (kernel/ref) max rel diff", float(((qsk / s) / qs[..., 0] - 1).abs().max()))
