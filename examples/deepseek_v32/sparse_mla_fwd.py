"""DeepSeek-V3.2 sparse MLA forward (DSA) (reference: examples/deepseek_v32/sparse_mla_fwd.py).

Every query token attends only to its ``topk`` selected latent-KV rows (chosen by the lightning
indexer).  Q is [B, S, H, D + D_tail] (D = 512 latent, D_tail = 64 rope), KV is
[B, S_kv, G, D + D_tail], Indices [B, S, G, topk] (entries > the query position, e.g. the
padding value S_kv, are masked -- causal).  MI355X schedule: one block per (query token,
64-head slice, batch*group); each step gathers ``block_I`` selected KV rows into LDS
(data-dependent row gather), runs S = Q KV^T (+ the rope tail) and O += P KV on MFMA with the
64 heads as M, and the online softmax in registers -- heads play the role of query rows, so a
single query token already gives a full MFMA tile.
"""
import argparse


LOG2E = 1.44269504


from tilelang.ops.dsa import sparse_mla_fwd  # noqa: E402,F401  (kernel lives in the library)


def ref_program(q, kv, indices, dim=512, sm_scale=None):
    """fp32 reference: q [B,S,H,D+T], kv [B,SKV,G,D+T], indices [B,S,G,topk] (> query pos = masked)."""
    import torch
    B, S, H, DQ = q.shape
    _, SKV, G, _ = kv.shape
    past = SKV - S
    sm_scale = DQ**-0.5 if sm_scale is None else sm_scale
    qf, kf = q.float(), kv.float()
    out = torch.zeros(B, S, H, dim)
    hpg = H // G
    for b in range(B):
        for s in range(S):
            for g in range(G):
                idx = indices[b, s, g].long()
                ok = (idx <= s + past) & (idx >= 0)
                sel = idx[ok]
                k = kf[b, sel, g]                        # [n, DQ]
                sc = qf[b, s, g * hpg:(g + 1) * hpg] @ k.t() * sm_scale
                p = torch.softmax(sc, -1)
                out[b, s, g * hpg:(g + 1) * hpg] = p @ k[:, :dim]
    return out.to(q.dtype)


def make_indices(B, S, SKV, G, topk, device="cpu", seed=0):
    import torch
    g = torch.Generator().manual_seed(seed)
    past = SKV - S
    idx = torch.full((B, S, G, topk), SKV, dtype=torch.int32)
    for b in range(B):
        for s in range(S):
            for gg in range(G):
                n = min(topk, s + past + 1)
                idx[b, s, gg, :n] = torch.randperm(s + past + 1, generator=g)[:n].int()
    return idx.to(device)


def main(B=1, S=1024, SKV=4096, H=128, DQK=576, DV=512, topk=2048):
    import torch
    kernel = sparse_mla_fwd(B, S, SKV, H, DV, DQK - DV, topk)
    q = torch.randn(B, S, H, DQK, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(B, SKV, 1, DQK, device="cuda", dtype=torch.bfloat16)
    idx = make_indices(B, S, SKV, 1, topk, "cuda")
    o, lse = kernel(q, kv, idx)
    sub = slice(S - 4, S)
    ref = ref_program(q[:, sub].cpu(), kv.cpu(), idx[:, sub].cpu() - 0, DV)
    torch.testing.assert_close(o[:, sub].float().cpu(), ref.float(), rtol=3e-2, atol=3e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, kv, idx))
    print(f"sparse MLA fwd: {lat:.3f} ms, {B * S * (DQK + DV) * topk * 2 * H / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--S", type=int, default=1024)
    p.add_argument("--SKV", type=int, default=4096)
    p.add_argument("--topk", type=int, default=2048)
    a = p.parse_args()
    main(S=a.S, SKV=a.SKV, topk=a.topk)
