"""DeepSeek-V3.2 lightning indexer logits in fp8 (reference: examples/deepseek_v32/fp8_lighting_indexer.py).

Logits[s, n] = sum_h relu(q[s, h] . k[n]) * w[s, h] * k_scale[n]   for ks[s] <= n < ke[s], else -inf

IndexQ is [S * H, D] (rows ordered token-major, head-minor), IndexK [S_kv, D] (one shared
index head), both OCP e4m3.  MI355X schedule: one block per ``block_Q`` query tokens covers
``block_Q * H`` (= 128 for H = 64) Q rows; each KV step computes the fp8 MFMA tile
S = K Q^T [block_N x block_Q*H] with the gfx950 scaled 16x16x128 MFMA (K-contiguous operands
on both sides), applies relu * weight * k_scale in registers, stages it through LDS and sums
the H heads of each token with a short serial reduction per (token, key) lane.
"""
import argparse



from tilelang.ops.dsa import mqa_attn_return_logits  # noqa: E402,F401  (kernel lives in the library)


def ref_program(q, kv, kv_scale, weights, ks, ke):
    """q [S, H, D] fp8, kv [SKV, D] fp8, kv_scale [SKV], weights [S, H], ks/ke [S]."""
    import torch
    score = torch.einsum("mhd,nd->hmn", q.float(), kv.float())
    logits = (score.relu() * weights.float().t().unsqueeze(-1)).sum(0) * kv_scale.float()[None, :]
    n = torch.arange(kv.shape[0], device=kv.device)
    mask = (n[None, :] >= ks[:, None]) & (n[None, :] < ke[:, None])
    return logits.masked_fill(~mask, float("-inf"))


def make_inputs(S, SKV, H, D, device="cuda", seed=0):
    import torch
    g = torch.Generator().manual_seed(seed)
    q = (torch.randn(S, H, D, generator=g) * 0.5).to(torch.float8_e4m3fn).to(device)
    kv = (torch.randn(SKV, D, generator=g) * 0.5).to(torch.float8_e4m3fn).to(device)
    kv_scale = (torch.rand(SKV, generator=g) + 0.5).to(device)
    weights = (torch.randn(S, H, generator=g) * 0.1).to(device)
    ks = torch.zeros(S, dtype=torch.int32, device=device)
    ke = torch.clamp(torch.arange(S, dtype=torch.int32, device=device) + (SKV - S) + 1, max=SKV)
    return q, kv, kv_scale, weights, ks, ke


def main(S=4096, SKV=8192, H=64, D=128):
    import torch
    q, kv, kv_scale, w, ks, ke = make_inputs(S, SKV, H, D)
    kernel = mqa_attn_return_logits(S, SKV, H, D)
    logits = kernel(q.view(S * H, D), kv, kv_scale, w, ks, ke)
    ref = ref_program(q[:64], kv, kv_scale, w[:64], ks[:64], ke[:64])
    torch.testing.assert_close(logits[:64], ref, rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q.view(S * H, D), kv, kv_scale, w, ks, ke))
    print(f"fp8 lightning indexer S={S} SKV={SKV} H={H}: {lat:.3f} ms, {2 * S * SKV * H * D / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--S", type=int, default=4096)
    p.add_argument("--SKV", type=int, default=8192)
    a = p.parse_args()
    main(a.S, a.SKV)
