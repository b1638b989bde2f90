"""DeepSeek-style MoE FFN: shared experts + routed SwiGLU experts
(reference: examples/fusedmoe/example_fusedmoe_tilelang.py, example_fusedmoe_torch.py).

y = SharedExpert(x) + sum_k w_k * Expert_{e_k}(x)      (top-k softmax router)

MI355X schedule (tilelang.ops.moe):
* routed tokens are packed by expert into ``block_M``-aligned row tiles; one grouped GEMM
  kernel does every expert's gate|up projection (the tile's expert id selects the weight
  slab), a fused SiLU*mul kernel forms the activation, a second grouped GEMM the down
  projection -- shapes are static (worst-case padding) so the launches are graph-capturable;
* the shared expert is a dense SwiGLU on all tokens, issued on a second HIP stream so it
  overlaps the routed experts' GEMMs (the two are independent until the final add).
"""
import argparse

import torch

from tilelang.models.moe import route
from tilelang.ops.moe import expert_ffn


def init_weights(d_hidden, d_expert, n_routed, n_shared, dtype=torch.float16, device="cuda", seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)

    def rnd(*shape, scale):
        return (torch.randn(*shape, generator=g) * scale).to(dtype).to(device)

    H, F = d_hidden, d_expert
    Fs = d_expert * n_shared
    return {
        "router": rnd(n_routed, H, scale=H**-0.5),
        "w1": rnd(n_routed, 2 * F, H, scale=H**-0.5),  # [gate | up] per expert
        "w2": rnd(n_routed, H, F, scale=F**-0.5),
        "shared_w1": rnd(1, 2 * Fs, H, scale=H**-0.5),
        "shared_w2": rnd(1, H, Fs, scale=Fs**-0.5),
    }


class FusedMoE:

    def __init__(self, weights, top_k, block_M=128):
        self.w = weights
        self.top_k = top_k
        self.block_M = block_M
        self.side = torch.cuda.Stream() if weights["w1"].is_cuda else None

    def shared(self, x):
        zeros = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        return expert_ffn(x, zeros, self.w["shared_w1"], self.w["shared_w2"], self.block_M)

    def routed(self, x):
        T_ = x.shape[0]
        ids, wts = route(x, self.w["router"], self.top_k)
        tok = torch.arange(T_, device=x.device).repeat_interleave(self.top_k)
        y = expert_ffn(x[tok], ids.reshape(-1), self.w["w1"], self.w["w2"], self.block_M)
        out = torch.zeros(T_, x.shape[1], dtype=torch.float32, device=x.device)
        out.index_add_(0, tok, y.float() * wts.reshape(-1, 1))
        return out

    def __call__(self, x):
        shp = x.shape
        x = x.reshape(-1, shp[-1])
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                ys = self.shared(x)
            yr = self.routed(x)
            torch.cuda.current_stream().wait_stream(self.side)
        else:
            ys, yr = self.shared(x), self.routed(x)
        return (yr + ys.float()).to(x.dtype).reshape(shp)


def ref_program(x, w, top_k):
    from tilelang.models.moe import moe_reference
    xf = x.reshape(-1, x.shape[-1])
    Fs = w["shared_w2"].shape[-1]
    h = xf.float() @ w["shared_w1"][0].float().t()
    ys = (torch.nn.functional.silu(h[:, :Fs]) * h[:, Fs:]) @ w["shared_w2"][0].float().t()
    yr = moe_reference(xf, w["router"], w["w1"], w["w2"], top_k)
    return (ys + yr).to(x.dtype).reshape(x.shape)


def main(d_hidden=7168, d_expert=2048, n_routed_experts=8, n_shared_experts=1, n_experts_per_token=4,
         batch_size=1, seq_len=8192):
    w = init_weights(d_hidden, d_expert, n_routed_experts, n_shared_experts)
    x = torch.randn(batch_size, seq_len, d_hidden, device="cuda", dtype=torch.float16)
    moe = FusedMoE(w, n_experts_per_token)
    out = moe(x)
    torch.testing.assert_close(out.float(), ref_program(x, w, n_experts_per_token).float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    lat = do_bench(lambda: moe(x))
    T_ = batch_size * seq_len
    flops = 6 * T_ * d_hidden * d_expert * (n_experts_per_token + n_shared_experts)
    print(f"fused MoE T={T_} H={d_hidden} F={d_expert} E={n_routed_experts} k={n_experts_per_token}: "
          f"{lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--d_hidden", type=int, default=7168)
    p.add_argument("--d_expert", type=int, default=2048)
    p.add_argument("--n_routed_experts", type=int, default=8)
    p.add_argument("--n_experts_per_token", type=int, default=4)
    p.add_argument("--seq_len", type=int, default=8192)
    a = p.parse_args()
    main(a.d_hidden, a.d_expert, a.n_routed_experts, 1, a.n_experts_per_token, 1, a.seq_len)
