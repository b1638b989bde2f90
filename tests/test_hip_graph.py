"""hipGraph capture / replay of tilelang launches (tilelang/runtime/graph.py): the launcher runs on
PyTorch's current stream with no host sync, so a GEMM, a FlashAttention forward and a whole MoE
layer (router, align, expert GEMMs, combine) replay from a graph and match eager execution."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("gemm", "flash_attention"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import tilelang  # noqa: E402
from tilelang.runtime.graph import capture  # noqa: E402


def test_capture_rejects_wrong_inputs_cpu():
    """Input checks of GraphStep without a GPU (a fake graph)."""
    from tilelang.runtime.graph import GraphStep

    class G:
        n = 0

        def replay(self):
            G.n += 1

    x = torch.zeros(4)
    step = GraphStep(G(), (x, ), x, None)
    step(torch.ones(4))
    assert G.n == 1 and x.sum() == 4
    with pytest.raises(ValueError):
        step(torch.ones(5))
    with pytest.raises(ValueError):
        step(torch.ones(4), torch.ones(4))


@pytest.mark.gpu
def test_graph_gemm_and_attention():
    from example_gemm import matmul
    from example_mha_fwd_pipelined import flashattn_pipelined as fa
    M = N = K = 512
    gk = matmul(M, N, K, 256, 256, 64, 512, 2, "float16", trans_B=True, staged_epilogue=True)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(N, K, device="cuda", dtype=torch.float16)
    B_, H, S, D = 1, 4, 512, 128
    ak = fa(B_, H, S, D, False, 1, 256, 64, 512, 2, "bfloat16", True, True, sum_mfma=True, fold_max=True)
    q, k, v = (torch.randn(B_, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))

    def step(a, b, q, k, v):
        return gk(a, b), ak(q, k, v)

    g = capture(step, a, b, q, k, v)
    for _ in range(2):  # new data through the captured launches
        a2, b2 = torch.randn_like(a), torch.randn_like(b)
        q2, k2, v2 = torch.randn_like(q), torch.randn_like(k), torch.randn_like(v)
        c, o = g(a2, b2, q2, k2, v2)
        torch.cuda.synchronize()
        c_ref, o_ref = step(a2, b2, q2, k2, v2)
        torch.testing.assert_close(c, c_ref, rtol=0, atol=0)
        torch.testing.assert_close(o, o_ref, rtol=0, atol=0)


@pytest.mark.gpu
def test_graph_moe_layer():
    from tilelang.models.moe import MoEConfig, MoELayer
    cfg = MoEConfig(hidden=1024, ffn=512, n_experts=8, topk=2, dtype=torch.bfloat16, block_M=256,
                    gemm_cfg=dict(block_N=256, block_K=64, num_stages=2, threads=512, ext_M=32))
    layer = MoELayer(cfg, "local", device="cuda")
    x = torch.randn(512, 1024, device="cuda").to(torch.bfloat16)
    g = capture(layer, x)
    for _ in range(2):
        x2 = torch.randn_like(x.float()).to(x.dtype)
        y = g(x2).clone()
        torch.cuda.synchronize()
        torch.testing.assert_close(y, layer(x2), rtol=0, atol=0)
