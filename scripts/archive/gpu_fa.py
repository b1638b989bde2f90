import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "examples", "flash_attention"))
import torch
from example_mha_fwd import flashattn, ref_program
from tilelang.profiler import do_bench
torch.manual_seed(0)
for (b, h, s, d, causal, cfg) in [(1, 2, 256, 128, False, {}), (1, 2, 512, 64, True, {}), (2, 4, 512, 128, True, {})]:
    k = flashattn(b, h, s, d, causal, 1, **cfg)
    q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    o = k(q, kk, v)
    ref = ref_program(q, kk, v, causal)
    print(f"fa b{b} h{h} s{s} d{d} causal={causal}: max err {(o.float()-ref.float()).abs().max().item():.4f}", flush=True)
b, h, s, d = 1, 64, 4096, 128
q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
kk = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
v = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
flops = 4.0 * b * h * s * s * d
import torch.nn.functional as F
qt, kt, vt = q.transpose(1, 2), kk.transpose(1, 2), v.transpose(1, 2)
try:
    t = do_bench(lambda: F.scaled_dot_product_attention(qt, kt, vt))
    print(f"torch sdpa b{b} h{h} s{s} d{d}: {t:.3f} ms {flops/t*1e-9:.1f} TF", flush=True)
except Exception as e:
    print("sdpa failed", e)
for cfg in [dict(block_M=128, block_N=64, threads=256, num_stages=2), dict(block_M=128, block_N=32, threads=256, num_stages=2),
            dict(block_M=64, block_N=64, threads=256, num_stages=2), dict(block_M=256, block_N=64, threads=512, num_stages=2),
            dict(block_M=128, block_N=64, threads=256, num_stages=1), dict(block_M=128, block_N=128, threads=256, num_stages=2)]:
    try:
        k = flashattn(b, h, s, d, False, 1, **cfg)
        o = k(q, kk, v)
        t = do_bench(lambda: k(q, kk, v))
        print(f"cfg {cfg}: {t:.3f} ms {flops/t*1e-9:.1f} TF", flush=True)
    except Exception as e:
        print(f"cfg {cfg}: FAILED {type(e).__name__} {str(e)[:200]}", flush=True)
