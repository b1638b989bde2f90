"""fp8 lightning indexer (S4096 SKV8192 H64 D128) tile sweep, one process, checked on 64 tokens.

    python scripts/indexer_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "deepseek_v32")]
import torch  # noqa: E402

from fp8_lighting_indexer import make_inputs, ref_program  # noqa: E402
from tilelang.ops.dsa import mqa_attn_return_logits  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

S, SKV, H, D = 4096, 8192, 64, 128
q, kv, sc, w, ks, ke = make_inputs(S, SKV, H, D)
ref = ref_program(q[:64], kv, sc, w[:64], ks[:64], ke[:64])
fin = torch.isfinite(ref)
CFGS = [dict(), dict(block_Q=4), dict(block_Q=1), dict(block_N=128), dict(block_Q=4, block_N=128),
        dict(threads=512, block_N=128), dict()]
if len(sys.argv) > 1:
    CFGS = eval(sys.argv[1])
for cfg in CFGS:
    try:
        k = mqa_attn_return_logits(S, SKV, H, D, **cfg)
        out = k(q.view(S * H, D), kv, sc, w, ks, ke)
        ok = torch.equal(torch.isfinite(out[:64]), fin) and torch.allclose(out[:64][fin], ref[fin], rtol=2e-2, atol=2e-2)
        t = do_bench(lambda: k(q.view(S * H, D), kv, sc, w, ks, ke), warmup=5, rep=30)
        print(f"{cfg}: {t:.4f} ms {2 * S * SKV * H * D / t * 1e-9:.0f} TF ok={ok}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{cfg}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
