"""GQA + sink causal fwd (the reference's headline attention kernel, b1 h64 kvh8 s4096 d128 bf16):
split-loop schedule vs the staged FA route (impl="staged"), one process, cold.
    python scripts/sink_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "attention_sink")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_gqa_sink_fwd_bhsd as m  # noqa: E402

b, h, g, s, d = 1, 64, 8, 4096, 128
torch.manual_seed(0)
q = torch.randn(b, h, s, d, device="cuda", dtype=torch.bfloat16)
k = torch.randn(b, h // g, s, d, device="cuda", dtype=torch.bfloat16)
v = torch.randn_like(k)
sk = torch.randn(h, device="cuda", dtype=torch.bfloat16)
flops = 4.0 * b * h * s * s * d * 0.5
for win in (None, 128):
    ref = m.ref_program(q, k, v, sk, win).float()
    res = {}
    for impl in ("split", "staged", "staged+fold"):
        kern = m.flashattn_sink(b, h, s, s, d, g, win, impl=impl.split("+")[0], fold=impl.endswith("fold"))
        err = (kern(q, k, v, sk).float() - ref).abs().max().item()
        best = 0.0
        for _ in range(3):
            ms = do_bench(lambda: kern(q, k, v, sk), warmup=25, rep=100)
            best = max(best, flops / ms * 1e-9)
        res[impl] = (best, err)
    print(f"sink causal window={win}: " + ", ".join(f"{i} {t:.0f} TF (err {e:.3f})" for i, (t, e) in res.items()),
          flush=True)
