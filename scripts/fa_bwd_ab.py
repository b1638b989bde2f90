"""A/B of pass configs on the FA backward kernels (examples/flash_attention/example_mha_bwd.py) at
the tuned tiles (fp16 b8 h32 s1024 d64): dK/dV (dq_mode="none") and the atomic-free dQ kernel,
each checked against fp32 autograd gradients and timed cold, one process.

    python scripts/fa_bwd_ab.py '[{}, {"tl.gemm_rs_pipe": 4}]' [--causal]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "flash_attention")]
import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
import example_mha_bwd as E  # noqa: E402

causal = "--causal" in sys.argv
args = [a for a in sys.argv[1:] if not a.startswith("--")]
variants = json.loads(args[0]) if args else [{}, {"tl.gemm_rs_pipe": 4}]
B, H, S, D = 8, 32, 1024, 64
torch.manual_seed(0)
q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
o, lse = E.flashattn_fwd(B, H, S, D, causal, dtype="float16")(q, k, v)
delta = E.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
E.ref_program(qr, kr, vr, causal).float().backward(do.float())
gq, gk, gv = qr.grad, kr.grad, vr.grad
unit = 2.0 * B * H * S * S * D * (0.5 if causal else 1.0)
bw, dqt = E._tiles(D, D, "bwd", causal), E._tiles(D, D, "dq", causal)
for pc in variants:
    cfg = dict(E.FAST_MATH)
    cfg.update(pc)
    tag = json.dumps(pc, sort_keys=True)
    try:
        f = E.flashattn_bwd.get_tir(B, H, S, D, causal, dtype="float16", dq_mode="none", **bw)
        kd = tilelang.compile(f, target="hip", pass_configs=cfg)
        dk, dv = torch.empty_like(k), torch.empty_like(v)
        kd(q, k, v, do, lse, delta, dk, dv)
        e1 = max((dk.float() - gk).abs().max().item(), (dv.float() - gv).abs().max().item())
        t1 = do_bench(lambda: kd(q, k, v, do, lse, delta, dk, dv), warmup=10, rep=50)
        f = E.flashattn_bwd_dq.get_tir(B, H, S, D, causal, dtype="float16", **dqt)
        kq = tilelang.compile(f, out_idx=[6], target="hip", pass_configs=cfg)
        dq = kq(q, k, v, do, lse, delta)
        e2 = (dq.float() - gq).abs().max().item()
        t2 = do_bench(lambda: kq(q, k, v, do, lse, delta), warmup=10, rep=50)
        print(f"{tag}: dkv {t1 * 1e3:.1f} us {4 * unit / t1 * 1e-9:.0f} TF err {e1:.3f} | dq {t2 * 1e3:.1f} us "
              f"{3 * unit / t2 * 1e-9:.0f} TF err {e2:.3f}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{tag}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
