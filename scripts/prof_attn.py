"""Run one attention kernel N times (for rocprofv3 --kernel-trace / --pmc)."""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT] + sorted(d for d in glob.glob(os.path.join(ROOT, "examples", "*")) if os.path.isdir(d))
import torch  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "sink"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
if which in ("sink", "sink_nc"):
    import example_gqa_sink_fwd_bhsd as m
    B, H, S, D, G = 1, 64, 4096, 128, 8
    k = m.flashattn_sink(B, H, S, S, D, G, causal=(which == "sink"))
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(B, H // G, S, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(kk)
    s = torch.randn(H, device="cuda", dtype=torch.bfloat16)
    run = lambda: k(q, kk, v, s)  # noqa: E731
elif which == "fa":
    import example_mha_fwd as m
    k = m.flashattn(1, 64, 4096, 128, False, 1, 256, 64, 512, 2, "bfloat16")
    q = torch.randn(1, 4096, 64, 128, device="cuda", dtype=torch.bfloat16)
    run = lambda: k(q, q, q)  # noqa: E731
elif which == "mamba":
    import example_mamba_chunk_scan as m
    args = m.make_inputs(8, 4096, 256, 1, 80, 64, 128)
    k = m.chunk_scan_fwd(8, 4096, 256, 1, 80, 64, 128)
    run = lambda: k(*args)  # noqa: E731
elif which == "fa_bwd":
    import example_mha_bwd as m
    B, S, H, D = 8, 1024, 32, 64
    Q = torch.randn(B, S, H, D, dtype=torch.half, device="cuda").requires_grad_()
    O = m.attention(Q, Q.detach().clone().requires_grad_(), Q.detach().clone().requires_grad_(), False)
    dO = torch.randn_like(Q)
    run = lambda: O.backward(dO, retain_graph=True)  # noqa: E731
for _ in range(reps):
    run()
torch.cuda.synchronize()
print("done", which)
