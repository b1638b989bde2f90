import sys, os
R = os.path.join(os.path.dirname(__file__), "..")
for p in ("", "examples/gemm_fp8", "examples/deepseek_mla"):
    sys.path.insert(0, os.path.join(R, p))
import torch
from tilelang.profiler import do_bench
from example_tilelang_gemm_fp8 import matmul as f8mm
from example_mla_decode import mla_decode, flops as mla_flops
M = N = K = 8192
a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
try:
    sa, sb = torch.tensor(1.0, device="cuda"), torch.tensor(1.0, device="cuda")
    t = do_bench(lambda: torch._scaled_mm(a, b.t(), sa, sb, out_dtype=torch.bfloat16))
    print(f"torch._scaled_mm fp8 8192^3: {t:.3f} ms {2*M*N*K/t*1e-9:.1f} TF", flush=True)
except Exception as e:
    print("scaled_mm failed", str(e)[:200], flush=True)
for cfg in [(256, 256, 128, 512, 2), (256, 256, 128, 512, 3), (128, 128, 128, 256, 2), (256, 128, 128, 256, 2), (256, 256, 256, 512, 2)]:
    try:
        k = f8mm(M, N, K, *cfg)
        c = k(a, b)
        t = do_bench(lambda: k(a, b))
        print(f"fp8 gemm cfg {cfg}: {t:.3f} ms {2*M*N*K/t*1e-9:.1f} TF", flush=True)
    except Exception as e:
        print(f"fp8 cfg {cfg} FAILED {type(e).__name__} {str(e)[:300]}", flush=True)
for batch in (64, 128):
    for kv in (1024, 4096, 8192, 16384):
        best = None
        for ns in (1, 2, 4, 8):
            try:
                k = mla_decode(batch, 128, 1, kv, 512, 64, num_split=ns)
                q = torch.randn(batch, 128, 512, device="cuda", dtype=torch.float16)
                qp = torch.randn(batch, 128, 64, device="cuda", dtype=torch.float16)
                kvt = torch.randn(batch, kv, 1, 512, device="cuda", dtype=torch.float16)
                kp = torch.randn(batch, kv, 1, 64, device="cuda", dtype=torch.float16)
                g = torch.empty(batch, 128, ns, device="cuda")
                po = torch.empty(batch, 128, ns, 512, device="cuda")
                t = do_bench(lambda: k(q, qp, kvt, kp, g, po))
                tf = mla_flops(batch, 128, kv, 512, 64) / t * 1e-9
                if best is None or tf > best[0]:
                    best = (tf, ns, t)
            except Exception as e:
                print(f"mla b{batch} kv{kv} ns{ns} FAILED {type(e).__name__} {str(e)[:200]}", flush=True)
        print(f"MLA decode b{batch} h128 kv{kv}: best {best[0]:.1f} TF (num_split={best[1]}, {best[2]:.3f} ms)", flush=True)
