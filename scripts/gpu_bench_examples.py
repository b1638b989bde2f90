"""Benchmark the example kernels on one MI355X (numbers go to docs/RESULTS.md).

    python scripts/gpu_bench_examples.py [name ...]      (default: all)
Each entry checks numerics first, then times with tilelang.profiler.do_bench (HIP events,
L2+MALL flush between runs).  One line per workload is printed as JSON.
"""
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT] + sorted(d for d in glob.glob(os.path.join(ROOT, "examples", "*")) if os.path.isdir(d))

import torch  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

HBM_PEAK_GBS = 8000.0


def _emit(name, ms, **kw):
    d = dict(workload=name, ms=round(ms, 4), **kw)
    print(json.dumps(d), flush=True)


def b_elementwise():
    import example_elementwise_add as m
    M = N = 8192
    k = m.elementwise_add(M, N)
    a, b = torch.randn(M, N, device="cuda"), torch.randn(M, N, device="cuda")
    torch.testing.assert_close(k(a, b), a + b)
    ms = do_bench(lambda: k(a, b))
    gbs = 3 * M * N * 4 / ms * 1e-6
    _emit("elementwise_add fp32 8192^2", ms, GBs=round(gbs, 1), pct_hbm=round(100 * gbs / HBM_PEAK_GBS, 1))


def b_rms():
    import rms_norm as m
    M, N = 8192, 8192
    k = m.rms_norm(M, N, 4)
    x = torch.randn(M, N, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-4)
    ms = do_bench(lambda: k(x))
    gbs = 2 * M * N * 4 / ms * 1e-6
    _emit("rms_norm fp32 8192^2", ms, GBs=round(gbs, 1), pct_hbm=round(100 * gbs / HBM_PEAK_GBS, 1),
          torch_ms=round(do_bench(lambda: m.ref_program(x)), 4))


def b_softmax():
    import online_softmax as m
    M, N = 4096, 8192
    k = m.online_softmax(M, N)
    x = torch.randn(M, N, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-6)
    ms = do_bench(lambda: k(x))
    _emit("online_softmax fp32 4096x8192", ms, GBs_effective=round(2 * M * N * 4 / ms * 1e-6, 1),
          torch_ms=round(do_bench(lambda: torch.softmax(x, -1)), 4))


def b_cast():
    import example_per_token_cast_to_fp8 as m
    M = N = 8192
    k = m.per_token_cast_to_fp8(M, N, 8)
    x = torch.randn(M, N, device="cuda")
    ms = do_bench(lambda: k(x))
    gbs = M * N * 5 / ms * 1e-6
    _emit("per_token_cast_to_fp8 8192^2", ms, GBs=round(gbs, 1), pct_hbm=round(100 * gbs / HBM_PEAK_GBS, 1))


def b_gemv():
    import example_gemv as m
    N = K = 16384
    k = m.gemv(N, K)
    A = torch.randn(N, K, device="cuda", dtype=torch.float16)
    x = torch.randn(K, device="cuda", dtype=torch.float16)
    ms = do_bench(lambda: k(A, x))
    gbs = N * K * 2 / ms * 1e-6
    _emit("gemv fp16 16384^2", ms, GBs=round(gbs, 1), pct_hbm=round(100 * gbs / HBM_PEAK_GBS, 1),
          torch_ms=round(do_bench(lambda: A @ x), 4))


def b_splitk():
    import example_tilelang_gemm_splitk as m
    M, N, K = 1024, 1024, 16384
    k = m.matmul_splitk(M, N, K, split_k=8)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = torch.zeros(M, N, device="cuda")

    def run():
        c.zero_()
        k(a, b, c)

    ms = do_bench(run)
    _emit("splitk gemm 1024x1024x16384 (split 8)", ms, TFLOPS=round(2 * M * N * K / ms * 1e-9, 1),
          torch_ms=round(do_bench(lambda: a @ b), 4))


def b_fa_bwd():
    import example_mha_bwd as m
    B, S, H, D = 8, 1024, 32, 64
    Q = torch.randn(B, S, H, D, dtype=torch.half, device="cuda").requires_grad_()
    K = torch.randn_like(Q).requires_grad_()
    V = torch.randn_like(Q).requires_grad_()
    dO = torch.randn_like(Q)
    O = m.attention(Q, K, V, False)
    ms = do_bench(lambda: O.backward(dO, retain_graph=True))
    flops = 5 * 2.0 * B * H * S * S * D
    _emit("flash_attention bwd fp16 b8 h32 s1024 d64", ms, TFLOPS=round(flops / ms * 1e-9, 1))


def b_hadamard():
    import example_hadamard as m
    k = m.hadamard(64, 32768)
    x = torch.randn(64, 32768, device="cuda")
    ms = do_bench(lambda: k(x))
    _emit("hadamard 64x32768 fp32", ms)


def b_sink():
    import example_gqa_sink_fwd_bhsd as m
    B, H, S, D, G = 1, 64, 4096, 128, 8
    k = m.flashattn_sink(B, H, S, S, D, G)
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(B, H // G, S, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(kk)
    s = torch.randn(H, device="cuda", dtype=torch.bfloat16)
    ms = do_bench(lambda: k(q, kk, v, s))
    _emit("gqa+sink fwd causal bf16 b1 h64 kvh8 s4096 d128 (reference headline 497 TF on H800)", ms,
          TFLOPS=round(m.flops(B, H, S, S, D) / ms * 1e-9, 1))


def b_decode():
    import example_gqa_decode as m
    b, h, g, s, d, ns = 32, 32, 8, 8192, 128, 8
    k = m.gqa_decode(b, h, g, s, d, num_split=ns)
    q = torch.randn(b, h, d, device="cuda", dtype=torch.float16)
    kk = torch.randn(b, s, g, d, device="cuda", dtype=torch.float16)
    v = torch.randn_like(kk)
    lens = torch.full((b, ), s, dtype=torch.int32, device="cuda")
    glse = torch.empty(b, h, ns, device="cuda")
    part = torch.empty(b, h, ns, d, device="cuda")
    ms = do_bench(lambda: k(q, kk, v, lens, glse, part))
    gbs = 2 * b * s * g * d * 2 / ms * 1e-6
    _emit("gqa decode fp16 b32 h32 g8 kv8192 d128", ms, GBs=round(gbs, 1), pct_hbm=round(100 * gbs / HBM_PEAK_GBS, 1))


def b_mamba():
    import example_mamba_chunk_scan as m
    for seq in (1024, 4096, 16384):
        args = m.make_inputs(8, seq, 256, 1, 80, 64, 128)
        k = m.chunk_scan_fwd(8, seq, 256, 1, 80, 64, 128)
        ms = do_bench(lambda: k(*args))
        _emit(f"mamba2 chunk scan b8 h80 chunk256 d64 dstate128 seq{seq} (reference 126-136 TF on H800)", ms,
              TFLOPS=round(m.flops(8, seq, 256, 80, 64, 128) / ms * 1e-9, 1))


def b_linear_attn():
    import example_linear_attn_fwd as m
    B, S, H, D = 1, 8192, 32, 128
    k = m.linear_attn_fwd(B, S, H, D, D)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) * 0.1
    kk = torch.randn_like(q) * 0.1
    v = torch.randn_like(q)
    ms = do_bench(lambda: k(q, kk, v))
    flops = B * H * (S // 64) * (2 * 64 * 64 * D * 2 + 2 * 64 * D * D * 2)
    _emit("linear attention fwd b1 s8192 h32 d128", ms, TFLOPS=round(flops / ms * 1e-9, 1))


BENCHES = {n[2:]: f for n, f in globals().items() if n.startswith("b_")}

if __name__ == "__main__":
    names = sys.argv[1:] or list(BENCHES)
    for n in names:
        t = time.time()
        try:
            BENCHES[n]()
        except Exception as e:  # noqa: BLE001 - report and continue with the next workload
            print(json.dumps(dict(workload=n, error=f"{type(e).__name__}: {str(e)[:300]}")), flush=True)
        sys.stderr.write(f"{n}: {time.time() - t:.1f}s\n")
