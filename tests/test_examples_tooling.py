"""Tooling examples: carver-driven autotune, static analyzer, dynamic shapes."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("gemm", "analyze", "dynamic_shape"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))


def test_carver_configs_fit_mi355x():
    from example_gemm_autotune import get_configs, kernel
    import tilelang
    cfgs = get_configs(4096, 4096, 4096, with_roller=True, topk=6)
    assert cfgs and all(c["thread_num"] % 64 == 0 for c in cfgs)
    for c in cfgs[:3]:  # the recommended tilings lower within the 160 KiB LDS budget
        a = tilelang.lower(kernel(4096, 4096, 4096, **c), target="hip")
        assert a.lds_bytes <= 160 * 1024


def test_analyzer_flops():
    from example_gemm_analyze import main, M, N, K
    r = main()
    assert r.total_flops == 2 * M * N * K
    assert r.total_global_bytes > 0 and r.estimated_time_us > 0


def test_dynamic_shape_cpu():
    from example_dynamic import matmul_dynamic
    import example_dynamic
    import tilelang
    f = example_dynamic.matmul_dynamic_mnk.get_tir(64, 64, 32, False, True, "float16", "float32", "float32", 2, 128)
    k = tilelang.compile(f, target="cpu")
    for m, n, kk in ((64, 128, 64), (80, 72, 96)):
        A = torch.randn(m, kk, dtype=torch.float16)
        B = torch.randn(n, kk, dtype=torch.float16)
        C = torch.empty(m, n)
        k(A, B, C)
        torch.testing.assert_close(C, A.float() @ B.float().T, rtol=1e-2, atol=1e-2)
    assert matmul_dynamic is not None


@pytest.mark.gpu
def test_autotune_gpu():
    from example_gemm_autotune import autotune
    res = autotune(1024, 1024, 1024, with_roller=True, topk=4, warmup=2, rep=5)
    assert res.config is not None and res.latency > 0


@pytest.mark.gpu
def test_dynamic_shape_gpu():
    from example_dynamic import matmul_dynamic
    for m, n, k in ((1024, 1024, 1024), (776, 1536, 2048), (136, 200, 264)):
        matmul_dynamic(m, n, k, 128, 128, 32, False, False, "float16", "float16", "float32", 3, 256)
        matmul_dynamic(m, n, k, 128, 128, 32, True, True, "float16", "float16", "float32", 2, 256)
