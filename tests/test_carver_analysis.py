"""Carver analysis of arbitrary loop-nest programs (reference carver/roller/node.py,
matmul_analysis.py): axis classification, GEMM recognition, recommendation dispatch."""
import pytest

import tilelang.language as T
from tilelang.carver.analysis import AnalysisError, PrimFuncNode, gemm_info, implicit_gemm, recommend


def naive_gemm(M, N, K, trans_b=True):
    if not trans_b:
        @T.prim_func
        def nn(A: T.Tensor((M, K), "float16"), B: T.Tensor((K, N), "float16"), C: T.Tensor((M, N), "float32")):
            with T.Kernel(1, threads=1) as bx:
                for i, j, k in T.grid(M, N, K):
                    C[i, j] = C[i, j] + T.Cast("float32", A[i, k]) * T.Cast("float32", B[k, j])

        return nn

    @T.prim_func
    def nt(A: T.Tensor((M, K), "float16"), B: T.Tensor((N, K), "float16"), C: T.Tensor((M, N), "float32")):
        with T.Kernel(1, threads=1) as bx:
            for i, j, k in T.grid(M, N, K):
                C[i, j] = C[i, j] + T.Cast("float32", A[i, k]) * T.Cast("float32", B[j, k])

    return nt


def test_gemm_recognised_and_ranked():
    node = PrimFuncNode.from_func(naive_gemm(4096, 2048, 1024))
    assert [v.name for v in node.spatial] == ["i", "j"] and [v.name for v in node.reduce] == ["k"]
    assert node.reduce_kind == "sum" and node.get_space_dim() == [4096, 2048] and node.get_reduce_dim() == [1024]
    assert node.infer_shapes() == {"C": [4096, 2048], "A": [4096, 1024], "B": [2048, 1024]}
    g = gemm_info(node)
    assert (g.M, g.N, g.K, g.batch, g.trans_A, g.trans_B) == (4096, 2048, 1024, 1, False, True)
    hints, what = recommend(naive_gemm(4096, 2048, 1024), topk=4)
    assert what["kind"] == "gemm" and len(hints) == 4
    cfg = hints[0].to_config()
    assert {"block_M", "block_N", "block_K", "threads", "num_stages"} <= set(cfg)
    assert gemm_info(PrimFuncNode.from_func(naive_gemm(256, 256, 256, trans_b=False))).trans_B is False


def test_batched_gemm():
    @T.prim_func
    def bmm(A: T.Tensor((8, 128, 64), "float16"), B: T.Tensor((8, 96, 64), "float16"),
            C: T.Tensor((8, 128, 96), "float32")):
        with T.Kernel(1, threads=1) as bx:
            for b, i, j, k in T.grid(8, 128, 96, 64):
                C[b, i, j] = C[b, i, j] + A[b, i, k] * B[b, j, k]

    g = gemm_info(PrimFuncNode.from_func(bmm))
    assert (g.batch, g.M, g.N, g.K) == (8, 128, 96, 64)


def test_reduction_and_elementwise():
    @T.prim_func
    def rowmax(X: T.Tensor((1024, 4096), "float32"), Y: T.Tensor((1024, ), "float32")):
        with T.Kernel(1, threads=1) as bx:
            for i, j in T.grid(1024, 4096):
                Y[i] = T.max(Y[i], X[i, j])

    hints, what = recommend(rowmax, topk=3)
    assert what == {"kind": "reduction", "reduce_len": 4096} and hints

    @T.prim_func
    def add(X: T.Tensor((1024, 1024), "float16"), Z: T.Tensor((1024, 1024), "float16"),
            Y: T.Tensor((1024, 1024), "float16")):
        with T.Kernel(1, threads=1) as bx:
            for i, j in T.grid(1024, 1024):
                Y[i, j] = X[i, j] + Z[i, j]

    hints, what = recommend(add, topk=3)
    assert what["kind"] == "elementwise" and hints[0].threads in (128, 256, 512)


def test_direct_conv_is_implicit_gemm():
    N_, H, W, C, F, R = 2, 16, 16, 32, 64, 3

    @T.prim_func
    def conv(X: T.Tensor((N_, H + 2, W + 2, C), "float16"), Wt: T.Tensor((F, R, R, C), "float16"),
             Y: T.Tensor((N_, H, W, F), "float32")):
        with T.Kernel(1, threads=1) as bx:
            for n, h, w, f, r, s, c in T.grid(N_, H, W, F, R, R, C):
                Y[n, h, w, f] = Y[n, h, w, f] + X[n, h + r, w + s, c] * Wt[f, r, s, c]

    node = PrimFuncNode.from_func(conv)
    assert gemm_info(node) is None
    assert implicit_gemm(node) == (N_ * H * W, F, R * R * C)
    hints, what = recommend(conv, topk=2)
    assert what["kind"] == "conv_like" and hints


def test_non_accumulating_reduce_axis_is_refused():
    @T.prim_func
    def bad(X: T.Tensor((64, 64), "float32"), Y: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=1) as bx:
            for i, j in T.grid(64, 64):
                Y[i] = X[i, j]

    with pytest.raises(AnalysisError, match="does not accumulate"):
        PrimFuncNode.from_func(bad)
