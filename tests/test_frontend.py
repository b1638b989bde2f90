import pytest
import tilelang.language as T
from tilelang.ir import stmt as S


def _gemm_func(M=256, N=256, K=128, bm=128, bn=128, bk=32):

    @T.prim_func
    def gemm(A: T.Tensor((M, K), "float16"), B: T.Tensor((K, N), "float16"), C: T.Tensor((M, N), "float16")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=256) as (bx, by):
            A_shared = T.alloc_shared((bm, bk), "float16")
            B_shared = T.alloc_shared((bk, bn), "float16")
            C_local = T.alloc_fragment((bm, bn), "float")
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=3):
                T.copy(A[by * bm, k * bk], A_shared)
                T.copy(B[k * bk, bx * bn], B_shared)
                T.gemm(A_shared, B_shared, C_local)
            T.copy(C_local, C[by * bm, bx * bn])

    return gemm


def test_trace_gemm_structure():
    f = _gemm_func()
    ops = [s.op for s in S.walk(f.body) if isinstance(s, S.TileOpStmt)]
    kinds = [o.kind for o in ops]
    assert kinds == ["fill", "copy", "copy", "gemm", "copy"]
    loops = [s for s in S.walk(f.body) if isinstance(s, S.ForStmt)]
    assert loops[0].kind == "pipelined" and loops[0].annotations["num_stages"] == 3
    # point copy regions pick up the shared tile extents
    cp = ops[1]
    assert cp.src.static_extents() == [128, 32]
    script = f.script()
    assert "T.Pipelined(4, num_stages=3)" in script
    assert "T.gemm(A_shared" in script


def test_dynamic_control_flow_and_vars():

    @T.prim_func
    def k(A: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=64) as bx:
            x = T.alloc_var("int32")
            x = 3
            if bx > 0 and x < 5:
                x = x + 1
            else:
                x = 0
            i = T.alloc_var("int32")
            i = 0
            while i < 4:
                i = i + 1
            for j in range(4):
                if j == 2:
                    break
                A[j] = A[j] + x

    s = k.script()
    assert "if bx > 0 and x[0] < 5:" in s
    assert "while i[0] < 4:" in s
    assert "T.loop_break()" in s
    assert "x[0] = x[0] + 1" in s


def test_static_python_branches_are_not_traced():
    flag = False

    @T.prim_func
    def k(A: T.Tensor((8, ), "float32")):
        with T.Kernel(1, threads=64):
            if flag:
                A[0] = 1.0
            else:
                A[1] = 2.0

    s = k.script()
    assert "A[1] = 2.0" in s and "A[0]" not in s


def test_macro_inlines():

    @T.macro
    def twice(buf, i):
        buf[i] = buf[i] * 2

    @T.prim_func
    def k(A: T.Tensor((8, ), "float32")):
        with T.Kernel(1, threads=64):
            for i in T.serial(8):
                twice(A, i)

    assert "A[i] = A[i] * 2" in k.script()


def test_missing_annotation_errors():
    with pytest.raises(TypeError):

        @T.prim_func
        def k(A):
            pass
