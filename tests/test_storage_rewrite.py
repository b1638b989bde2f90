"""StorageRewrite for per-thread local arrays (transform/storage_rewrite.py)."""
import torch

import tilelang
import tilelang.language as T
from tilelang.transform.storage_rewrite import rewrite_local_storage


def _prog(n=256):

    @T.prim_func
    def main(A: T.Tensor((n, 8), "float32"), I: T.Tensor((n, ), "int32"), B: T.Tensor((n, ), "float32"),
             C: T.Tensor((n, ), "float32")):
        with T.Kernel(n, threads=64) as bx:  # one row per block (every lane computes it)
            u = T.alloc_local((8, ), "float32")  # dynamically indexed: a private array
            v = T.alloc_local((8, ), "float32")  # same dtype/shape, live only after u dies
            w = T.alloc_local((4, ), "float32")  # different shape: kept
            for j in T.serial(8):
                u[j] = A[bx, j]
            B[bx] = u[I[bx] % 8]
            for j in T.serial(8):
                v[j] = A[bx, j] * 2.0
            w[0] = v[(I[bx] + 1) % 8]
            C[bx] = w[0]

    return main


def test_disjoint_local_arrays_share_storage():
    f = _prog()
    k2, merged = rewrite_local_storage([s for s in __import__("tilelang.ir.stmt", fromlist=["walk"]).walk(f.body)
                                        if type(s).__name__ == "KernelStmt"][0])
    assert merged == {"v": "u"}
    src = tilelang.compile(f, out_idx=[2, 3], target="hip").get_kernel_source()
    assert " v[" not in src and "u[" in src
    src_off = tilelang.compile(f, out_idx=[2, 3], target="hip",
                               pass_configs={"tir.disable_storage_rewrite": True}).get_kernel_source()
    assert " v[" in src_off or "v[8]" in src_off


def test_merged_program_computes_the_same():
    f = _prog()
    k = tilelang.compile(f, out_idx=[2, 3], target="cpu")
    A = torch.randn(256, 8)
    I = torch.randint(0, 100, (256, ), dtype=torch.int32)
    b, c = k(A, I)
    rows = torch.arange(256)
    torch.testing.assert_close(b, A[rows, (I % 8).long()])
    torch.testing.assert_close(c, 2 * A[rows, ((I + 1) % 8).long()])


def _inplace_prog(n=64, shifted=False):

    @T.prim_func
    def main(A: T.Tensor((n, 8), "float32"), I: T.Tensor((n, ), "int32"), C: T.Tensor((n, ), "float32")):
        with T.Kernel(n, threads=64) as bx:
            u = T.alloc_local((8, ), "float32")
            v = T.alloc_local((8, ), "float32")
            for j in T.serial(8):
                u[j] = A[bx, j]
            if shifted:
                for j in T.serial(8):
                    v[j] = u[(j + 1) % 8] * 2.0  # reads an element another iteration overwrites
            else:
                for j in T.serial(8):
                    v[j] = u[j] * 2.0 + 1.0  # element-wise: v may live in u's storage
            C[bx] = v[I[bx] % 8]

    return main


def _kernel_of(f):
    from tilelang.ir import stmt as S
    return [s for s in S.walk(f.body) if isinstance(s, S.KernelStmt)][0]


def test_inplace_detection():
    _, merged = rewrite_local_storage(_kernel_of(_inplace_prog()))
    assert merged == {}  # live ranges touch: not merged without in-place detection
    _, merged = rewrite_local_storage(_kernel_of(_inplace_prog()), detect_inplace=True)
    assert merged == {"v": "u"}
    _, merged = rewrite_local_storage(_kernel_of(_inplace_prog(shifted=True)), detect_inplace=True)
    assert merged == {}
    for shifted in (False, True):
        f = _inplace_prog(shifted=shifted)
        k = tilelang.compile(f, out_idx=[2], target="cpu", pass_configs={"tl.storage_rewrite_detect_inplace": True})
        A = torch.randn(64, 8)
        I = torch.randint(0, 100, (64, ), dtype=torch.int32)
        rows = torch.arange(64)
        j = (I % 8).long()
        ref = 2 * A[rows, (j + 1) % 8] if shifted else 2 * A[rows, j] + 1
        torch.testing.assert_close(k(A, I), ref)
        src = tilelang.compile(f, out_idx=[2], target="hip",
                               pass_configs={"tl.storage_rewrite_detect_inplace": True}).get_kernel_source()
        assert ("v[" in src) == shifted


def _reread_prog(n=64):

    @T.prim_func
    def main(A: T.Tensor((n, 8), "float32"), I: T.Tensor((n, ), "int32"), C: T.Tensor((n, ), "float32")):
        with T.Kernel(n, threads=64) as bx:
            u = T.alloc_local((8, ), "float32")
            v = T.alloc_local((8, ), "float32")
            w = T.alloc_local((8, ), "float32")
            for j in T.serial(8):
                u[j] = A[bx, j]
            for j in T.serial(8):
                v[j] = u[j] * 2.0
                w[j] = u[j] + 1.0  # reads u[j] AFTER v[j] was written: v must not take u's storage
            C[bx] = v[I[bx] % 8] + w[I[bx] % 8]

    return main


def test_inplace_rejects_read_after_write():
    _, merged = rewrite_local_storage(_kernel_of(_reread_prog()), detect_inplace=True)
    assert merged.get("v") != "u"
    k = tilelang.compile(_reread_prog(), out_idx=[2], target="cpu",
                         pass_configs={"tl.storage_rewrite_detect_inplace": True})
    A = torch.randn(64, 8)
    I = torch.randint(0, 100, (64, ), dtype=torch.int32)
    x = A[torch.arange(64), (I % 8).long()]
    torch.testing.assert_close(k(A, I), 3 * x + 1)
