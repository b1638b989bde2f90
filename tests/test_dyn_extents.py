"""Dynamic tensor extents of the form a*n + b (jit/kernel.py _affine_of): proved on the IR, so a
non-affine extent (min, max, floordiv, mod) is refused at compile time instead of having the
launcher size an output or bind the symbol with a formula fitted at three sample points."""
import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang.jit.kernel import _linear_in


def pad_copy(n, ext_fn):

    @T.prim_func
    def main(A: T.Tensor((n, ), "float32"), B: T.Tensor((ext_fn(n), ), "float32")):
        with T.Kernel(1, threads=64):
            for i in T.serial(n):
                B[i] = A[i] * 2.0

    return main


def test_affine_extent_allocates_output():
    n = T.dynamic("n")
    k = tilelang.compile(pad_copy(n, lambda v: 2 * v + 3), out_idx=[1], target="cpu")
    a = torch.randn(10)
    b = k(a)
    assert b.shape == (23, )
    torch.testing.assert_close(b[:10], a * 2)


@pytest.mark.parametrize("ext", [lambda v: T.min(v, 64), lambda v: v + v // 8, lambda v: T.max(v, 1),
                                 lambda v: v % 7 + v])
def test_non_affine_extent_refused(ext):
    n = T.dynamic("n")
    with pytest.raises(ValueError, match="unsupported dynamic shape"):
        tilelang.compile(pad_copy(n, ext), out_idx=[1], target="cpu")


def test_linear_form():
    n = T.dynamic("n")
    assert _linear_in(3 * (n + 2) - n, n) == (2, 6)
    assert _linear_in(n * 4 - 1, n) == (4, -1)
    assert _linear_in(n * n, n) is None
    assert _linear_in(T.min(n, 64), n) is None
