"""int64 index promotion (reference src/transform/config_index_bitwidth.cc): tensors of >= 2^31
elements are addressed with 64-bit offsets; 32-bit kernels refuse tensors that would overflow."""
import pytest
import torch

import tilelang
import tilelang.language as T


def copy_kernel(M, N, bm=64, bn=256, dtype="float16"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=256) as (bx, by):
            S = T.alloc_shared((bm, bn), dtype)
            T.copy(A[by * bm, bx * bn], S)
            T.copy(S, B[by * bm, bx * bn])

    return main


def test_large_static_tensor_uses_int64():
    k = tilelang.compile(copy_kernel(65536, 32768), target="hip")
    assert "(int64_t)" in k.get_kernel_source()
    assert not k.artifact.kernels[0].narrow_index
    small = tilelang.compile(copy_kernel(1024, 1024), target="hip")
    assert "int64" not in small.get_kernel_source()
    assert small.artifact.kernels[0].narrow_index == {"A", "B"}


def test_pass_config_forces_bitwidth():
    k = tilelang.compile(copy_kernel(1024, 1024), target="hip", pass_configs={"tl.config_index_bitwidth": 64})
    assert "(int64_t)" in k.get_kernel_source()
    with pytest.raises(Exception, match="config_index_bitwidth=32"):
        tilelang.compile(copy_kernel(65536, 32768), target="hip", pass_configs={"tl.config_index_bitwidth": 32})


def test_runtime_refuses_overflowing_dynamic_tensor():
    k = tilelang.compile(copy_kernel(T.dynamic("m"), 1024), target="cpu")
    a = torch.empty((2**21 + 64, 1024), dtype=torch.float16)  # > 2^31 elements, never touched
    with pytest.raises(ValueError, match="32-bit offsets"):
        k(a, a)
    k64 = tilelang.compile(copy_kernel(T.dynamic("m"), 1024), target="cpu",
                           pass_configs={"tl.config_index_bitwidth": 64})
    assert not k64.artifact.kernels[0].narrow_index


@pytest.mark.gpu
def test_copy_more_than_2e31_elements_gpu():
    M, N = 65536, 32768 + 256  # 2^31 + 2^24 elements (4.03 GiB fp16)
    k = tilelang.compile(copy_kernel(M, N), target="hip")
    a = torch.empty(M, N, dtype=torch.float16, device="cuda")
    a[-8:].copy_(torch.randn(8, N, device="cuda").half())
    a[:8].copy_(torch.randn(8, N, device="cuda").half())
    b = torch.zeros_like(a)
    k(a, b)
    torch.cuda.synchronize()
    assert torch.equal(b[-8:], a[-8:]) and torch.equal(b[:8], a[:8])
    del a, b
    torch.cuda.empty_cache()
