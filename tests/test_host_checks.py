"""Host-side argument checks of the native launcher, one test per class of the reference's
``maint/host_checks/01..10_*.py`` (num args, pointer type, ndim, dtype, shape, strides, device
type, device id, null data pointer, scalar type).  The reference's scripts are manual repros;
here every class must raise a precise error before anything is launched."""
import pytest
import torch

import tilelang
import tilelang.language as T


def _matmul(M=64, N=64, K=64, target="cpu"):

    @T.prim_func
    def main(A: T.Tensor((M, K), "float32"), B: T.Tensor((K, N), "float32"), C: T.Tensor((M, N), "float32")):
        with T.Kernel(T.ceildiv(N, 32), T.ceildiv(M, 32), threads=64) as (bx, by):
            A_s = T.alloc_shared((32, 32), "float32")
            B_s = T.alloc_shared((32, 32), "float32")
            acc = T.alloc_fragment((32, 32), "float32")
            T.clear(acc)
            for k in T.Pipelined(K // 32, num_stages=1):
                T.copy(A[by * 32, k * 32], A_s)
                T.copy(B[k * 32, bx * 32], B_s)
                T.gemm(A_s, B_s, acc)
            T.copy(acc, C[by * 32, bx * 32])

    return tilelang.compile(main, out_idx=[2], target=target)


def _scalar_kernel(target="cpu"):

    @T.prim_func
    def main(x: T.int32, flag: T.bool, s: T.float32, O: T.Tensor((4, ), "float32")):
        with T.Kernel(1, threads=4):
            for i in T.Parallel(4):
                O[i] = T.Cast("float32", x) + T.Cast("float32", flag) + s

    return tilelang.compile(main, out_idx=[3], target=target)


@pytest.fixture(scope="module")
def mm():
    return _matmul()


def _ab(dev="cpu", dtype=torch.float32):
    return torch.randn(64, 64, device=dev, dtype=dtype), torch.randn(64, 64, device=dev, dtype=dtype)


def test_01_num_args(mm):
    a, _ = _ab()
    with pytest.raises(ValueError, match="expected 2 inputs, got 1"):
        mm(a)


def test_02_pointer_type(mm):
    _, b = _ab()
    with pytest.raises(TypeError, match="argument 'A' expects a pointer"):
        mm(1, b)


def test_03_ndim(mm):
    a, b = _ab()
    with pytest.raises(ValueError, match="argument 'A' has 3 dims, expected 2"):
        mm(a.reshape(1, 64, 64), b)


def test_04_dtype(mm):
    a, b = _ab()
    with pytest.raises(ValueError, match="argument 'B' has dtype float16, expected float32"):
        mm(a, b.half())


def test_05_shape(mm):
    a, b = _ab()
    with pytest.raises(ValueError, match="argument 'A' dim 0 is 32, expected 64"):
        mm(a[:32], b)


def test_06_strides(mm):
    a, b = _ab()
    with pytest.raises(ValueError, match="argument 'A' must be contiguous"):
        mm(a.t(), b)


def test_07_device_type_cpu_kernel():
    """A CPU kernel refuses device tensors (and a GPU kernel host tensors: tested on the GPU)."""
    k = _matmul()
    if not torch.cuda.is_available():
        a, b = _ab()
        assert k(a, b).shape == (64, 64)
        return
    a, b = _ab("cuda")
    with pytest.raises(ValueError, match="must be a CPU tensor"):
        k(a, b)


@pytest.mark.gpu
def test_07_device_type_gpu_kernel():
    k = _matmul(target="hip")
    a, b = _ab()
    with pytest.raises(ValueError, match="must be on a ROCm"):
        k(a, b)


@pytest.mark.gpu
def test_08_device_id():
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    k = _matmul(target="hip")
    a = torch.randn(64, 64, device="cuda:0")
    b = torch.randn(64, 64, device="cuda:1")
    with pytest.raises(ValueError, match="is on device 1 but other arguments are on device 0"):
        k(a, b)


def test_09_null_data_pointer(mm):
    """An undefined tensor / ``None`` where a buffer is expected."""
    _, b = _ab()
    with pytest.raises(TypeError, match="argument 'A' expects a pointer \\(torch.Tensor\\), got NoneType"):
        mm(None, b)


def test_10_scalar_type():
    k = _scalar_kernel()
    out = k(3, True, 0.5)
    assert torch.equal(out, torch.full((4, ), 4.5))
    with pytest.raises(TypeError, match="argument 'x' expects an integer, got float"):
        k(1.0, True, 0.5)
    with pytest.raises(TypeError, match="argument 'flag' expects a bool, got float"):
        k(1, 2.5, 0.5)
    with pytest.raises(TypeError, match="argument 'flag' expects a bool, got the integer 2"):
        k(1, 2, 0.5)
    with pytest.raises(TypeError, match="argument 's' expects a float, got str"):
        k(1, True, "x")
    assert torch.equal(k(1, 0, 2), torch.full((4, ), 3.0))  # int for float, 0/1 for bool: accepted
