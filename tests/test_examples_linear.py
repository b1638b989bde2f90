"""Linear-attention / SSM family beyond the chunk scan: Mamba-2 chunk state and RetNet retention.
CPU-target numerics (plus a gfx950 compile) and the same kernels on an MI355X against fp32 PyTorch."""
import pytest
import torch

import tilelang


def test_mamba_chunk_state_cpu():
    import example_mamba_chunk_state as m
    f = m.chunk_state_fwd.get_tir(1, 512, 128, 1, 2, 64, 64, block_K=32)
    assert len(tilelang.compile(f, out_idx=[4], target="hip").code[0]) > 0
    args = m.make_inputs(1, 512, 128, 1, 2, 64, 64, device="cpu")
    k = tilelang.compile(f, out_idx=[4], target="cpu")
    torch.testing.assert_close(k(*args).float(), m.ref_program(*args), rtol=1e-2, atol=2e-2)


def test_retention_fwd_cpu():
    import example_retention_fwd as m
    f = m.chunk_retention_fwd.get_tir(1, 256, 2, 64, 64)
    assert len(tilelang.compile(f, out_idx=[3], target="hip").code[0]) > 0
    q, k, v = [torch.randn(1, 256, 2, 64).half() for _ in range(3)]
    o = tilelang.compile(f, out_idx=[3], target="cpu")(q, k, v)
    torch.testing.assert_close(o.float(), m.ref_program(q, k, v), rtol=1e-2, atol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [1, 2])
def test_mamba_chunk_state_gpu(groups):
    import example_mamba_chunk_state as m
    args = m.make_inputs(2, 1024, 256, groups, 4, 64, 128)
    out = m.chunk_state_fwd(2, 1024, 256, groups, 4, 64, 128)(*args)
    torch.testing.assert_close(out.float(), m.ref_program(*args), rtol=2e-2, atol=5e-2)


@pytest.mark.gpu
def test_retention_fwd_gpu():
    import example_retention_fwd as m
    q, k, v = [torch.randn(2, 512, 4, 128, device="cuda", dtype=torch.float16) for _ in range(3)]
    o = m.chunk_retention_fwd(2, 512, 4, 128, 128)(q, k, v)
    torch.testing.assert_close(o.float(), m.ref_program(q, k, v), rtol=2e-2, atol=5e-2)
