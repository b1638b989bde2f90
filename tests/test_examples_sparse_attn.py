"""Sparse attention families: MInference vertical-slash, sparse GQA decode."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("minference", "blocksparse_attention"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import tilelang  # noqa: E402


def _vs_inputs(B, H, S, device, nv, slashes):
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(B, H, S, 64, generator=g).half().to(device) for _ in range(3))
    v_idx = torch.stack([torch.randperm(S, generator=g)[:nv] for _ in range(B * H)]).view(B, H, -1).to(device)
    s_idx = torch.tensor(slashes).view(1, H, -1).expand(B, H, -1).contiguous().to(device)
    return q, k, v, v_idx, s_idx


@pytest.mark.parametrize("num_split", [1, 3])
def test_vertical_slash_cpu(num_split):
    """num_split 3: each query block's key work over three workgroups + the LSE combine (some
    splits of the short blocks are empty: weight 0)."""
    from example_vertical_slash_sparse_attn import ref_program, vs_sparse_flashattn, convert_vertical_slash_indexes
    q, k, v, v_idx, s_idx = _vs_inputs(1, 2, 512, "cpu", 40, [[0, 300], [0, 100]])
    bc, bo, cc, ci = convert_vertical_slash_indexes(v_idx, s_idx, 512, 64, 32)
    assert int(cc.sum()) > 0 and int(bc.sum()) > 0  # both phases exercised
    f = vs_sparse_flashattn.get_tir(1, 2, 512, 64, bo.shape[-1], ci.shape[-1], 64, 32, 128, num_split=num_split)
    kern = tilelang.compile(f, out_idx=[-1], target="cpu", pass_configs={"tl.enable_fast_math": True})
    extra = () if num_split == 1 else (torch.empty(1, 2, num_split, 512, 64), torch.empty(1, 2, num_split, 512))
    o = kern(q, k, v, bc, bo, cc, ci, *extra)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, v_idx, s_idx, 64, 32), rtol=2e-2, atol=2e-2)


def _check_convert(device):
    from example_vertical_slash_sparse_attn import convert_vertical_slash_indexes, convert_vertical_slash_indexes_torch
    cases = ((512, 40, [[0, 300], [0, 100]], 64, 32), (1024, 100, [[0, 7, 300], [0, 64, 513]], 64, 64))
    for S, nv, slashes, bm, bn in cases:
        _, _, _, v_idx, s_idx = _vs_inputs(1, 2, S, device, nv, slashes)
        bc, bo, cc, ci = convert_vertical_slash_indexes(v_idx, s_idx, S, bm, bn, merged=False)
        rbc, rbo, rcc, rci = convert_vertical_slash_indexes_torch(v_idx, s_idx, S, bm, bn)
        assert torch.equal(bc.cpu(), rbc.cpu()) and torch.equal(cc.cpu(), rcc.cpu())
        for h in range(2):
            for qb in range(bc.shape[2]):
                n, c = int(bc[0, h, qb]), int(cc[0, h, qb])
                assert bo[0, h, qb, :n].tolist() == rbo[0, h, qb, :n].tolist()  # ascending in both
                assert sorted(ci[0, h, qb, :c].tolist()) == rci[0, h, qb, :c].tolist()  # input order vs sorted
                assert (bo[0, h, qb, n:] == -1).all() and (ci[0, h, qb, c:] == -1).all()


def _check_convert_merged(device):
    from example_vertical_slash_sparse_attn import convert_vertical_slash_indexes, convert_vertical_slash_merged_py
    g = torch.Generator().manual_seed(3)
    for S, nv, ns, bm, bn in ((512, 40, 6, 64, 32), (2048, 200, 60, 128, 64), (1000, 50, 9, 128, 128)):
        v_idx = torch.stack([torch.randperm(S, generator=g)[:nv] for _ in range(2)]).view(1, 2, -1).int().to(device)
        s_idx = torch.stack([torch.randperm(S, generator=g)[:ns] for _ in range(2)]).view(1, 2, -1).int()
        s_idx[..., 0] = 0
        s_idx = s_idx.to(device)
        bc, bo, cc, ci = convert_vertical_slash_indexes(v_idx, s_idx, S, bm, bn, merged=True)
        for b, h, qb, offs, cols in convert_vertical_slash_merged_py(v_idx.cpu(), s_idx.cpu(), S, bm, bn):
            n, c = int(bc[b, h, qb]), int(cc[b, h, qb])
            assert bo[b, h, qb, :n].tolist() == offs
            assert sorted(ci[b, h, qb, :c].tolist()) == sorted(cols)


def test_vertical_slash_merged_attention_cpu():
    """The attention kernel over merged unaligned segments (dense tiles at arbitrary key offsets)."""
    from example_vertical_slash_sparse_attn import ref_program, vs_sparse_flashattn, convert_vertical_slash_indexes
    q, k, v, v_idx, s_idx = _vs_inputs(1, 2, 512, "cpu", 40, [[0, 300, 37], [0, 100, 7]])
    bc, bo, cc, ci = convert_vertical_slash_indexes(v_idx, s_idx, 512, 64, 32, merged=True)
    f = vs_sparse_flashattn.get_tir(1, 2, 512, 64, bo.shape[-1], ci.shape[-1], 64, 32, 128, num_split=2)
    kern = tilelang.compile(f, out_idx=[-1], target="cpu", pass_configs={"tl.enable_fast_math": True})
    o = kern(q, k, v, bc, bo, cc, ci, torch.empty(1, 2, 2, 512, 64), torch.empty(1, 2, 2, 512))
    torch.testing.assert_close(o.float(), ref_program(q, k, v, v_idx, s_idx, 64, 32, merged=True), rtol=2e-2,
                               atol=2e-2)


def test_vertical_slash_convert_merged_cpu():
    """Merged unaligned slash segments (the default conversion) against its Python definition."""
    _check_convert_merged("cpu")


@pytest.mark.gpu
def test_vertical_slash_convert_merged_gpu():
    _check_convert_merged("cuda")


def test_vertical_slash_convert_cpu():
    """The device index conversion (vs_convert) selects exactly the blocks / columns of the
    vectorised-PyTorch form."""
    _check_convert("cpu")


@pytest.mark.gpu
def test_vertical_slash_convert_gpu():
    _check_convert("cuda")


@pytest.mark.gpu
def test_vertical_slash_gpu():
    from example_vertical_slash_sparse_attn import ref_program, vertical_slash_sparse_attention
    q, k, v, v_idx, s_idx = _vs_inputs(2, 2, 1024, "cuda", 100, [[0, 7, 300], [0, 64, 513]])
    for bm, bn, th, ns in ((64, 64, 256, 1), (128, 128, 512, None), (128, 64, 512, 1), (128, 64, 512, 4)):
        o = vertical_slash_sparse_attention(q, k, v, v_idx, s_idx, bm, bn, th, num_split=ns)
        torch.testing.assert_close(o.float(), ref_program(q, k, v, v_idx, s_idx, bm, bn), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("variant", ["varlen_indice", "varlen_mask", "paged"])
def test_sparse_gqa_decode_cpu(variant):
    import importlib
    m = importlib.import_module(f"example_tilelang_sparse_gqa_decode_{variant}")
    m.run(batch=2, heads=32, heads_kv=2, max_cache_seqlen=256, dim=64, block_size=32, sparse_ratio=0.5, device="cpu",
          num_split=2)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["varlen_indice", "varlen_mask", "paged"])
def test_sparse_gqa_decode_gpu(variant):
    import importlib
    m = importlib.import_module(f"example_tilelang_sparse_gqa_decode_{variant}")
    m.run(batch=4, heads=32, heads_kv=4, max_cache_seqlen=2048, dim=128, block_size=32, sparse_ratio=0.7,
          device="cuda", num_split=4)
