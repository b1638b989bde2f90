import itertools

import pytest

from tilelang.layout import (mfma_c_fragment, mfma_a_fragment, make_linear_fragment, SwizzleLayout,
                             choose_swizzle, swizzle_report, compute_warp_partition, make_hierarchical_layout,
                             make_blockwise_zz_layout, Fragment)
from tilelang.transform.layout_inference import reduce_dst_layout


def _check_bijective(f):
    seen = {}
    for t in range(f.num_threads):
        for r in range(f.local_size):
            idx = tuple(f.inverse(t, r))
            assert f.forward_index(*idx) == r
            seen.setdefault(idx, []).append(t)
    n = 1
    for s in f.shape:
        n *= s
    assert len(seen) == n
    assert all(len(v) == f.replicate_size for v in seen.values())


@pytest.mark.parametrize("M,N,wm,wn", [(128, 128, 2, 2), (64, 128, 4, 1), (256, 256, 2, 4), (32, 64, 1, 4)])
def test_mfma_c_layout_matches_cdna4_formula(M, N, wm, wn):
    f = mfma_c_fragment(M, N, wm, wn)
    _check_bijective(f)
    WM, WN = M // wm, N // wn
    n_rep = WN // 16
    for t in range(0, f.num_threads, 7):
        w, lane = t // 64, t % 64
        wy, wx = w // wn, w % wn
        for r in range(f.local_size):
            mi, rest = divmod(r, n_rep * 4)
            ni, v = divmod(rest, 4)
            # swapped-operand CDNA4 16x16x32: lane holds C[m=lane&15][n=4*(lane>>4)+v]
            exp = [wy * WM + mi * 16 + (lane & 15), wx * WN + ni * 16 + 4 * (lane >> 4) + v]
            assert f.inverse(t, r) == exp


def test_accumulator_is_kperm_a_operand():
    c = mfma_c_fragment(128, 64, 4, 1)
    a = mfma_a_fragment(128, 64, 4, 1, kperm=1)
    assert c.is_equal(a)
    a0 = mfma_a_fragment(128, 64, 4, 1, kperm=0)
    assert not c.is_equal(a0)
    _check_bijective(a0)


def test_reduce_layout_is_row_projection():
    c = mfma_c_fragment(128, 64, 4, 1)
    r = reduce_dst_layout(c, 1, [128])
    assert r.shape == [128]
    for t in range(256):
        rows_c = {tuple(c.inverse(t, i))[0] for i in range(c.local_size)}
        rows_r = {r.inverse(t, i)[0] for i in range(r.local_size)}
        assert rows_c == rows_r


def test_linear_fragment_and_replication():
    f = make_linear_fragment([64, 64], 256, 8)
    _check_bijective(f)
    assert f.inner_vector_width() == 8
    g = make_linear_fragment([8], 256, 1)
    assert g.replicate_size == 32
    _check_bijective(g)


def test_warp_partition_policies():
    assert compute_warp_partition(128, 128, 4, 0) == (2, 2)
    assert compute_warp_partition(128, 128, 4, 1) == (4, 1)
    assert compute_warp_partition(128, 128, 4, 2) == (1, 4)
    with pytest.raises(ValueError):
        compute_warp_partition(16, 16, 8, 1)


def test_swizzle_is_involution_and_conflict_free_in_model():
    for kind, rows, cols in [("k_rows", 128, 32), ("k_rows", 128, 64), ("tr", 32, 128), ("tr_kperm", 64, 128)]:
        bits = choose_swizzle(kind, rows, cols, 2)
        lay = SwizzleLayout([rows, cols], 2, list(bits))
        seen = set()
        for r, c in itertools.product(range(rows), range(cols)):
            off = lay.forward(r, c)[0]
            assert lay.inverse(off) == [r, c]
            seen.add(off)
        assert len(seen) == rows * cols
        rep = swizzle_report(kind, rows, cols, 2, bits)
        assert rep["cycles"] == rep["conflict_free"], rep
        assert rep["cycles_unswizzled"] > rep["cycles"]


def test_hierarchical_layout_roundtrip():
    hl = make_hierarchical_layout((2, 4, 16, 2, 4, 16), (8192, 1024, 16, 4096, 256, 1), ((0, 3), (3, 6)))
    assert hl.logical_shape == (128, 128)
    seen = set()
    for i in range(0, 128, 3):
        for j in range(0, 128, 5):
            off = hl.offset([i, j])
            assert hl.offset_to_logical(off) == [i, j]
            seen.add(off)
    zz = make_blockwise_zz_layout((64, 96), (32, 32))
    assert zz.offset([0, 32]) == 32 * 32
    assert zz.offset([1, 0]) == 32
    assert zz.offset([32, 0]) == 32 * 96


def test_reference_style_fragment_constructor():
    # thread = i % 16 + 16 * (j // 4), local = j % 4 (a 16x16 MFMA-like tile over 64 lanes)
    f = Fragment([16, 16], forward_thread_fn=lambda i, j: i % 16 + 16 * (j // 4),
                 forward_index_fn=lambda i, j: j % 4, num_threads=64)
    assert f.num_threads == 64 and f.local_size == 4
    assert f.forward_thread(3, 9) == 3 + 32
