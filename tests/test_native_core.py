"""The native compiler core (tilelang._tl_core, csrc/core) against its Python specifications."""
import random

import pytest

from tilelang import _native
from tilelang.analysis import lds_bank
from tilelang.layout import mfma as MF
from tilelang.layout.fragment import Digit, Fragment, make_linear_fragment
from tilelang.layout.hierarchical_layout import make_blockwise_zz_layout, make_hierarchical_layout

core = _native.core()


def _py_inverse(f: Fragment, t, r):
    # executable spec: Fragment.inverse with Python ints
    return tuple(int(x) for x in f.inverse(t, r))


@pytest.mark.parametrize("frag", [
    MF.mfma_c_fragment(128, 128, 2, 2),
    MF.mfma_a_fragment(64, 64, 4, 1, 1),
    make_linear_fragment([32, 256], 256, 4),
    make_linear_fragment([4, 512], 256, 4).replicate(2),
])
def test_fragment_inverse_and_table_match_python(frag):
    nf = frag.native
    nd = len(frag.shape)
    tab = nf.table()
    for t in range(0, frag.num_threads, 7):
        for r in range(frag.local_size):
            assert nf.inverse(t, r) == _py_inverse(frag, t, r)
            o = (t * frag.local_size + r) * nd
            assert tuple(tab[o:o + nd]) == _py_inverse(frag, t, r)
    t = frag.num_threads - 1
    assert nf.thread_local_map(t) == {_py_inverse(frag, t, r): r for r in range(frag.local_size)}


def test_fragment_equality_is_numeric():
    a = Fragment([16, 16], [Digit(0, 1, 16), Digit(1, 4, 4)], [Digit(1, 1, 4)])
    b = Fragment([16, 16], [Digit(0, 1, 16), Digit(1, 8, 2), Digit(1, 4, 2)], [Digit(1, 1, 4)])
    c = Fragment([16, 16], [Digit(1, 4, 4), Digit(0, 1, 16)], [Digit(1, 1, 4)])
    assert a.native.equals(b.native) and a.is_equal(b)
    assert not a.native.equals(c.native)


def test_fragment_rejects_non_tiling_digits():
    with pytest.raises(ValueError, match="do not tile"):
        core.Fragment([16], [(0, 2, 8)], [(0, 1, 4)])


def test_resolve_affine_ownership_and_uniformity():
    loop = make_linear_fragment([8, 128], 256, 4)
    row = Fragment([8], [Digit(-1, 1, 32), Digit(0, 1, 8)], [])  # row = t % 8: wrong owners
    from tilelang.transform.layout_inference import project_layout
    proj = project_layout(loop, [0], [8])  # the projection every thread of the nest owns
    for r in range(loop.local_size):
        assert loop.native.resolve_affine(proj.native, [1, 0], [0], r) >= 0
    assert any(loop.native.resolve_affine(row.native, [1, 0], [0], r) == -1 for r in range(loop.local_size))
    # a transposed access of a 2-D buffer laid out like the loop is not uniform
    sq = make_linear_fragment([64, 64], 256, 4)
    res = {sq.native.resolve_affine(sq.native, [0, 1, 1, 0], [0, 0], r) for r in range(sq.local_size)}
    assert res & {-1, -2}


def test_lds_cycles_native_matches_python_model():
    rng = random.Random(0)
    for instr in lds_bank.INSTRUCTIONS:
        width = lds_bank.INSTRUCTIONS[instr][1]
        for _ in range(20):
            addrs = [rng.randrange(0, 65536 // width) * width for _ in range(64)]
            assert lds_bank.instruction_cycles(instr, addrs) == lds_bank.instruction_cycles_py(instr, addrs)
    # conflict-free ds_read_b128 of 64 consecutive 16-byte chunks costs one cycle per lane group
    assert lds_bank.instruction_cycles("ds_read_b128", [16 * i for i in range(64)]) == 4


def test_swizzle_search_removes_transposed_read_conflicts():
    bits = MF.choose_swizzle("tr", 64, 128, 2)
    rep = MF.swizzle_report("tr", 64, 128, 2, bits)
    assert rep["cycles"] <= rep["cycles_unswizzled"]
    assert rep["cycles"] == rep["conflict_free"]


def test_arena_planner():
    offs, total = core.plan_arena([1000, 4096, 10], [0, 0, 1], [0, 1, 1], 16, False, 163840)
    assert total == 1008 + 4096 + 16 and sorted(offs) == [0, 4096, 4096 + 1008]
    offs, total = core.plan_arena([4096, 4096], [0, 1], [0, 1], 16, True, 163840)
    assert total == 4096 and offs == [0, 0]
    with pytest.raises(ValueError, match="bytes of LDS"):
        core.plan_arena([200000], [0], [0], 16, False, 163840)


def test_hierarchical_native_offsets():
    zz = make_blockwise_zz_layout((64, 96), (32, 32))
    assert zz.is_bijective()
    offs = zz.offsets()
    for i, j in [(0, 0), (5, 40), (33, 1), (63, 95)]:
        assert offs[i * 96 + j] == zz.offset([i, j]) == (i // 32) * 32 * 96 + (j // 32) * 1024 + (i % 32) * 32 + j % 32
        assert zz.offset_to_logical(zz.offset([i, j])) == [i, j]
    h = make_hierarchical_layout([2, 4, 8], [32, 1, 4], [(0, 2), (2, 3)])
    assert h.offset([5, 3]) == 1 * 32 + 1 * 1 + 3 * 4
    with pytest.raises(ValueError, match="partition"):
        make_hierarchical_layout([2, 4], [4, 1], [(0, 1), (0, 1)])
    assert core.shard_hier([8, 32, 4, 32], [(0, 2), (2, 4)], 0, 4) == [2, 32, 4, 32]


def test_runtime_package_surface():
    import tilelang.runtime as R
    assert R.available() in (True, False)
    for name in ("device_info", "Workspace", "can_access_peer", "NativeRuntimeMissing"):
        assert hasattr(R, name)
