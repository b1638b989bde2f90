"""Parity of the mesh routing schedule with the reference lowering tests
(``testing/python/language/test_tilelang_language_comm.py``: 4x4 mesh, 128x128 fp32 tiles),
plus the direct xGMI transfer sets this framework executes instead."""
import pytest

import tilelang.language as T
from tilelang.ir import stmt as S
from tilelang.ir import tileop as O
from tilelang.parallel import device_mesh_config
from tilelang.parallel.comm_plan import reference_schedule, transfer_bytes, xgmi_transfers


def _ops(func):
    return [s.op for s in S.walk(func.body) if isinstance(s, S.TileOpStmt) and isinstance(s.op, O.CommOp)]


def _trace(body_fn, *shapes):
    with device_mesh_config(4, 4):

        @T.prim_func
        def main(A: T.Tensor((1024, 1024), "float16")):
            with T.Kernel(8, 8, threads=128) as (bx, by):
                A_local = T.alloc_fragment([128, 128], "float")
                bufs = [T.alloc_fragment(s, "float") for s in shapes]
                T.copy(A[by * 128, bx * 128], A_local)
                body_fn(A_local, *bufs)

        return _ops(main)


def test_broadcast_all_schedule():
    (op,) = _trace(lambda a, b: T.comm.broadcast(a, b, (1, 2), direction="all"), [128, 128])
    sched = [(b.core, b.direction, b.size) for b in reference_schedule(op, 4, 4)]
    # reference: broadcast_(A, B, 16384, 6, 1) then broadcast_(B, B, 16384, {2,6,10,14}, 0)
    assert sched == [(6, 1, 16384), (2, 0, 16384), (6, 0, 16384), (10, 0, 16384), (14, 0, 16384)]
    xs = xgmi_transfers(op, 4, 4)
    assert sorted(t.dst for t in xs) == list(range(16)) and all(t.src == 6 for t in xs)


def test_put_schedule_keeps_reference_two_hop_quirk():
    (op,) = _trace(lambda a, b: T.comm.put(a, b, (1, 2), (2, 3)), [128, 128])
    sched = [(b.core, b.direction, b.size, tuple(b.mask)) for b in reference_schedule(op, 4, 4)]
    # reference: broadcast_(..., 16384, 6, 1, 0, 1, 3) ; broadcast_(..., 16384, 7, 0, 0, 1, 2)
    assert sched == [(6, 1, 16384, (0, 1, 3)), (7, 0, 16384, (0, 1, 2))]
    # executed on xGMI: one direct hop
    (t,) = xgmi_transfers(op, 4, 4)
    assert (t.src, t.dst, t.elements) == (6, 11, 16384)


def test_all_gather_all_schedule():
    (op,) = _trace(lambda a, c: T.comm.all_gather(a, c, direction="all"), [16, 128, 128])
    sched = reference_schedule(op, 4, 4)
    h = [(b.core, b.dst_offset, b.size, b.direction) for b in sched[:16]]
    assert h == [(k, k * 16384, 16384, 0) for k in range(16)]
    v = [(b.core, b.src_offset, b.size, b.direction) for b in sched[16:]]
    assert v == [(i * 4 + j, i * 65536, 65536, 1) for j in range(4) for i in range(4)]
    xs = xgmi_transfers(op, 4, 4)
    assert len(xs) == 256
    remote, local = transfer_bytes(op, 4, 4, 4)
    assert remote == 240 * 16384 * 4 and local == 16 * 16384 * 4


def test_all_reduce_schedule():
    with device_mesh_config(4, 4):

        @T.prim_func
        def main(A: T.Tensor((131072, 131072), "float16")):
            with T.Kernel(128, 128, threads=128) as (bx, by):
                A_local = T.alloc_fragment([1024, 1024], "float")
                E_local = T.alloc_fragment([1024], "float")
                T.copy(A[by * 1024, bx * 1024], A_local)
                T.comm.all_reduce(A_local, E_local, "sum", "all", dim=-1, clear=False)

        (op,) = _ops(main)
    sched = reference_schedule(op, 4, 4)
    row = [(b.core, b.dst_offset, b.size, b.direction) for b in sched[:16]]
    assert row == [(i * 4 + j, j * 1024, 1024, 0) for i in range(4) for j in range(4)]
    col = [(b.core, b.dst_offset, b.size, b.direction) for b in sched[16:]]
    assert col == [(i * 4 + j, i * 1024, 1024, 1) for j in range(4) for i in range(4)]
    assert op.tmp is not None and list(op.tmp.buffer.shape) == [1024]


def test_comm_api_validation():
    with device_mesh_config(4, 4):
        with pytest.raises(AssertionError, match="Receive buffer shape"):

            @T.prim_func
            def bad(A: T.Tensor((128, 128), "float32")):
                with T.Kernel(1, threads=128) as bx:
                    a = T.alloc_fragment([128, 128], "float")
                    c = T.alloc_fragment([8, 128, 128], "float")
                    T.comm.all_gather(a, c, direction="all")

        with pytest.raises(AssertionError, match="out of bounds"):

            @T.prim_func
            def bad2(A: T.Tensor((128, 128), "float32")):
                with T.Kernel(1, threads=128) as bx:
                    a = T.alloc_fragment([128, 128], "float")
                    b = T.alloc_fragment([128, 128], "float")
                    T.comm.broadcast(a, b, (4, 0))

        with pytest.raises(ValueError, match="Invalid reduce output shape"):

            @T.prim_func
            def bad3(A: T.Tensor((128, 128), "float32")):
                with T.Kernel(1, threads=128) as bx:
                    a = T.alloc_fragment([128, 128], "float")
                    b = T.alloc_fragment([64], "float")
                    T.comm.all_reduce(a, b, "sum")

        with pytest.raises(AssertionError, match="Reduction op"):

            @T.prim_func
            def bad4(A: T.Tensor((128, 128), "float32")):
                with T.Kernel(1, threads=128) as bx:
                    a = T.alloc_fragment([128, 128], "float")
                    b = T.alloc_fragment([128], "float")
                    T.comm.all_reduce(a, b, "prod")


def test_core_id_helpers():
    with device_mesh_config(4, 4):
        assert T.comm.CoreId((1, 2)).value == 6
        assert T.comm.CoreId(11).value == 11
        assert T.comm.core_id_to_tuple(7) == (1, 3)
        with pytest.raises(AssertionError):
            T.comm.CoreId(16)
    with device_mesh_config(2, 4):
        assert T.comm.core_tuple_to_id((1, 3)) == 7
