"""Builtins: synchronisation, wave (64-lane) intrinsics, debug printing, annotations.

Reference: ``tilelang/language/builtin.py`` (shuffles ``:633-675``, syncs ``:676-701``),
``print.py`` (``T.print`` / ``T.device_assert``), ``annotations.py``
(``use_swizzle``, ``annotate_layout``, ``annotate_safe_value``, ``annotate_l2_hit_ratio``).
NVIDIA-only builtins (TMA, mbarrier, wgmma, tcgen05) are intentionally absent.
"""
from __future__ import annotations

from ..ir import stmt as S
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import Var, call, convert, StringImm, IntImm
from ..ir import dtypes as _dt
from .builder import current_builder


def _eval(e):
    current_builder().emit(S.EvaluateStmt(e))


def sync_threads(barrier_id=None, arrive_count=None):
    _eval(call("tl.sync_threads", [], _dt.void))


def sync_warp(mask=None):
    _eval(call("tl.sync_warp", [], _dt.void))


def set_priority(level: int):
    """Wave issue priority (``s_setprio``, 0..3) for the rest of the wave's stream.  On CDNA4 the
    two waves of a SIMD arbitrate VALU issue by priority, then age: raising the younger half of
    an 8-wave workgroup once before the main loop (``if wave >= 4: T.set_priority(1)``) removes
    its start-of-segment penalty (MI355X microarchitecture notes, 'Two waves per SIMD', item 4).
    A no-op on the CPU target."""
    level = int(level)
    if not 0 <= level <= 3:
        raise ValueError(f"T.set_priority: level must be 0..3, got {level}")
    _eval(call("tl.setprio", [IntImm(level)], _dt.void))


def sync_global():
    _eval(call("tl.sync_grid", [], _dt.void))


sync_grid = sync_global


def fence_proxy_async(*args, **kwargs):
    """No-op on gfx950 (no async proxy)."""
    return None


def memory_fence(scope="agent"):
    _eval(call("tl.fence", [StringImm(scope)], _dt.void))


def _tid():
    from .kernel import get_thread_binding
    return get_thread_binding(0)


def get_lane_idx(warp_size=None):
    """Lane within a wave (64 on gfx950); with ``warp_size``, within groups of that many threads
    (the reference's argument: 32 gives CUDA-warp numbering)."""
    if warp_size is None or int(warp_size) == 64:
        return call("tl.lane_id", [], _dt.int32)
    return _tid() % int(warp_size)


def get_warp_idx(warp_size=None):
    if warp_size is None or int(warp_size) == 64:
        return call("tl.wave_id", [], _dt.int32)
    return _tid() // int(warp_size)


def get_warp_idx_sync(warp_size=None):
    return get_warp_idx(warp_size)


def get_warp_group_idx(warp_size=None, warps_per_group=None):
    """Warp group = ``warps_per_group`` (default 4) consecutive waves."""
    wpg = 4 if warps_per_group is None else int(warps_per_group)
    if warp_size is None or int(warp_size) == 64:
        return call("tl.wave_id", [], _dt.int32) // wpg
    return _tid() // (int(warp_size) * wpg)


def shfl_xor(value, offset, width=64):
    value = convert(value)
    return call("tl.shfl_xor", [value, convert(offset), convert(width)], value.dtype)


def shfl_down(value, offset, width=64):
    value = convert(value)
    return call("tl.shfl_down", [value, convert(offset), convert(width)], value.dtype)


def shfl_up(value, offset, width=64):
    value = convert(value)
    return call("tl.shfl_up", [value, convert(offset), convert(width)], value.dtype)


def shfl_sync(value, src_lane, width=64):
    value = convert(value)
    return call("tl.shfl", [value, convert(src_lane), convert(width)], value.dtype)


def ballot(pred):
    return call("tl.ballot", [convert(pred)], _dt.uint64)


def clock():
    return call("tl.clock", [], _dt.int64)


def call_extern(dtype, func_name, *args):
    return call("extern", [StringImm(func_name)] + [convert(a) for a in args], dtype)


def call_intrin(dtype, func_name, *args):
    return call_extern(dtype, func_name, *args)


def evaluate(expr):
    _eval(expr)


def loop_break():
    current_builder().emit(S.BreakStmt())


def device_assert(cond, msg: str = ""):
    current_builder().emit(S.AssertStmt(convert(cond), msg))


def print(obj=None, msg: str = "", warp_group_id: int = 0, warp_id: int = 0):  # noqa: A001
    """Device printf of a scalar or a whole buffer (reference ``language/print.py:144``)."""
    if isinstance(obj, (Buffer, BufferRegion)):
        buf = obj.buffer if isinstance(obj, BufferRegion) else obj
        _eval(call("tl.print_buffer", [StringImm(msg), StringImm(buf.name), buf.data], _dt.void, buffer=buf))
    else:
        _eval(call("tl.print", [StringImm(msg), convert(obj)], _dt.void))


def use_swizzle(panel_size: int = 8, order: str = "row", enable: bool = True):
    """Block rasterisation for L2 reuse.  On MI355X this also remaps block ids so that each
    XCD (private 4 MiB L2) receives a contiguous chunk of tiles (guide T1)."""
    if not enable:
        return None
    current_builder().attrs["use_swizzle"] = {"panel_size": int(panel_size), "order": order}
    return None


def annotate_layout(layout_map: dict):
    for buf, layout in layout_map.items():
        if layout is None:  # e.g. make_metadata_layout of a global tensor: nothing to annotate
            continue
        buf.layout = layout
        buf.layout_annotated = True


def annotate_safe_value(safe_value_map: dict):
    for buf, v in safe_value_map.items():
        buf.safe_value = convert(v)


def annotate_l2_hit_ratio(*args, **kwargs):
    """CUDA L2 access-policy window; the MI355X L2 has no equivalent knob (no-op)."""
    return None


def annotate_padding(*args, **kwargs):
    return None


def annotate_nontemporal(*buffers):
    """gfx950 addition: the global ``buffers`` are streamed once -- every vector access to them is
    non-temporal (``global_load/store ... nt``), as ``T.copy(..., eviction_policy="evict_first")``
    does for a copy's global side.  For element loops that read or write global memory directly."""
    for b in buffers:
        buf = b.buffer if hasattr(b, "buffer") else b
        if buf.scope != "global":
            raise ValueError(f"T.annotate_nontemporal: {buf.name} is not a global tensor")
        buf.nontemporal = True
        current_builder().emit(S.AttrStmt("tl.nontemporal", buf.name))


def attr(node, key, value):
    current_builder().emit(S.AttrStmt(key, value))


def block_attr(attrs: dict):
    for k, v in attrs.items():
        current_builder().attrs[k] = v


def import_source(source=None):
    if source is not None:
        current_builder().attrs.setdefault("import_source", []).append(source)


def no_set_max_nreg():
    return None


def set_max_nreg(*args):
    return None


def disable_warp_group_reg_alloc():
    return None


def assume(cond):
    current_builder().emit(S.AttrStmt("assume", convert(cond)))


def address_of(load):
    return call("tl.address_of", [load], _dt.handle)


def tvm_mfma(*args, **kwargs):
    raise NotImplementedError("use T.gemm; MFMA fragments are scheduled by the compiler")


def dynamic(name: str, dtype="int32"):
    """A symbolic (dynamic) shape variable, bound from tensor shapes at call time."""
    return Var(name, _dt.as_dtype(dtype), nonneg=True)


symbolic = dynamic
