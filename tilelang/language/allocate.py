"""Buffer allocation: ``T.alloc_shared/fragment/local/var/reducer`` and ``T.empty``.

Reference: ``tilelang/language/allocate.py:37-291``.  Scope strings are kept
compatible (``shared.dyn``, ``local.fragment``, ``local.var``).  On gfx950 every
shared buffer lives in ONE LDS arena (see ``transform/lds_plan.py``), which is what
keeps hipcc's counted ``vmcnt`` waits intact around LDS-DMA.
"""
from __future__ import annotations

from ..ir import stmt as S
from ..ir.buffer import Buffer
from ..ir.expr import IntImm, PrimExpr, convert
from ..ir import dtypes as _dt
from .builder import current_builder


def _alloc(shape, dtype, scope, name=None):
    if isinstance(shape, (int, )) or hasattr(shape, "dtype") and not isinstance(shape, (list, tuple)):
        shape = [shape]
    b = current_builder()
    auto = name is None
    buf = Buffer(b.fresh(name or {"shared": "shared", "fragment": "frag", "local": "local",
                                  "var": "var"}[_scope_key(scope)]), list(shape), dtype, scope)
    buf._auto_name = auto
    b.emit(S.AllocStmt(buf))
    return buf


def _scope_key(scope):
    if scope.startswith("shared"):
        return "shared"
    if scope in ("local.fragment", "fragment"):
        return "fragment"
    if scope in ("local.var", "var"):
        return "var"
    return "local"


def alloc_shared(shape, dtype, scope: str = "shared.dyn"):
    return _alloc(shape, dtype, "shared")


def alloc_fragment(shape, dtype, scope: str = "local.fragment"):
    return _alloc(shape, dtype, "fragment")


def alloc_local(shape, dtype, scope: str = "local"):
    return _alloc(shape, dtype, "local")


def alloc_var(dtype="int32", *args, init=None, scope: str = "local.var"):
    # reference signature alloc_var(dtype, [init], scope=...)
    if args:
        if isinstance(args[0], str) and args[0].startswith("local"):
            scope = args[0]
        else:
            init = args[0]
    buf = _alloc([1], dtype, "var")
    if init is not None:
        buf.init_value = convert(init)
        current_builder().store(buf, [IntImm(0)], init)
    return buf


def alloc_buffer(shape, dtype, scope: str = "global"):
    return _alloc(shape, dtype, scope)


def alloc_reducer(shape, dtype, op: str = "sum", replication=None):
    """A fragment whose replicas are combined by ``T.finalize_reducer`` (reference allocate.py:201)."""
    buf = _alloc(shape, dtype, "fragment")
    buf.reducer_op = op
    buf.reducer_replication = replication
    return buf


def alloc_barrier(arrive_count):
    raise NotImplementedError("mbarriers are NVIDIA-only; gfx950 synchronises with s_barrier (T.sync_threads)")


def alloc_tmem(*args, **kwargs):
    raise NotImplementedError("TMEM is Blackwell-only; on gfx950 accumulators live in AGPRs (T.alloc_fragment)")


def alloc_descriptor(*args, **kwargs):
    raise NotImplementedError("wgmma/tcgen05 descriptors are NVIDIA-only")


alloc_wgmma_desc = alloc_descriptor
alloc_tcgen05_smem_desc = alloc_descriptor
alloc_tcgen05_instr_desc = alloc_descriptor


class EmptyTensor:
    """``T.empty(shape, dtype)``: an output tensor allocated by the launcher (lazy_jit)."""

    def __init__(self, shape, dtype):
        self.shape = list(shape)
        self.dtype = _dt.as_dtype(dtype)


def empty(*shape, dtype="float32"):
    """``T.empty(M, N, dtype=...)`` / ``T.empty((M, N), dtype)``: inside a ``@tilelang.lazy_jit``
    body, an output tensor the launcher allocates and the call returns."""
    if len(shape) == 2 and isinstance(shape[0], (list, tuple)) and not isinstance(shape[1], (int, PrimExpr)):
        shape, dtype = shape[0], shape[1]
    elif len(shape) == 1 and isinstance(shape[0], (list, tuple)):
        shape = shape[0]
    shape = list(shape)
    from .annot import LAZY_STACK
    if LAZY_STACK:
        b = Buffer("out", shape, dtype, "global")
        b._auto_name = True
        LAZY_STACK[-1].outputs.append(b)
        return b
    return EmptyTensor(shape, dtype)
