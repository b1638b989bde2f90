"""Kernel-argument annotations: ``T.Tensor``, ``T.StridedTensor``, ``T.dyn`` and the Mesh extensions.

Reference: ``tilelang/language/v2/annot.py``.  ``T.MeshTensor`` (fork addition,
``annot.py:518-714``) annotates a *global* tensor that is sharded over a
``nrows x ncols`` device mesh; the kernel sees the per-device shard and the
PrimFunc records global/sharded metadata in its ``tensor_meta`` attribute.
On MI355X a mesh "core" is one GPU of the node (up to 8, see
``tilelang/parallel/mesh.py``).

Sharding rules (kept identical so programs are portable):
  * ``x`` splits a dim by ``ncols``; ``y`` splits a dim by ``nrows`` (ceil);
  * ``cross_mesh_dim`` splits one dim by ``nrows*ncols``;
  * ``replicate`` in {NONE, ROW, COLUMN, ALL}; ROW forbids an x split, COLUMN a y split;
  * hierarchical layouts shard the most significant hierarchical dim of the group.
"""
from __future__ import annotations

import threading

import math
from enum import Enum
from typing import Any, Optional, Tuple

from ..ir import dtypes as _dt
from ..ir.buffer import Buffer
from ..ir.expr import PrimExpr, Var
from .parser import TensorAnnot, ScalarAnnot


def _row_major_strides(shape) -> Tuple:
    strides = []
    acc = 1
    for s in reversed(list(shape)):
        strides.append(acc)
        acc = acc * s
    return tuple(reversed(strides))


class _TensorFactory:
    """``T.Tensor(shape, dtype)`` and ``T.Tensor[shape, dtype]``."""

    def __init__(self, scope="global"):
        self.scope = scope

    def __call__(self, shape, dtype="float32", data=None, strides=None, elem_offset=None, scope=None,
                 align=0, offset_factor=0, buffer_type="", axis_separators=None):
        if data is not None:
            # inside a kernel: a new view of an existing buffer's storage, e.g.
            # T.Tensor((KH * KW * C, F), dtype, kernel.data)
            from ..ir.buffer import DATA_OWNERS
            owner = data if isinstance(data, Buffer) else DATA_OWNERS.get(getattr(data, "uid", None))
            if owner is None:
                raise ValueError("T.Tensor(..., data=...) needs the .data of a buffer")
            from .tileops import view
            return view(owner, shape, dtype)
        return TensorAnnot(shape, dtype, strides=strides, scope=scope or self.scope)

    def __getitem__(self, key):
        if not isinstance(key, tuple) or len(key) != 2:
            raise TypeError("T.Tensor[shape, dtype]")
        shape, dtype = key
        if _is_template(shape, None, dtype):
            return TensorTemplate(shape, dtype)
        return TensorAnnot(shape, dtype, scope=self.scope)


def _is_concrete_dim(d):
    return isinstance(d, (int, PrimExpr)) and not isinstance(d, bool)


def _is_template(shape, strides, dtype):
    if isinstance(shape, (int, PrimExpr)):
        shape = [shape]
    dims = list(shape) + list(strides or [])
    return any(not _is_concrete_dim(d) for d in dims) or dtype is Any or dtype is None


class TensorTemplate:
    """A ``@tilelang.lazy_jit`` parameter annotation specialised from the call-site tensor
    (reference ``tilelang/language/v2/annot.py``): each dim / stride is

      * ``int``            -> static, taken from the argument (one compiled kernel per value);
      * a Python int       -> static, must match;
      * ``T.dyn`` / ``T.dyn['name']`` -> a runtime symbol (one kernel for every value; named
        symbols are shared between parameters);

    and the dtype is fixed or ``Any`` (taken from the argument)."""

    def __init__(self, shape, dtype=Any, strides=None):
        if isinstance(shape, (int, PrimExpr)) or shape is int:
            shape = [shape]
        self.shape = list(shape)
        self.strides = list(strides) if strides is not None else None
        self.dtype = None if dtype is Any or dtype is None else _dt.as_dtype(dtype)

    def __repr__(self):
        return f"TensorTemplate({self.shape}, {self.dtype}, strides={self.strides})"


class _StridedTensorFactory:
    """``T.StridedTensor(shape, strides, dtype)`` and ``T.StridedTensor[shape, strides, dtype]``."""

    def __call__(self, shape, strides, dtype="float32"):
        if _is_template(shape, strides, dtype):
            return TensorTemplate(shape, dtype, strides)
        return TensorAnnot(shape, dtype, strides=list(strides))

    def __getitem__(self, key):
        if not isinstance(key, tuple) or len(key) != 3:
            raise TypeError("T.StridedTensor[shape, strides, dtype]")
        return self(*key)


StridedTensor = _StridedTensorFactory()


class DynAnnot:
    """``T.dyn[int, 'X']``: a runtime integer (scalar parameter or shape symbol) named X."""

    def __init__(self, dtype="int32", name=None):
        self.dtype = _dt.as_dtype("int32" if dtype is int else dtype)
        self.name = name


class _PtrFactory:
    """``T.ptr`` (lazy_jit annotation of a raw tensor pointer, bound with ``T.make_tensor``) and
    ``T.ptr()`` (the matching placeholder in ``par_compile`` signatures)."""

    def __call__(self, dtype="handle"):
        return PtrSpec()

    def __repr__(self):
        return "T.ptr"


class PtrSpec:
    pass


ptr = _PtrFactory()


class _DTypeAnnot:
    """``T.dtype``: annotation of a compile-time dtype parameter; ``T.dtype(x)`` converts."""

    def __call__(self, x):
        return _dt.as_dtype(x)

    def __instancecheck__(self, obj):
        return isinstance(obj, _dt.DType)


dtype = _DTypeAnnot()


Tensor = _TensorFactory("global")
Buffer_ = _TensorFactory("global")
FragmentBuffer = _TensorFactory("fragment")
SharedBuffer = _TensorFactory("shared")
LocalBuffer = _TensorFactory("local")


class _Dyn:
    """``T.dyn[int32]`` / ``T.dyn['name']`` / ``T.dyn[int, 'name']`` / ``T.dyn('m')``: dynamic
    scalar/shape symbol."""

    def __getitem__(self, key):
        if isinstance(key, tuple):
            return DynAnnot(*key)
        if isinstance(key, str) and key not in _dt.NAMES:
            return DynAnnot("int32", key)
        if key is int:
            return DynAnnot("int32")
        return ScalarAnnot(key)

    def __call__(self, name="n", dtype="int32"):
        return Var(name, _dt.as_dtype(dtype), nonneg=True)


dyn = _Dyn()


class MeshReplicationType(Enum):
    NONE = 0
    ROW = 1
    COLUMN = 2
    ALL = 3


class MeshShardingPolicy:

    def __init__(self, x: Optional[int] = None, y: Optional[int] = None,
                 replicate: MeshReplicationType = MeshReplicationType.NONE, cross_mesh_dim: Optional[int] = None):
        if cross_mesh_dim is not None and (x is not None or y is not None):
            raise ValueError("cross_mesh_dim is mutually exclusive with x/y splits")
        self.x = x
        self.y = y
        self.replicate = replicate
        self.cross_mesh_dim = cross_mesh_dim

    def __repr__(self):
        if self.cross_mesh_dim is not None:
            return f"MeshLayout(split_dim={self.cross_mesh_dim} across XxY)"
        parts = []
        if self.x is not None:
            parts.append(f"x→dim{self.x}")
        if self.y is not None:
            parts.append(f"y→dim{self.y}")
        if self.replicate != MeshReplicationType.NONE:
            parts.append(f"replicate={self.replicate.name}")
        return "MeshLayout(" + ", ".join(parts) + ")" if parts else "MeshLayout(replicated)"

    def to_dict(self):
        return {"x": self.x, "y": self.y, "replicate": self.replicate.name, "cross_mesh_dim": self.cross_mesh_dim}


class TensorWithMeta(TensorAnnot):
    """A sharded tensor annotation carrying global/sharded metadata."""

    def __init__(self, shape, dtype, strides, meta):
        super().__init__(shape, dtype, strides=strides, meta=meta)
        self.meta_data = meta

    @property
    def buffer(self):
        return self


def _check_dim(d, rank, what):
    if not 0 <= d < rank:
        raise ValueError(f"Invalid {what}: {d}, tensor rank is {rank}")


class MeshTensorAnnot:

    @staticmethod
    def _get_sharded_shape(shape, policy: MeshShardingPolicy, nrows: int, ncols: int):
        out = list(shape)
        if policy.replicate == MeshReplicationType.ALL:
            return tuple(out)
        rank = len(out)
        if policy.cross_mesh_dim is not None:
            _check_dim(policy.cross_mesh_dim, rank, "cross_mesh_dim")
            out[policy.cross_mesh_dim] = int(math.ceil(out[policy.cross_mesh_dim] / (nrows * ncols)))
            return tuple(out)
        split_x = policy.x is not None
        split_y = policy.y is not None
        if policy.replicate == MeshReplicationType.ROW and split_x:
            raise ValueError("Cannot shard on x-axis when replicating on rows")
        if policy.replicate == MeshReplicationType.COLUMN and split_y:
            raise ValueError("Cannot shard on y-axis when replicating on columns")
        if split_x:
            _check_dim(policy.x, rank, "x-split dimension")
            out[policy.x] = int(math.ceil(out[policy.x] / ncols))
        if split_y:
            _check_dim(policy.y, rank, "y-split dimension")
            out[policy.y] = int(math.ceil(out[policy.y] / nrows))
        return tuple(out)

    @staticmethod
    def _get_sharded_hierarchical_layout(hdims, hgroups, policy: MeshShardingPolicy, nrows: int, ncols: int):
        out = list(hdims)
        factors = []
        if policy.cross_mesh_dim is not None:
            factors.append((policy.cross_mesh_dim, nrows * ncols))
        else:
            if policy.y is not None:
                factors.append((policy.y, nrows))
            if policy.x is not None:
                factors.append((policy.x, ncols))
        from .._native import core
        groups = [tuple(g) for g in hgroups]
        for dim, f in factors:
            out = core().shard_hier(out, groups, dim, f)  # csrc/core/hier.cc
        return tuple(out)

    @staticmethod
    def _derive_sharded_hstrides(sharded_hdims, global_hstrides):
        if not sharded_hdims:
            return ()
        order = sorted(range(len(global_hstrides)), key=lambda i: global_hstrides[i])
        out = [0] * len(sharded_hdims)
        acc = 1
        for i in order:
            out[i] = acc
            acc *= sharded_hdims[i]
        return tuple(out)

    def __call__(self, shape, sharding_policy: MeshShardingPolicy, device_mesh_config, dtype="float32", data=None,
                 strides=None, elem_offset=None, scope=None, align=0, offset_factor=0, buffer_type="",
                 axis_separators=None, hierarchical_dims=None, hierarchical_strides=None,
                 hierarchical_groups=None) -> TensorWithMeta:
        if isinstance(shape, (int, PrimExpr)):
            shape = (shape, )
        shape = tuple(shape)
        nrows, ncols = device_mesh_config
        sharded = self._get_sharded_shape(shape, sharding_policy, nrows, ncols)
        sharded_strides = _row_major_strides(sharded)
        meta = dict(global_shape=shape, global_strides=_row_major_strides(shape))
        if hierarchical_dims is not None:
            sh = self._get_sharded_hierarchical_layout(hierarchical_dims, hierarchical_groups, sharding_policy, nrows,
                                                       ncols)
            meta.update(global_hdims=tuple(hierarchical_dims), global_hstrides=tuple(hierarchical_strides),
                        global_hgroups=tuple(tuple(g) for g in hierarchical_groups), sharded_hdims=sh,
                        sharded_hstrides=self._derive_sharded_hstrides(sh, hierarchical_strides),
                        sharded_hgroups=tuple(tuple(g) for g in hierarchical_groups))
        else:
            meta.update(global_hdims=shape, global_hstrides=_row_major_strides(shape),
                        global_hgroups=tuple((i, i + 1) for i in range(len(shape))), sharded_hdims=sharded,
                        sharded_hstrides=sharded_strides,
                        sharded_hgroups=tuple((i, i + 1) for i in range(len(shape))))
        t = TensorWithMeta(sharded, dtype, list(sharded_strides), meta)
        t.sharding_policy = sharding_policy
        t.device_mesh_config = (nrows, ncols)
        return t


MeshTensor = MeshTensorAnnot()


# ---------------------------------------------------------------------------
# lazy_jit tracing context (tilelang/jit/lazy.py)
# ---------------------------------------------------------------------------


class PtrParam:
    """A ``T.ptr`` parameter while a lazy_jit kernel is traced; ``T.make_tensor`` binds it."""

    def __init__(self, name):
        self.name = name


class LazyTrace:

    def __init__(self):
        self.outputs = []     # buffers created by T.empty, in creation order
        self.ptr_buffers = {}  # PtrParam -> Buffer


class _ThreadLocalStack:
    """A per-thread list: ``lazy_jit.par_compile`` traces kernels in a thread pool, and one
    thread's ``T.empty`` outputs / ``T.make_tensor`` bindings must never land on another's trace."""

    def __init__(self):
        self._tls = threading.local()

    def _list(self):
        lst = getattr(self._tls, "stack", None)
        if lst is None:
            lst = self._tls.stack = []
        return lst

    def append(self, x):
        self._list().append(x)

    def pop(self):
        return self._list().pop()

    def __getitem__(self, i):
        return self._list()[i]

    def __len__(self):
        return len(self._list())

    def __bool__(self):
        return bool(self._list())


LAZY_STACK = _ThreadLocalStack()


def make_tensor(ptr, shape, dtype="float32", strides=None):
    """``T.make_tensor(ptr, shape, dtype)``: view a ``T.ptr`` parameter as a global tensor."""
    if not isinstance(ptr, PtrParam) or not LAZY_STACK:
        raise TypeError("T.make_tensor needs a T.ptr parameter of a @tilelang.lazy_jit kernel")
    ctx = LAZY_STACK[-1]
    if ptr in ctx.ptr_buffers:
        raise ValueError(f"T.ptr parameter {ptr.name!r} is bound by T.make_tensor twice")
    if isinstance(shape, (int, PrimExpr)):
        shape = (shape, )
    b = Buffer(ptr.name, list(shape), dtype, "global", strides=strides)
    ctx.ptr_buffers[ptr] = b
    return b
