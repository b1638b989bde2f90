"""``import tilelang.language as T`` — the tile DSL (reference ``tilelang/language/__init__.py``)."""
from __future__ import annotations

from ..ir import dtypes as _dtypes
from ..ir.dtypes import (float16, bfloat16, float32, float64, float8_e4m3fn, float8_e5m2, float8_e4m3fnuz,
                         float8_e5m2fnuz, float8_e8m0fnu, float4_e2m1fn, int8, int16, int32, int64, uint8, uint16,
                         uint32, uint64, DType)
from ..ir.dtypes import boolean as bool  # noqa: A001
from ..ir.expr import PrimExpr, Var, IntImm, FloatImm, StringImm, const
from ..ir.buffer import BufferRegion
from ..ir.expr import BufferLoad
from .parser import prim_func, macro, TensorAnnot
from .annot import (Tensor, StridedTensor, FragmentBuffer, SharedBuffer, LocalBuffer, dyn, MeshTensor,
                    MeshShardingPolicy, MeshReplicationType, TensorWithMeta, MeshTensorAnnot, TensorTemplate, ptr,
                    dtype, make_tensor)
from ..ir.dtypes import float8_e4m3fn as float8_e4m3  # noqa: F401
from .annot import Buffer_ as Buffer
from .kernel import (Kernel, KernelLaunchFrame, get_thread_binding, get_thread_bindings, get_block_binding,
                     get_block_bindings, get_thread_extent, get_block_extent, get_thread_extents,
                     get_block_extents)
from .loop import Parallel, Pipelined, Persistent, serial, Serial, unroll, Unroll, vectorized, Vectorized, grid
from .allocate import (alloc_shared, alloc_fragment, alloc_local, alloc_var, alloc_buffer, alloc_reducer,
                       alloc_barrier, alloc_tmem, alloc_descriptor, alloc_wgmma_desc, alloc_tcgen05_smem_desc,
                       alloc_tcgen05_instr_desc, empty)
from .tileops import (copy, gather_rows, c2d_im2col, gemm, gemm_v1, gemm_v2, gemm_scaled, gemm_sp, gemm_sp_v2,
                      GemmWarpPolicy, fill, clear, reduce,
                      reduce_max, reduce_min, reduce_sum, reduce_abssum, reduce_absmax, reduce_bitand, reduce_bitor,
                      reduce_bitxor, cumsum, finalize_reducer, warp_reduce_sum, warp_reduce_max, warp_reduce_min,
                      warp_reduce_bitand, warp_reduce_bitor, atomic_add, atomic_max, atomic_min, atomic_addx2,
                      atomic_addx4, atomic_load, atomic_store, reshape, view)
from .math import *  # noqa: F401,F403
from .math import (max, min, abs, round, pow)  # noqa: A004,F401
from .builtin import (sync_threads, sync_warp, sync_global, sync_grid, fence_proxy_async, memory_fence, set_priority,
                      get_lane_idx, get_warp_idx, get_warp_idx_sync, get_warp_group_idx, shfl_xor, shfl_down, shfl_up,
                      shfl_sync, ballot, clock, call_extern, call_intrin, evaluate, loop_break, device_assert, print,
                      use_swizzle, annotate_layout, annotate_safe_value, annotate_l2_hit_ratio, annotate_padding,
                      annotate_nontemporal, attr,
                      block_attr, import_source, no_set_max_nreg, set_max_nreg, disable_warp_group_reg_alloc, assume,
                      address_of, dynamic, symbolic)
from .builder import _IfFrame as If, _ElseFrame as Else, _WhileFrame as While
from . import comm
from .logical import any_of, all_of
from ..layout import Layout, Fragment

ceildiv = ceildiv  # noqa: F405 (from math)

# C-style dtype aliases (reference frontend v2 dtypes): T.short, T.int, T.long, T.half, T.float,
# T.double (T.bool is the boolean dtype above)
short = int16
int = int32  # noqa: A001
long = int64
half = float16
float = float32  # noqa: A001
double = float64


def int_(x):
    return IntImm(x)


def float_(x):
    return FloatImm(x)


def index_to_coordinates(index, shape):
    coords = []
    for s in reversed(list(shape)):
        coords.append(index % s)
        index = index // s
    return list(reversed(coords))


def has_let_value(var):
    return False


def get_let_value(var):
    return None


def ws(*args, **kwargs):
    raise NotImplementedError("warp specialisation (T.ws) targets Hopper; gfx950 pipelines with LDS-DMA instead")
