"""``tilelang.lower``: PrimFunc -> gfx950 HIP (or CPU C++) source + launch metadata.

Reference: ``tilelang/engine/lower.py:217-272`` and the pass pipeline in
``tilelang/engine/phase.py`` (``PreLowerSemanticCheck`` -> ``LowerAndLegalize`` ->
``OptimizeForTarget``).  The MI355X pipeline:

  1. semantic checks (nested-loop / fragment-loop legality)
  2. layout inference (fragments + LDS swizzles)              transform/layout_inference.py
  3. software pipelining (LDS-DMA ring, counted vmcnt)         transform/pipeline.py
  4. tile-op + parallel-loop lowering (SIMT, vectorised)       transform/lower_tile_op.py
  5. barrier insertion                                         transform/thread_sync.py
  6. LDS arena planning (one __shared__ array, <=160 KiB)       transform/lds_plan.py
  7. code generation                                           codegen/hip.py
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..ir import stmt as S
from ..ir.buffer import Buffer
from ..ir.expr import PrimExpr, Var
from ..utils.target import Target, determine_target
from ..analysis.checks import semantic_check
from ..transform.layout_inference import infer_layouts
from ..transform.pipeline import inject_software_pipeline
from ..transform.lower_tile_op import lower_tile_ops
from ..transform.thread_sync import insert_thread_sync
from ..transform.lds_plan import plan_lds
from ..codegen.hip import generate, KernelSource


@dataclass
class CompiledArtifact:
    """Reference ``tilelang/engine/param.py:106-116``."""
    func: S.PrimFunc
    target: Target
    kernel_source: str
    kernel_name: str
    params: list
    grid: list
    block: list
    lds_bytes: int
    is_cpu: bool
    lowered_ir: Optional[S.Stmt] = None
    timings: Dict[str, float] = field(default_factory=dict)
    layout_info: Dict[str, str] = field(default_factory=dict)


def _find_kernel(body) -> S.KernelStmt:
    ks = [s for s in S.walk(body) if isinstance(s, S.KernelStmt)]
    if len(ks) != 1:
        raise ValueError(f"a prim_func must contain exactly one T.Kernel launch (found {len(ks)})")
    return ks[0]


def lower(func: S.PrimFunc, target="auto", target_host=None, pass_configs: Optional[dict] = None,
          enable_host_codegen=False, enable_device_compile=False, runtime_only=False) -> CompiledArtifact:
    t0 = time.perf_counter()
    target = determine_target(target)
    cfg = dict(pass_configs or {})
    kernel = _find_kernel(func.body)
    if target.kind == "cpu" and not kernel.is_cpu:
        # a GPU-style kernel compiled for the CPU target runs one "thread" per block
        kernel = S.KernelStmt(kernel.grid, [1], kernel.block_vars, kernel.thread_vars, kernel.body, True,
                              kernel.prelude)
    if kernel.is_cpu and target.kind != "cpu":
        target = Target("cpu", "host", target.mesh)
    if target.kind == "hip" and kernel.num_threads % 64 != 0:
        raise ValueError(f"T.Kernel threads={kernel.threads}: the block size must be a multiple of the 64-lane "
                         f"CDNA wavefront")
    if cfg.get("tl.disable_glds"):
        target.disable_glds = True
    T = kernel.num_threads if target.kind == "hip" else 1
    timings = {}
    semantic_check(func, kernel)
    t = time.perf_counter()
    li = infer_layouts(S.PrimFunc(func.name, func.params, kernel, func.attrs), T, target)
    timings["layout_inference"] = time.perf_counter() - t
    t = time.perf_counter()
    kernel = inject_software_pipeline(kernel, T, target)
    timings["pipeline"] = time.perf_counter() - t
    t = time.perf_counter()
    lk, ctx = lower_tile_ops(kernel, target, cfg)
    timings["lower_tile_op"] = time.perf_counter() - t
    if target.kind == "hip" and not cfg.get("tl.disable_thread_storage_sync", False):
        lk = insert_thread_sync(lk)
    offsets, total = plan_lds(lk)
    t = time.perf_counter()
    ks: KernelSource = generate(func, lk, target, offsets, total, func.name + "_kernel", cfg)
    timings["codegen"] = time.perf_counter() - t
    timings["total"] = time.perf_counter() - t0
    layout_info = {b.name: repr(lay) for b, lay in li.frag.items()}
    return CompiledArtifact(func=func, target=target, kernel_source=ks.source, kernel_name=ks.kernel_name,
                            params=ks.params, grid=ks.grid, block=ks.block, lds_bytes=ks.lds_bytes,
                            is_cpu=ks.is_cpu, lowered_ir=lk, timings=timings, layout_info=layout_info)
