"""``tilelang.lower``: PrimFunc -> gfx950 HIP (or CPU C++) source + launch metadata.

Reference: ``tilelang/engine/lower.py:217-272`` and the pass pipeline in
``tilelang/engine/phase.py`` (``PreLowerSemanticCheck`` -> ``LowerAndLegalize`` ->
``OptimizeForTarget``).  The MI355X pipeline, run per ``T.Kernel`` of the program:

  1. semantic checks (nested-loop / fragment-loop legality)
  2. layout inference (fragments + LDS swizzles)              transform/layout_inference.py
  3. software pipelining (LDS-DMA ring, counted vmcnt)         transform/pipeline.py
  4. tile-op + parallel-loop lowering (SIMT, vectorised)       transform/lower_tile_op.py
  5. barrier insertion                                         transform/thread_sync.py
  6. LDS arena planning (one __shared__ array, <=160 KiB)       transform/lds_plan.py
  7. code generation                                           codegen/hip.py

A program may contain several ``T.Kernel`` scopes (e.g. split-KV attention + combine):
each becomes its own gfx950 kernel and the runtime launches them in program order on the
current stream.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..ir import stmt as S
from ..utils.target import Target, determine_target
from ..analysis.checks import semantic_check, SemanticError
from ..transform.layout_inference import infer_layouts
from ..transform.pipeline import inject_software_pipeline
from ..transform.lower_tile_op import lower_tile_ops
from ..transform.thread_sync import insert_thread_sync
from ..transform.lds_plan import LDSPlanError, plan_lds
from ..codegen.hip import generate, KernelSource
from ..transform.pass_config import validate_pass_configs


@dataclass
class DeviceKernel:
    source: str
    name: str
    grid: list
    block: list
    lds_bytes: int
    params: list
    lowered_ir: Optional[S.Stmt] = None
    layout_info: Dict[str, str] = field(default_factory=dict)
    mesh: Optional[dict] = None   # T.comm kernels: mesh shape, op count, workspace bytes
    narrow_index: set = field(default_factory=set)  # global params addressed with int32 offsets
    cooperative: bool = False     # uses T.sync_grid: launched cooperatively (all blocks resident)


@dataclass
class CompiledArtifact:
    """Reference ``tilelang/engine/param.py:106-116``."""
    func: S.PrimFunc
    target: Target
    kernels: List[DeviceKernel]
    is_cpu: bool
    timings: Dict[str, float] = field(default_factory=dict)

    # single-kernel conveniences (first kernel)
    @property
    def kernel_source(self) -> str:
        if len(self.kernels) == 1:
            return self.kernels[0].source
        return "\n// ---- next kernel ----\n".join(k.source for k in self.kernels)

    @property
    def kernel_name(self) -> str:
        return self.kernels[0].name

    @property
    def params(self):
        return self.kernels[0].params

    @property
    def grid(self):
        return self.kernels[0].grid

    @property
    def block(self):
        return self.kernels[0].block

    @property
    def lds_bytes(self):
        return max(k.lds_bytes for k in self.kernels)

    @property
    def lowered_ir(self):
        return self.kernels[0].lowered_ir

    @property
    def layout_info(self):
        out = {}
        for k in self.kernels:
            out.update(k.layout_info)
        return out


def _find_kernels(body) -> List[S.KernelStmt]:
    ks = [s for s in S.walk(body) if isinstance(s, S.KernelStmt)]
    if not ks:
        raise SemanticError("a prim_func must contain at least one T.Kernel launch")
    return ks


def _lower_one(func, kernel: S.KernelStmt, target: Target, cfg, name: str, timings):
    if target.kind == "cpu" and not kernel.is_cpu:
        # a GPU-style kernel compiled for the CPU target runs one "thread" per block
        kernel = S.KernelStmt(kernel.grid, [1], kernel.block_vars, kernel.thread_vars, kernel.body, True,
                              kernel.prelude)
    if target.kind == "hip" and kernel.num_threads % 64 != 0:
        raise ValueError(f"T.Kernel threads={kernel.threads}: the block size must be a multiple of the 64-lane "
                         f"CDNA wavefront")
    T = kernel.num_threads if target.kind == "hip" else 1
    semantic_check(func, kernel)
    if cfg.get("tl.force_let_inline"):
        from ..transform.let_inline import inline_lets
        kernel = inline_lets(kernel)
    from ..transform.stage_schedule import apply_stage_schedules
    kernel = apply_stage_schedules(kernel)  # T.Pipelined(order=, stage=, group=)
    if not cfg.get("tir.disable_storage_rewrite"):
        from ..transform.storage_rewrite import rewrite_local_storage
        # local arrays with disjoint lifetimes share storage (+ element-wise in-place reuse if asked)
        kernel, _ = rewrite_local_storage(kernel, bool(cfg.get("tl.storage_rewrite_detect_inplace")))
    quad_default = os.environ.get("TL_GEMM_QUAD", "1") != "0"  # process-wide A/B switch
    if target.kind == "hip" and cfg.get("tl.gemm_quad", quad_default) is not False:
        from ..transform.gemm_ksplit import mark_quad_loops
        kernel = mark_quad_loops(kernel, T, target)  # 256x256x64 NT loops -> tl::gemm_quad_nt_x
    phased = cfg.get("tl.gemm_phased")
    if target.kind == "hip" and phased is not False:  # default on: +15 % at 4096^3 (profiles/r2/gemm_phased.log)
        from ..transform.gemm_ksplit import split_gemm_k_halves
        kernel = split_gemm_k_halves(kernel, True if phased is None else phased)
    t = time.perf_counter()
    li = infer_layouts(S.PrimFunc(func.name, func.params, kernel, func.attrs), T, target)
    timings["layout_inference"] = timings.get("layout_inference", 0) + time.perf_counter() - t
    t = time.perf_counter()
    kernel = inject_software_pipeline(kernel, T, target)
    timings["pipeline"] = timings.get("pipeline", 0) + time.perf_counter() - t
    t = time.perf_counter()
    lk, ctx = lower_tile_ops(kernel, target, cfg)
    timings["lower_tile_op"] = timings.get("lower_tile_op", 0) + time.perf_counter() - t
    if target.kind == "hip" and not cfg.get("tl.disable_address_hoist"):
        from ..transform.hoist_addresses import hoist_dma_sources
        lk = hoist_dma_sources(lk)  # per-thread LDS-DMA source addresses out of pipelined loops
    if target.kind == "hip" and not cfg.get("tl.disable_thread_storage_sync", False):
        lk = insert_thread_sync(lk)
    from ..transform.unswitch import unswitch_marked
    lk = unswitch_marked(lk)  # T.Pipelined(order_alt=): one loop per wave group (after barriers)
    lk, offsets, total = plan_lds(lk, reuse=bool(cfg.get("tl.lds_reuse", True)),
                                  aggressive=bool(cfg.get("tl.enable_aggressive_shared_memory_merge", True)))
    if cfg.get("tl.layout_visualization_enable"):
        from ..analysis.layout_visual import dump_layouts
        dump_layouts(name, li, cfg.get("tl.layout_visualization_formats") or "txt")
    t = time.perf_counter()
    ks: KernelSource = generate(func, lk, target, offsets, total, name, cfg)
    timings["codegen"] = timings.get("codegen", 0) + time.perf_counter() - t
    layout_info = {b.name: repr(lay) for b, lay in li.frag.items()}
    src = ks.source
    if target.kind == "hip":
        from .callback import apply_hip_postproc
        src = apply_hip_postproc(src, target)  # register_hip_postproc hook (engine/callback.py)
    return DeviceKernel(src, ks.kernel_name, ks.grid, ks.block, ks.lds_bytes, ks.params, lk, layout_info,
                        lk.attrs.get("mesh"), set(lk.attrs.get("narrow_index", ())),
                        bool(lk.attrs.get("cooperative", False)))


def lower(func: S.PrimFunc, target="auto", target_host=None, pass_configs: Optional[dict] = None,
          enable_host_codegen=False, enable_device_compile=False, runtime_only=False) -> CompiledArtifact:
    t0 = time.perf_counter()
    import copy
    target = copy.copy(determine_target(target))  # per-compile options are set on the target below
    cfg = validate_pass_configs({str(k): v for k, v in dict(pass_configs or {}).items()})
    kernels = _find_kernels(func.body)
    if any(k.is_cpu for k in kernels) and target.kind != "cpu":
        target = Target("cpu", "host", target.mesh)
    if cfg.get("tl.disable_glds"):
        target.disable_glds = True
    target.mfma_shape = cfg.get("tl.mfma_shape")
    target.gemm_prefetch = cfg.get("tl.gemm_prefetch")      # register-prefetched K-half GEMM schedule
    target.gemm_interleave = cfg.get("tl.gemm_interleave")  # its 1 MFMA : 1 ds_read sched_group_barrier
    target.gemm_rs_pipe = cfg.get("tl.gemm_rs_pipe")        # register-A GEMM: B fragments streamed in groups
    if target.gemm_rs_pipe is None and os.environ.get("TL_GEMM_RS_PIPE"):  # process-wide A/B switch
        target.gemm_rs_pipe = int(os.environ["TL_GEMM_RS_PIPE"]) or None
    target.no_atomic_stage = os.environ.get("TL_ATOMIC_STAGE", "1") == "0"  # process-wide A/B switch
    # default unroll of lowered pipelined loops; TL_PIPELINE_UNROLL is the process-wide A/B switch
    target.pipeline_unroll = cfg.get("tl.pipeline_unroll") or int(os.environ.get("TL_PIPELINE_UNROLL") or 0) or None
    timings: Dict[str, float] = {}
    dks = []
    for i, k in enumerate(kernels):
        name = f"{func.name}_kernel" if i == 0 else f"{func.name}_kernel_{i}"
        try:
            dks.append(_lower_one(func, k, target, cfg, name, timings))
        except LDSPlanError:
            if target.kind != "hip":
                raise
            # the arena went past 160 KiB: retry without the LDS staging of fragment f32 atomics
            # (lower_tile_op.lower_atomic_staged), then also without the padded slots of small-tile
            # LDS-DMA (transform/pipeline.py _small_dma_plan: small tiles through registers)
            for flag in ("no_atomic_stage", "disable_small_dma"):
                t1 = copy.copy(target)
                t1.no_atomic_stage = True
                t1.disable_small_dma = flag == "disable_small_dma"
                try:
                    dks.append(_lower_one(func, k, t1, cfg, name, timings))
                    break
                except LDSPlanError:
                    if flag == "disable_small_dma":
                        raise
    timings["total"] = time.perf_counter() - t0
    return CompiledArtifact(func=func, target=target, kernels=dks, is_cpu=target.kind == "cpu", timings=timings)
