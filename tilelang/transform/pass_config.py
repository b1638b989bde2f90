"""Pass configuration keys (reference ``tilelang/transform/pass_config.py:6-153``).

Every key is either implemented on gfx950 or rejected (``validate_pass_configs``, run by
``tilelang.lower``): a program never gets a silently different compile.  Three kinds:

* implemented — changes what the compiler does (table ``EFFECT`` below says how);
* satisfied by construction — the reference uses the key to switch OFF an NVIDIA-only feature
  (TMA, WGMMA, warp specialisation, 256-bit vectors) or a TVM pass this compiler does not have;
  the "off" value is what gfx950 always does and is accepted, asking for the feature raises;
* unsupported — raises ``NotImplementedError`` (``tl.ptxas_register_usage_level``) with the
  gfx950 alternative in the message.
"""
from enum import Enum


class PassConfigKey(str, Enum):
    TL_DISABLE_WARP_SPECIALIZED = "tl.disable_warp_specialized"
    TL_DISABLE_TMA_LOWER = "tl.disable_tma_lower"
    TL_ENABLE_FAST_MATH = "tl.enable_fast_math"
    TL_DISABLE_FAST_MATH = "tl.disable_fast_math"
    TL_NO_NANS = "tl.no_nans"
    TL_GEMM_FOLD_DEFAULT_GUARD = "tl.gemm_fold_default_guard"
    TL_PTXAS_REGISTER_USAGE_LEVEL = "tl.ptxas_register_usage_level"
    TL_CONFIG_INDEX_BITWIDTH = "tl.config_index_bitwidth"
    TL_DISABLE_SAFE_MEMORY_ACCESS = "tl.disable_safe_memory_legalize"
    TL_DISABLE_VECTORIZE_256 = "tl.disable_vectorize_256"
    TL_DISABLE_WGMMA = "tl.disable_wgmma"
    TL_ENABLE_AGGRESSIVE_SHARED_MEMORY_MERGE = "tl.enable_aggressive_shared_memory_merge"
    TL_DISABLE_THREAD_STORAGE_SYNC = "tl.disable_thread_storage_sync"
    TL_FORCE_LET_INLINE = "tl.force_let_inline"
    TL_LAYOUT_VISUALIZATION_ENABLE = "tl.layout_visualization_enable"
    TL_LAYOUT_VISUALIZATION_FORMATS = "tl.layout_visualization_formats"
    TL_STORAGE_REWRITE_DETECT_INPLACE = "tl.storage_rewrite_detect_inplace"
    TL_DYNAMIC_ALIGNMENT = "tl.dynamic_alignment"
    TL_DISABLE_DYNAMIC_TAIL_SPLIT = "tl.disable_dynamic_tail_split"
    TIR_DISABLE_VECTORIZE = "tir.disable_vectorize"
    TIR_USE_ASYNC_COPY = "tir.use_async_copy"
    TIR_MERGE_STATIC_SMEM = "tir.merge_static_smem"
    TIR_DISABLE_CSE_TIR = "tir.disable_cse_tir"
    TIR_DISABLE_STORAGE_REWRITE = "tir.disable_storage_rewrite"
    # gfx950 additions
    TL_DISABLE_GLDS = "tl.disable_glds"            # stage through registers instead of LDS-DMA
    TL_MIN_WAVES_PER_EU = "tl.min_waves_per_eu"    # second __launch_bounds__ argument
    TL_LDS_REUSE = "tl.lds_reuse"                  # liveness-based LDS arena sharing (default on)
    TL_MFMA_SHAPE = "tl.mfma_shape"                # "16x16" (default) or "32x32" MFMA tiles
    TL_GEMM_PHASED = "tl.gemm_phased"              # K-half phased GEMM main loop (gemm_ksplit)
    TL_GEMM_QUAD = "tl.gemm_quad"                  # 256x256x64 NT tile: whole-loop quadrant schedule
    TL_GEMM_PREFETCH = "tl.gemm_prefetch"          # fragments read one phase ahead of their MFMAs
    TL_GEMM_INTERLEAVE = "tl.gemm_interleave"      # 1 MFMA : 1 ds_read sched_group_barrier pattern
    TL_DISABLE_ADDRESS_HOIST = "tl.disable_address_hoist"  # keep LDS-DMA source addresses in the loop
    TL_GEMM_RS_PIPE = "tl.gemm_rs_pipe"            # register-A GEMM: B fragments streamed in groups of N
    TL_PACK_F32 = "tl.pack_f32"                    # fp32 register pairs as packed v_pk_* math
    TL_PIPELINE_UNROLL = "tl.pipeline_unroll"      # default #pragma unroll N of lowered pipelined loops
    TL_ATOMIC_STAGE = "tl.atomic_stage"            # fragment f32 tile atomics through a row-contiguous LDS tile

    def __str__(self):
        return self.value


# what each implemented key does on gfx950
EFFECT = {
    "tl.enable_fast_math": "exp/log/exp2/log2/sin/cos on the hardware transcendental unit (codegen/hip.py)",
    "tl.disable_fast_math": "forces the precise OCML math even if tl.enable_fast_math is set",
    "tl.gemm_fold_default_guard": "default True: T.gemm's valid_m wave guards are compiled out when unused (the "
                                  "accumulator's initial values need not stay materialised); False keeps the "
                                  "runtime test (same-process A/B, scripts/guard_fold_ab.py: FA bwd dK/dV +3-4 % "
                                  "folded; FA fwd 0 to -4 % and sparse MLA fwd -3 % folded, so those two keep it)",
    "tl.no_nans": "the kernel promises no NaN values (-fno-honor-nans): fmaxf of MFMA results needs no "
                  "canonicalising v_max per operand; isnan checks and NaN-propagating selects may fold",
    "tl.config_index_bitwidth": "32 or 64: width of global-memory offsets (default: 64 only for tensors of "
                                ">= 2^31 elements; the launcher refuses tensors too large for a 32-bit kernel)",
    "tl.disable_safe_memory_legalize": "no bounds guards on global accesses",
    "tl.enable_aggressive_shared_memory_merge": "default True: LDS-DMA stage buffers of pipelined loops share "
                                                "the arena with later buffers (vmcnt(0) drain + barrier at "
                                                "the switch); False pins them for the whole kernel",
    "tl.lds_reuse": "liveness-based LDS arena sharing (False: every shared buffer gets its own bytes)",
    "tl.disable_thread_storage_sync": "no automatic __syncthreads insertion",
    "tl.force_let_inline": "every let binding inside a kernel is substituted into its uses",
    "tl.layout_visualization_enable": "dump the inferred fragment / LDS layouts (tilelang.analysis.layout_visual)",
    "tl.layout_visualization_formats": "'txt' (default), 'svg', 'png' or 'all' for the layout dump",
    "tl.dynamic_alignment": "dynamic shape extents are multiples of N (vectorised accesses on dynamic dims)",
    "tir.disable_vectorize": "scalar (1-element) accesses in every lowered loop and copy",
    "tir.use_async_copy": "False: stage tiles through registers instead of LDS-DMA (= tl.disable_glds)",
    "tl.disable_glds": "stage tiles through registers instead of LDS-DMA",
    "tl.min_waves_per_eu": "second __launch_bounds__ argument (register budget for N waves per SIMD)",
    "tl.mfma_shape": "'16x16' (default) or '32x32': matrix-core tile of T.gemm (f16/bf16, int8)",
    "tir.disable_storage_rewrite": "True: per-thread local arrays with disjoint lifetimes keep separate "
                                   "storage (transform/storage_rewrite.py merges them by default)",
    "tl.gemm_phased": "default on; False keeps BK=64 16-bit GEMM main loops whole instead of splitting them "
                      "into K halves refilled one phase apart (transform/gemm_ksplit.py + the phased "
                      "pipeline schedule); 'prio' also raises wave priority around the MFMA clusters",
    "tl.gemm_quad": "default on; False keeps the 256x256x64 NT GEMM main loop (512 threads, 4x2 waves) on the "
                    "K-half phased schedule instead of tl::gemm_quad_nt (tl/gemm_quad.h: 8-phase quadrant "
                    "schedule, one half-tile restaged per phase, counted vmcnt(6) once per K tile)",
    "tl.gemm_prefetch": "default on; False: in the phased K-half schedule, read each half's MFMA fragments "
                        "after its own barrier instead of one phase ahead (transform/pipeline.py "
                        "_prefetch_schedule, tl::gemm_ss_load / gemm_ss_mma)",
    "tl.disable_address_hoist": "True keeps the per-thread LDS-DMA source address arithmetic inside pipelined "
                                "loops (transform/hoist_addresses.py hoists it by default)",
    "tl.storage_rewrite_detect_inplace": "a local array first written by the element-wise statement that last "
                                         "reads another of the same dtype/shape takes over its storage "
                                         "(transform/storage_rewrite.py _inplace_ok)",
    "tl.pack_f32": "True: fp32 register pairs of unrolled fragment loops are emitted as packed floatx2 math "
                   "(v_pk_mul/add/fma_f32; codegen/hip.py _emit_pk_pair) -- for VALU-bound code: beside MFMAs "
                   "a packed op costs more than the two scalar ones",
    "tl.gemm_rs_pipe": "N > 0: a T.gemm with its A operand in registers streams the B fragments through the "
                       "MFMAs in groups of N (group g+1's ds_reads pinned between group g's MFMAs, across K "
                       "steps; tl::gemm_rs PIPE) instead of reading a whole K step before its first MFMA",
    "tl.gemm_interleave": "default on; False drops the 1 MFMA : 1 ds_read sched_group_barrier pattern of the "
                          "prefetched GEMM (the compiler schedules the two streams itself)",
    "tl.pipeline_unroll": "N > 1: every lowered T.Pipelined main loop without its own unroll= is emitted under "
                          "#pragma unroll N (N a multiple of the ring depth: the stage slots become constants)",
    "tl.atomic_stage": "default on; False keeps T.atomic_add(global_f32, fragment) in the accumulator layout "
                       "(per-element atomics, four 64-byte row pieces per wave instruction) instead of staging "
                       "the tile through LDS for 256-byte row-contiguous atomics (lower_tile_op.lower_atomic_staged)",
}

# NVIDIA-only features / TVM passes that do not exist here: the value meaning "off" is what
# gfx950 always does
SATISFIED = {
    "tl.disable_warp_specialized": True,
    "tl.disable_tma_lower": True,
    "tl.disable_wgmma": True,
    "tl.disable_vectorize_256": True,     # gfx950 vector memory accesses are at most 128 bits
    "tir.merge_static_smem": True,        # all LDS is always one arena
    "tir.disable_cse_tir": True,          # no TIR CSE pass (clang does CSE on the HIP source)
    "tl.disable_dynamic_tail_split": True,  # dynamic tails use guarded accesses, never a split loop
}

UNSUPPORTED = {
    "tl.ptxas_register_usage_level": "ptxas is NVIDIA-only; bound gfx950 registers with "
                                     "pass_configs={'tl.min_waves_per_eu': N}",
}

DEFAULTS = {"tl.disable_dynamic_tail_split": False, "tir.merge_static_smem": False,
            "tir.disable_cse_tir": False, "tl.disable_warp_specialized": False,
            "tl.disable_tma_lower": False, "tl.disable_wgmma": False, "tl.disable_vectorize_256": False}


def validate_pass_configs(cfg: dict) -> dict:
    """Normalise and check ``pass_configs``; raises for unknown keys and unsupported values."""
    out = {}
    known = {k.value for k in PassConfigKey}
    for k, v in dict(cfg or {}).items():
        k = str(k)
        if k not in known:
            if k.startswith("cuda."):
                raise ValueError(f"pass config {k!r} is CUDA-only; this compiler targets gfx950 only")
            raise ValueError(f"unknown pass config key {k!r}; valid keys: {sorted(known)}")
        if k in UNSUPPORTED and v not in (None, False, 0):
            raise NotImplementedError(f"pass config {k!r}: {UNSUPPORTED[k]}")
        if k in SATISFIED and v is not None and bool(v) != SATISFIED[k] and bool(v) != DEFAULTS.get(k, False):
            raise NotImplementedError(f"pass config {k}={v!r} asks for an NVIDIA-only feature that gfx950 "
                                      "does not have")
        if k == "tl.mfma_shape" and v not in (None, "16x16", "32x32"):
            raise ValueError(f"tl.mfma_shape must be '16x16' or '32x32', got {v!r}")
        if k == "tl.gemm_phased" and v not in (None, True, False, "prio"):
            raise ValueError(f"tl.gemm_phased must be a bool or 'prio', got {v!r}")
        if k == "tl.config_index_bitwidth" and v not in (None, 0, 32, 64):
            raise ValueError(f"tl.config_index_bitwidth must be 32 or 64, got {v!r}")
        if k == "tl.layout_visualization_formats" and v is not None:
            fmts = {f.strip() for f in str(v).split(",")}
            if not fmts <= {"txt", "svg", "png", "pdf", "all"}:
                raise ValueError(f"tl.layout_visualization_formats: unknown format in {v!r}")
        out[k] = v
    if out.get("tir.use_async_copy") is False:
        out["tl.disable_glds"] = True
    if out.get("tl.disable_fast_math"):
        out["tl.enable_fast_math"] = False
    return out
