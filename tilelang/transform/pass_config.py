"""Pass configuration keys (reference ``tilelang/transform/pass_config.py:6-153``).

Keys that only make sense on NVIDIA (TMA, WGMMA, warp specialisation, ptxas) are accepted and
ignored so reference programs run unchanged; gfx950-specific keys are added at the end.
"""
from enum import Enum


class PassConfigKey(str, Enum):
    TL_DISABLE_WARP_SPECIALIZED = "tl.disable_warp_specialized"
    TL_DISABLE_TMA_LOWER = "tl.disable_tma_lower"
    TL_ENABLE_FAST_MATH = "tl.enable_fast_math"
    TL_DISABLE_FAST_MATH = "tl.disable_fast_math"
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
    # gfx950 additions
    TL_DISABLE_GLDS = "tl.disable_glds"            # stage through registers instead of LDS-DMA
    TL_MIN_WAVES_PER_EU = "tl.min_waves_per_eu"    # second __launch_bounds__ argument

    def __str__(self):
        return self.value
