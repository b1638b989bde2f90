"""Library kernels built with the tile DSL (used by ``tilelang.models``).

* ``gemm.linear``        -- y = x W^T (MFMA GEMM, tiles picked by problem size)
* ``norm.rms_norm``      -- fused RMSNorm * weight (row in registers)
* ``quant.act_quant``    -- per-128-group fp8 (e4m3) activation quantisation with fp32 scales
* ``dsa``                -- DeepSeek sparse attention: sparse MLA, lightning indexer, top-k selector
* ``moe``                -- grouped-GEMM SwiGLU experts and token packing
"""
