"""Carver: analytical tile-configuration recommender for MI355X (reference ``tilelang/carver``).

    from tilelang.carver.template import MatmulTemplate
    from tilelang.carver.arch import CDNA
    hints = MatmulTemplate(M=4096, N=4096, K=4096).with_arch(CDNA("hip")).recommend_hints(topk=8)
    configs = [h.to_config() for h in hints]      # feed to @tilelang.autotune / a kernel factory

    from tilelang.carver.analysis import recommend   # any naive loop-nest T.prim_func
    hints, what = recommend(naive_gemm_func, CDNA("hip"), topk=8)   # what["kind"] == "gemm"
"""
from . import arch, template, roller, analysis  # noqa: F401
from .analysis import PrimFuncNode, gemm_info, recommend  # noqa: F401
from .arch import CDNA, CPU, TileDevice, auto_infer_current_arch  # noqa: F401
from .template import (MatmulTemplate, GEMVTemplate, ElementwiseTemplate, GeneralReductionTemplate,  # noqa: F401
                       FlashAttentionTemplate, ConvTemplate)
from .roller import Hint, DefaultPolicy, TensorCorePolicy  # noqa: F401
