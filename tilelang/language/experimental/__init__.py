"""Experimental language surface (reference ``tilelang/language/experimental``)."""
from .gemm_sp import gemm_sp, gemm_sp_v2  # noqa: F401
