"""``T.gemm_sp`` under its reference import path (``tilelang/language/experimental/gemm_sp.py``)."""
from ..tileops import gemm_sp, gemm_sp_v2  # noqa: F401
