"""tilelang (MI355X-native): a tile-programming DSL + JIT compiler for AMD Instinct MI355X (gfx950).

API-compatible with TileLang / TileLang-Mesh (``@tilelang.jit``, ``import tilelang.language as T``),
re-designed for CDNA4: the only device target is gfx950 HIP (plus a host C++ plumbing target).
"""
import logging as _logging

__version__ = "0.1.7+mi355x"

from . import ir  # noqa: F401
from . import language  # noqa: F401
from .env import env  # noqa: F401
from .jit import jit, lazy_jit, compile, par_compile, JITKernel  # noqa: F401,A004
from .engine.lower import lower  # noqa: F401
from .cache import clear_cache, disable_cache, enable_cache  # noqa: F401
from .utils.target import determine_target  # noqa: F401
from . import layout  # noqa: F401
from . import math  # noqa: F401,A004
from .math import cdiv, next_power_of_2  # noqa: F401


class _TqdmLoggingHandler(_logging.StreamHandler):
    pass


logger = _logging.getLogger("tilelang")
if not logger.handlers:
    _h = _TqdmLoggingHandler()
    _h.setFormatter(_logging.Formatter("[TileLang:%(name)s:%(levelname)s]: %(message)s"))
    logger.addHandler(_h)
    logger.setLevel(_logging.WARNING)


def set_log_level(level):
    if isinstance(level, str):
        level = getattr(_logging, level.upper())
    logger.setLevel(level)


def __getattr__(name):
    # lazily import heavier tooling
    if name in ("autotune", "AutoTuner"):
        from . import autotuner
        return getattr(autotuner, name)
    if name == "Profiler":
        from .profiler import Profiler
        return Profiler
    if name in ("testing", "carver", "tools", "quantize", "ops", "models", "parallel", "libinfo", "profiler",
                "autotuner", "analysis"):
        import importlib
        return importlib.import_module(f"{__name__}.{name}")
    if name == "TensorSupplyType":
        from .utils.tensor import TensorSupplyType
        return TensorSupplyType
    raise AttributeError(name)

from .transform.pass_config import PassConfigKey  # noqa: E402,F401
