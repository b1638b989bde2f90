"""Environment / configuration (reference ``tilelang/env.py:126-300``)."""
from __future__ import annotations

import os
from pathlib import Path

PACKAGE_ROOT = Path(__file__).resolve().parent
INCLUDE_DIR = PACKAGE_ROOT / "include"
ROCM_PATH = os.environ.get("ROCM_PATH", "/opt/rocm")


def _flag(name: str, default: str = "0") -> bool:
    return os.environ.get(name, default).lower() in ("1", "true", "yes", "on")


class EnvVar:
    """Descriptor reading an environment variable with a default (re-read on access)."""

    def __init__(self, key: str, default: str):
        self.key = key
        self.default = default

    def __get__(self, obj, objtype=None):
        return os.environ.get(self.key, self.default)

    def __set__(self, obj, value):
        os.environ[self.key] = str(value)


class Environment:
    TILELANG_CACHE_DIR = EnvVar("TILELANG_CACHE_DIR", str(Path.home() / ".tilelang" / "cache"))
    TILELANG_TMP_DIR = EnvVar("TILELANG_TMP_DIR", str(Path.home() / ".tilelang" / "tmp"))
    TILELANG_PRINT_ON_COMPILATION = EnvVar("TILELANG_PRINT_ON_COMPILATION", "0")
    TILELANG_DISABLE_CACHE = EnvVar("TILELANG_DISABLE_CACHE", "0")
    TILELANG_CLEAR_CACHE = EnvVar("TILELANG_CLEAR_CACHE", "0")
    TILELANG_AUTO_TUNING_DISABLE_CACHE = EnvVar("TILELANG_AUTO_TUNING_DISABLE_CACHE", "0")
    TILELANG_AUTO_TUNING_CPU_UTILITIES = EnvVar("TILELANG_AUTO_TUNING_CPU_UTILITIES", "0.9")
    TILELANG_AUTO_TUNING_CPU_COUNTS = EnvVar("TILELANG_AUTO_TUNING_CPU_COUNTS", "-1")
    TILELANG_AUTO_TUNING_MAX_CPU_COUNT = EnvVar("TILELANG_AUTO_TUNING_MAX_CPU_COUNT", "16")
    TL_TEMPLATE_PATH = EnvVar("TL_TEMPLATE_PATH", str(INCLUDE_DIR))
    ROCM_PATH = EnvVar("ROCM_PATH", ROCM_PATH)

    def is_cache_enabled(self) -> bool:
        return not _flag("TILELANG_DISABLE_CACHE")

    def is_print_on_compilation_enabled(self) -> bool:
        return _flag("TILELANG_PRINT_ON_COMPILATION")

    def is_autotune_cache_enabled(self) -> bool:
        return not _flag("TILELANG_AUTO_TUNING_DISABLE_CACHE")

    def disable_cache(self):
        os.environ["TILELANG_DISABLE_CACHE"] = "1"

    def enable_cache(self):
        os.environ["TILELANG_DISABLE_CACHE"] = "0"


env = Environment()
