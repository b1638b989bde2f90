"""Loader for the in-tree native runtime extension (``tilelang/_tl_runtime*.so``, built from csrc/).

There is deliberately no Python fallback: if the extension is missing, kernels cannot run and the
error says how to build it (``python setup.py build_ext --inplace``).
"""
_rt = None


class NativeRuntimeMissing(ImportError):
    pass


def runtime():
    global _rt
    if _rt is None:
        try:
            import torch  # noqa: F401  (loads libc10_hip.so, which the extension links against)
            from . import _tl_runtime as m  # noqa: F401
        except ImportError as e:
            raise NativeRuntimeMissing(
                "tilelang native runtime not built: run `python setup.py build_ext --inplace` "
                f"in the repository root ({e})") from e
        _rt = m
    return _rt


def available() -> bool:
    try:
        runtime()
        return True
    except ImportError:
        return False


_core = None


def core():
    """The native compiler core (``tilelang/_tl_core*.so`` from csrc/core).  Mandatory: layout
    inference, lowering and LDS planning run their numeric work in it."""
    global _core
    if _core is None:
        try:
            from . import _tl_core as m  # noqa: F401
        except ImportError as e:
            raise NativeRuntimeMissing(
                "tilelang native compiler core not built: run `python setup.py build_ext --inplace` "
                f"in the repository root ({e})") from e
        _core = m
    return _core
