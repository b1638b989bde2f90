"""Locations of the native libraries (reference: tilelang/libinfo.py finds libtilelang*.so)."""
import glob
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def find_lib_path(name: str = "_tl_runtime"):
    """Paths of the in-tree extension modules matching ``name`` (``_tl_runtime`` / ``_tl_core``)."""
    return sorted(glob.glob(os.path.join(_HERE, f"{name}*.so")))


def include_dir() -> str:
    """Device headers (``tl/*.h``) compiled into every kernel."""
    return os.path.join(_HERE, "include")
