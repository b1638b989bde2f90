"""Public face of the native runtime (``csrc/tl_runtime.cpp`` → ``tilelang/_tl_runtime*.so``).

The reference's runtime is TVM's packed-function host stubs plus ``tilelang/jit/adapter/`` wrappers
(SURVEY §2.4).  Here it is one C++ extension: a ``hipModuleLaunchKernel`` launcher with argument
validation, uncached workspace memory for cross-GPU flags, and IPC handles for peer-mapped xGMI
buffers.  This module re-exports the pieces a user may want directly; kernels reach the launcher
through ``JITKernel`` and need nothing from here.
"""
from __future__ import annotations

from .._native import NativeRuntimeMissing, available, runtime

__all__ = ["NativeRuntimeMissing", "available", "runtime", "device_info", "Workspace", "can_access_peer"]


def device_info(device: int = 0) -> dict:
    """HIP device properties the compiler and launcher rely on (CU count, LDS, arch, ...)."""
    return runtime().device_info(device)


def can_access_peer(device: int, peer: int) -> bool:
    return bool(runtime().can_access_peer(device, peer))


class Workspace:
    """Device memory owned by the native runtime (``uncached=True``: ``hipExtMallocWithFlags`` with
    ``hipDeviceMallocUncached``, what the Mesh uses for its cross-GPU flag words).  Zeroed on
    creation; freed on ``close()`` or garbage collection.  ``ipc_handle()`` exports it to another
    process."""

    def __init__(self, nbytes: int, device: int = 0, uncached: bool = False):
        self._rt = runtime()
        self.nbytes, self.device = int(nbytes), int(device)
        self.ptr = self._rt.ws_alloc(self.nbytes, self.device, 1 if uncached else 0)

    def zero(self):
        self._rt.ws_zero(self.ptr, self.nbytes, self.device)

    def ipc_handle(self) -> bytes:
        return self._rt.ipc_get_handle(self.ptr, self.device)

    def close(self):
        if self.ptr:
            self._rt.ws_free(self.ptr, self.device)
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
