"""Target resolution (reference ``tilelang/utils/target.py:10-197``).

Only two device kinds exist in this framework:
  * ``hip``  — AMD Instinct MI355X, ``gfx950`` (the only GPU target);
  * ``cpu``  — host C++ (the "c" / "llvm" / "cpu" plumbing target of the reference).
A mesh is attached to either as ``-mesh=<nrow>x<ncol>`` (``"hip -mesh=2x4"``); the
reference's ``Sunmmio`` target string maps to a cpu target with its default 4x4 mesh
(IR-only, like the reference).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Optional, Tuple

SUPPORTED_TARGETS = {
    "auto": "Pick hip (gfx950) when a ROCm device is visible, else cpu.",
    "hip": "AMD Instinct MI355X (gfx950, CDNA4).",
    "rocm": "Alias of hip.",
    "cpu": "Host C++ (plumbing / correctness target).",
    "c": "Alias of cpu (reference spelling).",
    "llvm": "Alias of cpu (reference spelling).",
    "Sunmmio": "Mesh IR target of the reference fork; maps to cpu with a 4x4 mesh config.",
}

GFX950 = "gfx950"


@dataclass
class Target:
    kind: str = "hip"            # "hip" | "cpu"
    arch: str = GFX950
    mesh: Optional[Tuple[int, int]] = None
    attrs: dict = field(default_factory=dict)
    disable_glds: bool = False
    disable_small_dma: bool = False  # set when small-tile LDS-DMA padding would overflow the LDS

    def __str__(self):
        s = self.kind if self.kind == "cpu" else f"hip -mcpu={self.arch}"
        if self.mesh:
            s += f" -mesh={self.mesh[0]}x{self.mesh[1]}"
        return s

    @property
    def is_gpu(self):
        return self.kind == "hip"

    def key(self) -> str:
        return str(self)


def check_hip_availability() -> bool:
    try:
        import torch
        return bool(torch.version.hip) and torch.cuda.device_count() > 0
    except Exception:  # noqa: BLE001
        return False


def check_cuda_availability() -> bool:
    return False


def check_metal_availability() -> bool:
    return False


def check_sunmmio_availability() -> bool:
    return False


def determine_target(target="auto", return_object: bool = True):
    if isinstance(target, Target):
        return target if return_object else str(target)
    if target is None:
        target = "auto"
    s = str(target).strip()
    mesh = None
    m = re.search(r"-mesh=(\d+)x(\d+)", s)
    if m:
        mesh = (int(m.group(1)), int(m.group(2)))
    m2 = re.search(r"device_mesh_nrow_(\d+),device_mesh_ncol_(\d+)", s)
    if m2:
        mesh = (int(m2.group(1)), int(m2.group(2)))
    head = s.split()[0] if s else "auto"
    if head == "auto":
        head = "hip" if check_hip_availability() else "cpu"
    if head in ("hip", "rocm"):
        arch = GFX950
        m3 = re.search(r"-mcpu=(\S+)", s)
        if m3 and m3.group(1) != GFX950:
            raise ValueError(f"this framework generates code for gfx950 (MI355X) only, got {m3.group(1)}")
        t = Target("hip", arch, mesh)
    elif head in ("cpu", "c", "llvm"):
        t = Target("cpu", "host", mesh)
    elif head.lower() == "sunmmio":
        t = Target("cpu", "host", mesh or (4, 4))
    elif head in ("cuda", "metal", "webgpu"):
        raise ValueError(f"target {head!r} is not supported: this is an MI355X-native framework (hip/gfx950 + cpu)")
    else:
        raise ValueError(f"unknown target {target!r}; supported: {sorted(SUPPORTED_TARGETS)}")
    return t if return_object else str(t)


def target_is_hip(t) -> bool:
    return determine_target(t).kind == "hip"


def target_is_cpu(t) -> bool:
    return determine_target(t).kind == "cpu"


def target_get_warp_size(t=None) -> int:
    return 64
