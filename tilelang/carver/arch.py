"""Device models for the tile-config recommender (reference ``tilelang/carver/arch/{arch_base,cdna}.py``).

``CDNA`` describes one MI355X (gfx950).  Values come from the device when a GPU is visible
(``torch.cuda.get_device_properties``) and from the CDNA4 data sheet otherwise, so hints can be
computed on a build machine without a GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List


@dataclass
class TileDevice:
    platform: str = "generic"
    compute_max_core: int = 1           # CUs
    warp_size: int = 64
    smem_cap: int = 64 * 1024           # LDS bytes per workgroup
    reg_cap: int = 512 * 64             # VGPR+AGPR per wave x lanes
    max_waves_per_simd: int = 8
    simds_per_core: int = 4
    l2_cache_size_bytes: int = 4 << 20
    bandwidth: List[int] = field(default_factory=lambda: [8000, 40000])  # GB/s: HBM, L2
    peak_tflops: dict = field(default_factory=dict)
    transaction_size: List[int] = field(default_factory=lambda: [64, 128])
    clock_ghz: float = 2.4
    num_xcds: int = 1

    def get_avaliable_tensorintrin_shapes(self):
        return [(16, 16, 32), (32, 32, 16)]

    # reference spelling kept for API compatibility
    get_available_tensorintrin_shapes = get_avaliable_tensorintrin_shapes


class CDNA(TileDevice):
    """AMD Instinct MI355X (CDNA4, gfx950): 256 CUs in 8 XCDs, 160 KiB LDS per CU, wave64,
    dense MFMA ~2.5 PF fp16/bf16 and ~5 PF fp8, HBM3E ~8 TB/s."""

    def __init__(self, target="hip"):
        super().__init__(platform="CDNA", compute_max_core=256, warp_size=64, smem_cap=160 * 1024,
                         reg_cap=512 * 64, l2_cache_size_bytes=4 << 20, bandwidth=[8000, 60000],
                         peak_tflops={"float16": 2500.0, "bfloat16": 2500.0, "float8_e4m3fn": 5000.0,
                                      "float8_e5m2": 5000.0, "int8": 5000.0, "float32": 157.0},
                         clock_ghz=2.4, num_xcds=8)
        self.target = target
        self.arch = "gfx950"
        try:
            import torch
            if torch.cuda.is_available():
                p = torch.cuda.get_device_properties(0)
                self.compute_max_core = int(p.multi_processor_count)
                self.arch = getattr(p, "gcnArchName", "gfx950").split(":")[0]
        except Exception:  # noqa: BLE001 - no device: keep the data-sheet values
            pass
        self.sm_partition = self.simds_per_core
        self.max_smem_usage = self.smem_cap

    def __repr__(self):
        return f"CDNA({self.arch}, CUs={self.compute_max_core}, LDS={self.smem_cap // 1024}KiB)"


class CPU(TileDevice):

    def __init__(self, target="cpu"):
        import os
        super().__init__(platform="CPU", compute_max_core=os.cpu_count() or 1, warp_size=1, smem_cap=1 << 20,
                         bandwidth=[100, 400], peak_tflops={"float32": 1.0})
        self.target = target


def is_cdna_arch(arch) -> bool:
    return isinstance(arch, CDNA)


def auto_infer_current_arch() -> TileDevice:
    return CDNA("hip")


__all__ = ["TileDevice", "CDNA", "CPU", "is_cdna_arch", "auto_infer_current_arch"]
