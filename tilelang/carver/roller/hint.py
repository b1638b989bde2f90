"""A recommended configuration (reference ``tilelang/carver/roller/hint.py``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

from .rasterization import NoRasterization, Rasterization


@dataclass
class Hint:
    block: List[int] = field(default_factory=list)       # tile extents of the output (e.g. [bm, bn])
    warp: List[int] = field(default_factory=list)        # per-wave tile extents
    rstep: List[int] = field(default_factory=list)       # reduction step(s) (block_K)
    pipeline_stage: int = 2
    threads: int = 256
    use_tc: bool = True
    rasterization_plan: Rasterization = field(default_factory=NoRasterization)
    estimated_us: float = 0.0
    score: Dict[str, float] = field(default_factory=dict)
    extra: Dict[str, int] = field(default_factory=dict)

    @property
    def warp_partition(self) -> Tuple[int, int]:
        return tuple(b // w for b, w in zip(self.block, self.warp))

    def to_config(self) -> Dict[str, int]:
        """The keyword arguments the examples' kernel factories take."""
        if (len(self.block) == 1 or "blk_m" in self.extra) and self.extra:
            # families that name their own tile keys (GEMV: block_N/block_K, row reductions: blk_m)
            return dict(self.extra, threads=self.threads)
        cfg = {"block_M": self.block[0], "threads": self.threads, "num_stages": self.pipeline_stage}
        if len(self.block) > 1:
            cfg["block_N"] = self.block[1]
        if self.rstep:
            cfg["block_K"] = self.rstep[0]
        if self.rasterization_plan.panel_width:  # T.use_swizzle(panel_size=...) of the plan
            cfg["panel_size"] = self.rasterization_plan.panel_width
        cfg.update(self.extra)
        return cfg

    def __repr__(self):
        return (f"Hint(block={self.block}, warp={self.warp}, rstep={self.rstep}, stages={self.pipeline_stage}, "
                f"threads={self.threads}, raster={self.rasterization_plan}, est={self.estimated_us:.1f}us)")
