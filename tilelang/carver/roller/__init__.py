"""Analytical tile-config search ("roller", reference ``tilelang/carver/roller``) for CDNA4.

Instead of the reference's BitBLAS-derived TensorCore policy over TVM compute DAGs, the
policy here enumerates the tile shapes the gfx950 lowering supports (MFMA 16x16x32 fragments,
wave64 partitions, LDS-DMA rings) and ranks them with a roofline + wave-quantisation model of
the MI355X (256 CUs, 160 KiB LDS, 512 VGPR+AGPR per wave)."""
from .hint import Hint  # noqa: F401
from .policy import DefaultPolicy, TensorCorePolicy, gemm_cost  # noqa: F401
from . import rasterization  # noqa: F401
