"""Operator templates for the config recommender (reference ``tilelang/carver/template/*.py``).

Each template describes one operator family; ``.with_arch(arch).recommend_hints(topk)``
returns ranked ``Hint`` objects whose ``to_config()`` matches the keyword arguments of the
corresponding example kernel factory (``examples/gemm``, ``examples/gemv``, ...).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

from .arch import CDNA, TileDevice
from .roller.hint import Hint
from .roller.policy import DefaultPolicy, TensorCorePolicy


@dataclass
class BaseTemplate:
    arch: Optional[TileDevice] = field(default=None, init=False)

    def with_arch(self, arch):
        self.arch = arch
        return self

    def has_arch(self) -> bool:
        return self.arch is not None

    def recommend_hints(self, topk: int = 10) -> List[Hint]:
        if self.arch is None:
            self.arch = CDNA("hip")
        return self._hints(topk)

    def equivalent_function(self):
        """The reference returns a TIR compute definition; here: the PyTorch semantics."""
        return self.reference

    def _hints(self, topk):
        raise NotImplementedError


@dataclass
class MatmulTemplate(BaseTemplate):
    M: int = 1024
    N: int = 1024
    K: int = 1024
    trans_A: bool = False
    trans_B: bool = True
    in_dtype: str = "float16"
    out_dtype: str = "float16"
    accum_dtype: str = "float"
    with_bias: bool = False

    def _hints(self, topk):
        return TensorCorePolicy(self.arch, self.M, self.N, self.K, self.in_dtype, self.trans_B).emit_config(topk)

    def reference(self, A, B):
        return A @ (B.t() if self.trans_B else B)


@dataclass
class GEMVTemplate(BaseTemplate):
    N: int = 1024
    K: int = 1024
    in_dtype: str = "float16"
    out_dtype: str = "float16"
    accum_dtype: str = "float"

    def _hints(self, topk):
        hs = DefaultPolicy(self.arch, [self.N, self.K], self.in_dtype, reduce_len=1).emit_config(topk * 4)
        out = []
        for h in hs:
            h.extra = {}
            out.append(Hint(block=[h.block[0]], warp=[h.block[0]], rstep=[h.block[1]], pipeline_stage=1,
                            threads=h.threads, estimated_us=h.estimated_us,
                            extra={"block_N": h.block[0], "block_K": h.block[1]}))
        return out[:topk]

    def reference(self, A, x):
        return A @ x


@dataclass
class ElementwiseTemplate(BaseTemplate):
    shape: List[int] = field(default_factory=lambda: [1024, 1024])
    dtype: str = "float16"

    def _hints(self, topk):
        return DefaultPolicy(self.arch, self.shape, self.dtype).emit_config(topk)

    def reference(self, a, b):
        return a + b


@dataclass
class GeneralReductionTemplate(BaseTemplate):
    """Row reductions (``structure="SR"``: spatial rows x reduced columns) with whole rows held in
    registers -- the shape of RMS norm / softmax / row sums (``examples/norm/rms_norm.py``:
    ``to_config()`` gives its ``blk_m`` and ``threads``).  Model: one HBM read + one write of the
    rows at the HBM rate, derated when the grid under-fills the 256 CUs (fewer than ~4 blocks per
    CU) and when a lane carries long serial chains; tiles whose rows do not fit the register
    budget (64 fp32 per lane) are rejected."""
    structure: str = "SR"  # spatial x reduce
    shape: List[int] = field(default_factory=lambda: [1024, 1024])
    dtype: str = "float16"

    def _hints(self, topk):
        import math
        from .roller.policy import _eb
        rows, cols = self.shape[0], self.shape[-1]
        eb = _eb(self.dtype)
        hints = []
        for th in (128, 256, 512):
            for bm in (1, 2, 4, 8, 16, 32):
                if bm > rows or th % bm:
                    continue
                per_lane = bm * cols / th
                if per_lane > 64 or per_lane < 1 or (th // bm) * max(1, 16 // eb) > cols * 4:
                    continue
                blocks = math.ceil(rows / bm)
                cover = blocks / (self.arch.compute_max_core * 4)
                t = 2 * rows * cols * eb / (self.arch.bandwidth[0] * 1e9) * 1e6
                t /= min(1.0, 0.3 + 0.7 * min(1.0, cover)) * (1.0 if per_lane <= 32 else 0.85)
                hints.append(Hint(block=[bm, cols], warp=[bm, cols], rstep=[cols], pipeline_stage=1, threads=th,
                                  estimated_us=t, score=dict(blocks=blocks, per_lane=per_lane),
                                  extra={"blk_m": bm}))
        hints.sort(key=lambda h: (h.estimated_us, -h.threads))
        return hints[:topk]

    def reference(self, x):
        return x.sum(-1)


@dataclass
class FlashAttentionTemplate(BaseTemplate):
    batch: int = 1
    heads: int = 8
    seq_len: int = 4096
    dim: int = 128
    causal: bool = False
    in_dtype: str = "bfloat16"

    def _hints(self, topk):
        from .roller.policy import gemm_cost
        hints = []
        for bm in (64, 128, 256):
            for bn in (32, 64, 128):
                for th in (256, 512):
                    waves = th // 64
                    if bm // waves < 16:
                        continue
                    eb = 2
                    lds = bm * self.dim * eb + 2 * 2 * bn * self.dim * eb
                    if lds > self.arch.smem_cap:
                        continue
                    # S = Q K^T then O = P V, both with per-wave tiles (bm / waves) x (bn | dim)
                    c1 = gemm_cost(self.arch, self.seq_len * self.heads * self.batch, self.seq_len, self.dim, bm, bn,
                                   32, th, 2, self.in_dtype, warp=(bm // waves, bn))
                    if c1 is None:
                        continue
                    t = 2 * c1["t_compute_us"] * (0.5 if self.causal else 1.0)
                    hints.append(Hint(block=[bm, bn], warp=[bm // waves, bn], rstep=[self.dim], pipeline_stage=2,
                                      threads=th, estimated_us=t, score=c1))
        hints.sort(key=lambda h: h.estimated_us)
        return hints[:topk]

    def reference(self, q, k, v):
        import torch
        return torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=self.causal)


@dataclass
class ConvTemplate(BaseTemplate):
    N: int = 128
    C: int = 128
    H: int = 64
    W: int = 64
    F: int = 128
    K: int = 3
    S: int = 1
    D: int = 1
    P: int = 1
    in_dtype: str = "float16"

    def _hints(self, topk):
        OH = (self.H + 2 * self.P - self.D * (self.K - 1) - 1) // self.S + 1
        OW = (self.W + 2 * self.P - self.D * (self.K - 1) - 1) // self.S + 1
        return TensorCorePolicy(self.arch, self.N * OH * OW, self.F, self.K * self.K * self.C,
                                self.in_dtype).emit_config(topk)

    def reference(self, a, b):
        import torch
        return torch.conv2d(a, b, stride=self.S, padding=self.P, dilation=self.D)


__all__ = ["BaseTemplate", "MatmulTemplate", "GEMVTemplate", "ElementwiseTemplate", "GeneralReductionTemplate",
           "FlashAttentionTemplate", "ConvTemplate"]
