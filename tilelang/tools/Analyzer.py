"""Static roofline analyzer (reference ``tilelang/tools/Analyzer.py``; its ARCH_CONFIGS are NVIDIA-only).

Walks a ``T.prim_func`` before lowering and counts, per ``T.Kernel``:
  * MFMA FLOPs of every ``T.gemm`` (2*M*N*K per call x trip counts of the enclosing loops x grid),
  * global-memory bytes moved by ``T.copy`` / atomics between global and on-chip buffers,
then reports the roofline-bound time on an MI355X (or any ``ARCH_CONFIGS`` entry).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.expr import as_int

ARCH_CONFIGS: Dict[str, dict] = {
    # dense (no 2:4 sparsity) MFMA peaks; HBM3E bandwidth
    "MI355X": dict(fp16_tflops=2500.0, bf16_tflops=2500.0, fp8_tflops=5000.0, fp32_tflops=157.0,
                   hbm_gbs=8000.0, cus=256, lds_kib=160),
    "MI300X": dict(fp16_tflops=1307.0, bf16_tflops=1307.0, fp8_tflops=2615.0, fp32_tflops=163.0,
                   hbm_gbs=5300.0, cus=304, lds_kib=64),
}


@dataclass
class AnalysisResult:
    total_flops: float
    total_global_bytes: float
    estimated_time_us: float
    expected_tflops: float
    expected_bandwidth_GBps: float
    bound: str

    def __repr__(self):
        return (f"AnalysisResult(flops={self.total_flops:.3e}, global_bytes={self.total_global_bytes:.3e}, "
                f"est={self.estimated_time_us:.1f}us ({self.bound}-bound), "
                f"{self.expected_tflops:.1f} TFLOPS, {self.expected_bandwidth_GBps:.0f} GB/s)")


def _trip(s) -> Optional[int]:
    mn, ext = as_int(s.min), as_int(s.extent)
    return ext if ext is not None else None


def _region_bytes(r) -> int:
    ext = r.static_extents()
    if ext is None:
        return 0
    n = 1
    for e in ext:
        n *= e
    return n * r.buffer.dtype.bytes


class Analyzer:

    def __init__(self, func: S.PrimFunc, arch: str = "MI355X"):
        self.func = func
        self.arch = ARCH_CONFIGS[arch if isinstance(arch, str) else "MI355X"]  # or a carver TileDevice
        self.flops = 0.0
        self.bytes = 0.0
        self.dtype_bits = 16

    def _walk(self, s, mult: float):
        if s is None:
            return
        if isinstance(s, S.KernelStmt):
            g = 1
            for e in s.grid:
                v = as_int(e)
                g *= v if v is not None else 1
            self._walk(s.body, mult * g)
            return
        if isinstance(s, S.ForStmt):
            t = _trip(s)
            self._walk(s.body, mult * (t if t is not None else 1))
            return
        if isinstance(s, S.TileOpStmt):
            op = s.op
            if isinstance(op, O.GemmOp):
                from ..transform.gemm_lower import _trailing2
                a, c = _trailing2(op.A), _trailing2(op.C)
                K = a[0] if op.trans_A else a[1]
                self.flops += mult * 2.0 * c[0] * c[1] * K
                self.dtype_bits = op.A.buffer.dtype.bits
            elif isinstance(op, (O.CopyOp, O.AtomicOp)):
                for r in (getattr(op, "src", None), getattr(op, "dst", None)):
                    if r is not None and hasattr(r, "buffer") and r.buffer.scope == "global":
                        self.bytes += mult * _region_bytes(r)
            return
        for c in S.stmt_children(s):
            self._walk(c, mult)

    def analyze(self) -> AnalysisResult:
        self._walk(self.func.body, 1.0)
        peak = {8: self.arch["fp8_tflops"], 16: self.arch["fp16_tflops"]}.get(self.dtype_bits,
                                                                              self.arch["fp32_tflops"])
        t_c = self.flops / (peak * 1e12)
        t_m = self.bytes / (self.arch["hbm_gbs"] * 1e9)
        t = max(t_c, t_m, 1e-12)
        return AnalysisResult(self.flops, self.bytes, t * 1e6, self.flops / t * 1e-12, self.bytes / t * 1e-9,
                              "compute" if t_c >= t_m else "memory")

    @classmethod
    def analysis(cls, func, arch: str = "MI355X") -> AnalysisResult:
        return cls(func, arch).analyze()


__all__ = ["Analyzer", "AnalysisResult", "ARCH_CONFIGS"]
