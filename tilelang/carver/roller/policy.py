"""CDNA4 tile-config policies (reference ``tilelang/carver/roller/policy/{default,tensorcore}.py``).

``TensorCorePolicy`` ranks GEMM-shaped tilings with an MI355X model:

* MFMA peak per CU = peak / CUs (4096 fp16 FLOP/clk/CU at 2.4 GHz);
* LDS feed: a wave computing a ``wm x wn`` tile reads ``(wm + wn) * bk`` operand elements
  per ``2 * wm * wn * bk`` FLOPs through ds_read_b128 at 128 B/clk/CU, so small wave tiles
  are LDS-bound (64x64 per wave is the break-even point for fp16);
* latency hiding from resident waves (LDS / accumulator-register limited occupancy);
* HBM traffic with L2 reuse inside a rasterisation panel, and wave quantisation over the CUs.

``DefaultPolicy`` sizes memory-bound (elementwise / GEMV / reduction) tiles for 16-byte
lanes and enough blocks to cover every CU several times.
"""
from __future__ import annotations

import itertools
import math
from typing import List, Optional, Sequence

from .bestfit import gemm_lds_bytes
from .hint import Hint
from .rasterization import NoRasterization, Rasterization2DRow, l2_panel_width

_EB = {"float16": 2, "bfloat16": 2, "float8_e4m3fn": 1, "float8_e5m2": 1, "int8": 1, "float32": 4, "float": 4}


def _eb(dtype) -> int:
    return _EB.get(str(dtype), 2)


# Sustained MFMA efficiency (fraction of the dense peak, one workgroup per CU, large K) of the main
# loop the compiler emits for a tiling, fitted to measured kernels on MI355X:
#   quad  -- tl::gemm_quad_nt_x (256x256, 128-byte K tiles, 512 threads, 2 stages, B [N, K]):
#            fp16 4096^3 1309-1311 TF, 8192^2x4096 1351 (profiles/r5/benchmarks/matmul_fp16.md,
#            docs/RESULTS.md round 5); fp8 8192^2 x 4096 2533 TF of 5000 (RESULTS r5 fp8 table)
#   phased -- the K-half register-prefetched schedule (256x256x64 fp16, 512 threads, 2 stages, B
#            [K, N]): 1179 TF NT before the quad loop, 1210-1227 NN (RESULTS r4 / r5)
#   generic -- the LDS-DMA ring + T.gemm per K step: 128x256x64 / 512 threads 1001 TF, 256x128x64
#            / 512 910, 256x128x64 / 256 827 at 4096^3 (profiles/r3/s3/gemm/tile_shape_sweep.log)
LOOP_EFF = {"quad": 0.578, "quad_fp8": 0.625, "phased": 0.525, "generic": 0.40}
# per-tile fixed cost (prologue fill + C epilogue), fitted to the K sweep of the quad loop at
# M = N = 8192 (K 256 ... 16384: 557 ... 1339 TF, profiles/r5/benchmarks/matmul_fp16.md): 9.4 us
# per 256x256 tile round = (C tile + two K stages of A and B) bytes at ~25 GB/s per CU
_PER_CU_BW = 25e9


def main_loop_kind(bm, bn, bk, threads, stages, in_dtype="float16", trans_b=True) -> str:
    """The main loop transform/gemm_ksplit.py + pipeline.py select for this tiling (quad_loop_ok /
    the phased K-half schedule), or 'generic'."""
    eb = _eb(in_dtype)
    if bm == 256 and bn == 256 and threads == 512 and stages == 2 and bk * eb == 128 and trans_b and \
            str(in_dtype) in ("float16", "bfloat16", "float8_e4m3fn", "float8_e5m2"):
        return "quad_fp8" if eb == 1 else "quad"
    if bm == 256 and bn == 256 and threads == 512 and stages == 2 and bk == 64 and eb == 2:
        return "phased"
    return "generic"


def gemm_cost(arch, M, N, K, bm, bn, bk, threads, stages, in_dtype="float16", warp=None,
              trans_b=True) -> Optional[dict]:
    """Modelled time (us) of one tiling, or None if it does not fit the hardware.

    time = rounds x (fixed + tile FLOPs / (per-CU peak x eff / blocks per CU)), with ``eff`` the
    measured efficiency of the main loop the compiler emits for the tiling (``LOOP_EFF``), scaled
    for the generic loop by the wave tile's LDS feed and the resident waves, and ``fixed`` the
    per-tile prologue + epilogue bytes at the per-CU share of HBM bandwidth."""
    eb = _eb(in_dtype)
    waves = threads // 64
    if threads % 64 or waves not in (1, 2, 4, 8, 16):
        return None
    if bk * eb < 32 or (bk * eb) % 64 and eb == 1:
        return None
    lds = gemm_lds_bytes(bm, bn, bk, stages, eb)  # best-fit arena (roller/bestfit.py)
    if lds > arch.smem_cap:
        return None
    acc_regs = bm * bn // threads  # fp32 accumulators per lane
    if acc_regs > 256 or acc_regs < 4:
        return None
    if warp is None:
        from ...layout.mfma import compute_warp_partition
        try:
            wpm, wpn = compute_warp_partition(bm, bn, waves, 0)
        except Exception:  # noqa: BLE001
            return None
        wm, wn = bm // wpm, bn // wpn
    else:
        wm, wn = warp
    if wm < 16 or wn < 16:
        return None
    per_cu_flops = arch.peak_tflops.get(str(in_dtype), 2500.0) * 1e12 / arch.compute_max_core
    kind = main_loop_kind(bm, bn, bk, threads, stages, in_dtype, trans_b)
    eff = LOOP_EFF[kind]
    # residency: LDS, registers (accumulators + ~64 operand/address VGPRs of the 512 per lane)
    # and the 8-waves-per-SIMD cap
    waves_per_simd_by_regs = min(8, 512 // (acc_regs + 64))
    blocks_by_regs = (waves_per_simd_by_regs * 4) // waves
    blocks_per_cu = max(1, min(arch.smem_cap // max(lds, 1), blocks_by_regs, 32 // waves))
    resident_waves = blocks_per_cu * waves
    if kind == "generic":
        # LDS feed of the wave tile (operand bytes per MFMA FLOP; 64x64 per wave is the measured
        # break-even), latency hiding by resident waves (8 per CU measured: 256x128 / 256 threads
        # ran 0.91x the 512-thread tile), one stage less of DMA in flight
        lds_feed = min(1.0, (wm * wn / (wm + wn)) / 32.0)
        occ = 0.87 + 0.13 * min(1.0, resident_waves / 8.0)
        eff *= lds_feed * occ * (1.0 if stages >= 2 else 0.75)
    tiles_m, tiles_n = math.ceil(M / bm), math.ceil(N / bn)
    n_tiles = tiles_m * tiles_n
    # blocks that actually share a CU: a grid smaller than CUs x residency leaves CUs to spare
    sharing = max(1, min(blocks_per_cu, math.ceil(n_tiles / arch.compute_max_core)))
    concurrent = arch.compute_max_core * blocks_per_cu
    rounds = math.ceil(n_tiles / concurrent)
    tile_flops = 2.0 * bm * bn * K
    fixed = (bm * bn * 2 + stages * (bm + bn) * bk * eb) / (_PER_CU_BW / sharing)
    t_tile = fixed + tile_flops / (per_cu_flops * eff / sharing)
    t_compute = rounds * t_tile
    # memory: compulsory bytes (A, B once, C) at the HBM rate; the operand re-reads of the other
    # tile rows / columns come from L2 and the 256 MiB Infinity Cache while A + B fit in it
    unique = (M * K + N * K) * eb + M * N * 2
    # (past the cache: the XCD-aware rasterisation's 8-tile panels keep 7 of 8 re-reads in L2)
    panel = 8 if n_tiles > arch.compute_max_core else 1
    rereads = (M * K * max(0, tiles_n - 1) + N * K * max(0, tiles_m - 1)) * eb
    if (M * K + N * K) * eb <= (192 << 20):
        t_mem = unique / (arch.bandwidth[0] * 1e9) + rereads / (arch.bandwidth[1] * 1e9)
    else:
        t_mem = (unique + rereads / panel) / (arch.bandwidth[0] * 1e9) + rereads / (arch.bandwidth[1] * 1e9)
    t = max(t_compute, t_mem)
    return dict(us=t * 1e6, eff=eff, loop=kind, occ=resident_waves, rounds=rounds, warp=(wm, wn),
                raster=panel > 1, lds_bytes=lds, t_compute_us=t_compute * 1e6, t_mem_us=t_mem * 1e6)


class TensorCorePolicy:

    def __init__(self, arch, M, N, K, in_dtype="float16", trans_b=False):
        self.arch, self.M, self.N, self.K = arch, M, N, K
        self.in_dtype = in_dtype
        self.trans_b = trans_b

    def candidates(self):
        bms = [b for b in (32, 64, 128, 256) if b <= max(32, self.M * 2)]
        bns = [b for b in (32, 64, 128, 256) if b <= max(32, self.N * 2)]
        eb = _eb(self.in_dtype)
        # a ragged K is fine (the quad loop zero-fills its last K tile; the generic loop pads)
        bks = [b for b in ((32, 64, 128) if eb == 2 else (64, 128, 256)) if b <= max(64, self.K)]
        return itertools.product(bms, bns, bks, (256, 512), (2, 3))

    def emit_config(self, topk: int = 10) -> List[Hint]:
        hints = []
        for bm, bn, bk, th, st in self.candidates():
            c = gemm_cost(self.arch, self.M, self.N, self.K, bm, bn, bk, th, st, self.in_dtype,
                          trans_b=self.trans_b)
            if c is None:
                continue
            pw = l2_panel_width(self.M, self.N, self.K, bm, bn, _eb(self.in_dtype), cus=self.arch.compute_max_core)
            hints.append(Hint(block=[bm, bn], warp=list(c["warp"]), rstep=[bk], pipeline_stage=st, threads=th,
                              rasterization_plan=Rasterization2DRow(pw) if c["raster"] else NoRasterization(),
                              estimated_us=c["us"], score=c))
        hints.sort(key=lambda h: (h.estimated_us, -h.block[0] * h.block[1]))
        return hints[:topk]


class DefaultPolicy:
    """Memory-bound tiles: ``shape`` is the output iteration space, ``reduce_len`` the per-output
    reduction length (GEMV / row reductions), 0 for elementwise."""

    def __init__(self, arch, shape: Sequence[int], dtype="float16", reduce_len: int = 0, bytes_per_elem=None):
        self.arch = arch
        self.shape = list(shape)
        self.dtype = dtype
        self.reduce_len = reduce_len
        self.eb = bytes_per_elem or _eb(dtype)

    def emit_config(self, topk: int = 10) -> List[Hint]:
        vec = max(1, 16 // self.eb)
        total = 1
        for s in self.shape:
            total *= s
        hints = []
        rows = self.shape[0] if len(self.shape) > 1 else 1
        cols = self.shape[-1]
        for th in (128, 256, 512):
            for bm in (1, 2, 4, 8, 16, 32, 64):
                if bm > rows:
                    continue
                for bn in (64, 128, 256, 512, 1024, 2048):
                    if bn > max(cols, vec) or (bm * bn) % (th * vec) and bm * bn >= th * vec:
                        continue
                    blocks = math.ceil(rows / bm) * math.ceil(cols / bn)
                    cover = blocks / (self.arch.compute_max_core * max(1, 2048 // th))
                    per_lane = bm * bn / th
                    if per_lane > 64 or per_lane < 1:
                        continue
                    moved = total * self.eb * (2 if not self.reduce_len else 1) + (
                        total * self.reduce_len * self.eb if self.reduce_len else 0)
                    t = moved / (self.arch.bandwidth[0] * 1e9) * 1e6
                    # under-filled chips and long per-lane serial chains both cost bandwidth
                    t /= min(1.0, 0.3 + 0.7 * min(1.0, cover)) * (1.0 if per_lane <= 32 else 0.8)
                    hints.append(Hint(block=[bm, bn], warp=[bm, bn], rstep=[], pipeline_stage=1, threads=th,
                                      estimated_us=t, score=dict(blocks=blocks, cover=cover)))
        hints.sort(key=lambda h: (h.estimated_us, -h.threads))
        return hints[:topk]
