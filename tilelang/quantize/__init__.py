"""Low-bit weight formats: packing on the host (PyTorch) and dequantisation expressions for use
inside kernels (reference ``tilelang/quantize/{quantization,mxfp,utils}.py``).

Formats (gfx950-relevant):
  * int4 (signed, two per byte, low nibble first) with group-wise scales  (W4A16 GEMM);
  * fp4 e2m1 (OCP MX) with e8m0 block scales (MXFP4, 32 elements per scale) -- the operand
    format of the gfx950 ``v_mfma_scale_f32_*_f8f6f4`` instructions;
  * e8m0 scales (power-of-two, bias 127).

The DSL helpers return ``PrimExpr``s, e.g. inside ``T.Parallel``::

    B_shared[n, k] = T.Cast("float16", Q.int4_to_float(Bq_shared[n, k // 2], k % 2) * scale)
"""
from __future__ import annotations

from typing import Tuple

# ---------------------------------------------------------------------------------------------
# DSL expressions
# ---------------------------------------------------------------------------------------------


def _T():
    import tilelang.language as T
    return T


def int4_to_float(byte, hi):
    """Signed int4 nibble ``hi`` (0 = low, 1 = high; may be an expression) of ``byte`` as fp32."""
    T = _T()
    nib = (byte >> (hi * 4)) & 15
    return T.Cast("float32", T.Cast("int32", nib) - T.if_then_else(nib >= 8, 16, 0))


def uint4_to_float(byte, hi, zero=8):
    """Unsigned int4 with a zero point (AWQ/GPTQ style)."""
    T = _T()
    nib = (byte >> (hi * 4)) & 15
    return T.Cast("float32", T.Cast("int32", nib) - zero)


def e2m1_to_float(nib):
    """OCP fp4 e2m1 -> fp32: magnitudes {0, .5, 1, 1.5, 2, 3, 4, 6} with a sign bit."""
    T = _T()
    e = (nib >> 1) & 3
    m = nib & 1
    mag = T.if_then_else(e == 0, T.Cast("float32", m) * 0.5,
                         T.exp2(T.Cast("float32", e) - 1.0) * (1.0 + T.Cast("float32", m) * 0.5))
    return T.if_then_else((nib & 8) != 0, -mag, mag)


def fp4_to_float(byte, hi):
    return e2m1_to_float((byte >> (hi * 4)) & 15)


def e8m0_to_float(byte):
    """e8m0 block scale -> fp32 (2^(byte - 127))."""
    T = _T()
    return T.exp2(T.Cast("float32", byte) - 127.0)


# ---------------------------------------------------------------------------------------------
# host-side packing (PyTorch)
# ---------------------------------------------------------------------------------------------


def pack_int4(q):
    """int tensor in [-8, 7] of shape [..., K] -> uint8 [..., K/2] (low nibble = even k)."""
    import torch
    u = (q.to(torch.int32) & 0xF).to(torch.uint8)
    return (u[..., 0::2] | (u[..., 1::2] << 4)).contiguous()


def unpack_int4(packed):
    import torch
    lo = (packed & 0xF).to(torch.int32)
    hi = (packed >> 4).to(torch.int32)
    q = torch.stack([lo, hi], -1).flatten(-2)
    return q - (q >= 8).to(torch.int32) * 16


def quantize_int4_groupwise(W, group_size: int = 128) -> Tuple:
    """Symmetric int4 with one scale per ``group_size`` along the last dim."""
    import torch
    shp = W.shape
    g = W.float().reshape(*shp[:-1], shp[-1] // group_size, group_size)
    scales = (g.abs().amax(-1) / 7.0).clamp(min=1e-8)
    q = torch.clamp(torch.round(g / scales.unsqueeze(-1)), -8, 7).reshape(shp)
    return pack_int4(q), scales.to(W.dtype)


def dequantize_int4_groupwise(packed, scales, group_size: int = 128):
    q = unpack_int4(packed).float()
    shp = q.shape
    g = q.reshape(*shp[:-1], shp[-1] // group_size, group_size)
    return (g * scales.float().unsqueeze(-1)).reshape(shp)


_E2M1 = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0]


def float_to_e2m1(x):
    """Round-to-nearest onto the e2m1 grid (saturating at 6); returns uint8 codes."""
    import torch
    grid = torch.tensor(_E2M1, device=x.device)
    mag = x.abs().clamp(max=6.0)
    code = (mag.unsqueeze(-1) - grid).abs().argmin(-1).to(torch.uint8)
    return code | ((x < 0).to(torch.uint8) << 3)


def e2m1_to_float_torch(code):
    import torch
    grid = torch.tensor(_E2M1, device=code.device)
    mag = grid[(code & 7).long()]
    return torch.where((code & 8) != 0, -mag, mag)


def quantize_mxfp4(W, block: int = 32) -> Tuple:
    """OCP MXFP4: per 32 elements an e8m0 scale 2^floor(log2(amax)) - 2 (so amax/scale <= 6)."""
    import torch
    shp = W.shape
    g = W.float().reshape(*shp[:-1], shp[-1] // block, block)
    amax = g.abs().amax(-1).clamp(min=2.0**-126)
    e = torch.floor(torch.log2(amax)) - 2
    scale = torch.exp2(e)
    codes = float_to_e2m1(g / scale.unsqueeze(-1)).reshape(shp)
    packed = (codes[..., 0::2] | (codes[..., 1::2] << 4)).contiguous()
    return packed, (e + 127).clamp(0, 254).to(torch.uint8)


def dequantize_mxfp4(packed, scales_e8m0, block: int = 32):
    import torch
    lo = e2m1_to_float_torch(packed & 0xF)
    hi = e2m1_to_float_torch(packed >> 4)
    v = torch.stack([lo, hi], -1).flatten(-2)
    shp = v.shape
    s = torch.exp2(scales_e8m0.float() - 127.0)
    return (v.reshape(*shp[:-1], shp[-1] // block, block) * s.unsqueeze(-1)).reshape(shp)


def fp6_grid(fmt: str):
    """The non-negative values of an OCP fp6 format, indexed by the 5-bit magnitude code:
    e2m3 (bias 1, max 7.5) or e3m2 (bias 3, max 28); subnormals at exponent 0, no inf/nan."""
    if fmt == "e2m3":
        eb, mb, bias = 2, 3, 1
    elif fmt == "e3m2":
        eb, mb, bias = 3, 2, 3
    else:
        raise ValueError(f"fp6 format must be 'e2m3' or 'e3m2', got {fmt!r}")
    out = []
    for code in range(32):
        e, m = code >> mb, code & ((1 << mb) - 1)
        if e == 0:
            out.append(m / (1 << mb) * 2.0**(1 - bias))
        else:
            out.append((1 + m / (1 << mb)) * 2.0**(e - bias))
    return out


def float_to_fp6(x, fmt: str):
    """Round-to-nearest onto the fp6 grid (saturating); uint8 codes, bit 5 = sign."""
    import torch
    grid = torch.tensor(fp6_grid(fmt), device=x.device)
    mag = x.abs().clamp(max=grid[-1].item())
    code = (mag.unsqueeze(-1) - grid).abs().argmin(-1).to(torch.uint8)
    return code | ((x < 0).to(torch.uint8) << 5)


def fp6_to_float_torch(code, fmt: str):
    import torch
    grid = torch.tensor(fp6_grid(fmt), device=code.device)
    mag = grid[(code & 31).long()]
    return torch.where((code & 32) != 0, -mag, mag)


def pack_fp6(codes):
    """``[..., K]`` 6-bit codes -> ``[..., 3K/4]`` bytes: a little-endian bit stream, element k at
    bits 6k..6k+5 of its row (4 elements per 3 bytes)."""
    import torch
    c = codes.to(torch.int32)
    shp = c.shape
    if shp[-1] % 4:
        raise ValueError(f"pack_fp6: the last dim ({shp[-1]}) must be a multiple of 4")
    q = c.reshape(*shp[:-1], shp[-1] // 4, 4)
    w = q[..., 0] | (q[..., 1] << 6) | (q[..., 2] << 12) | (q[..., 3] << 18)
    b = torch.stack([w & 255, (w >> 8) & 255, (w >> 16) & 255], -1)
    return b.reshape(*shp[:-1], shp[-1] // 4 * 3).to(torch.uint8).contiguous()


def unpack_fp6(packed):
    import torch
    b = packed.to(torch.int32)
    shp = b.shape
    t = b.reshape(*shp[:-1], shp[-1] // 3, 3)
    w = t[..., 0] | (t[..., 1] << 8) | (t[..., 2] << 16)
    q = torch.stack([(w >> (6 * i)) & 63 for i in range(4)], -1)
    return q.reshape(*shp[:-1], shp[-1] // 3 * 4).to(torch.uint8)


def quantize_mxfp6(W, fmt: str = "e2m3", block: int = 32) -> Tuple:
    """OCP MXFP6: per 32 elements an e8m0 scale 2^(floor(log2(amax)) - emax) with emax the
    format's largest exponent (2 for e2m3, 4 for e3m2), elements rounded to the fp6 grid and
    packed with ``pack_fp6``.  Returns (packed bytes ``[..., 3K/4]``, scales ``[..., K/32]``)."""
    import torch
    emax = {"e2m3": 2, "e3m2": 4}[fmt]
    shp = W.shape
    g = W.float().reshape(*shp[:-1], shp[-1] // block, block)
    amax = g.abs().amax(-1).clamp(min=2.0**-126)
    e = torch.floor(torch.log2(amax)) - emax
    codes = float_to_fp6(g / torch.exp2(e).unsqueeze(-1), fmt).reshape(shp)
    return pack_fp6(codes), (e + 127).clamp(0, 254).to(torch.uint8)


def dequantize_mxfp6(packed, scales_e8m0, fmt: str = "e2m3", block: int = 32):
    import torch
    v = fp6_to_float_torch(unpack_fp6(packed), fmt)
    shp = v.shape
    s = torch.exp2(scales_e8m0.float() - 127.0)
    return (v.reshape(*shp[:-1], shp[-1] // block, block) * s.unsqueeze(-1)).reshape(shp)


__all__ = ["int4_to_float", "uint4_to_float", "e2m1_to_float", "fp4_to_float", "e8m0_to_float", "pack_int4",
           "unpack_int4", "quantize_int4_groupwise", "dequantize_int4_groupwise", "float_to_e2m1",
           "e2m1_to_float_torch", "quantize_mxfp4", "dequantize_mxfp4", "fp6_grid", "float_to_fp6",
           "fp6_to_float_torch", "pack_fp6", "unpack_fp6", "quantize_mxfp6", "dequantize_mxfp6",
           "preshuffle_mx_scales"]


def preshuffle_mx_scales(scales, block_rows: int, block_K: int):
    """e8m0 scales ``[rows, K/32]`` -> the pre-shuffled tile order of
    ``T.gemm_scaled(scale_layout="preshuffled")``: one contiguous
    ``block_rows * block_K / 32``-byte tile per (row tile, K tile), row tiles outer.  Inside a tile,
    row = 64 q + 16 b + r and scale column = 4 kk + g go to byte
    ``(((kk * block_rows/64 + q) * 4 + g) * 16 + r) * 4 + b`` (tl/gemm.h gemm_ss_mx).  A one-time
    transform for weights; activations' quantizers can write this order directly.  Returned as
    ``[rows * K / 32 / 64, 64]`` (2-D, the same bytes) so tiles are 2-D operands."""
    R, C = scales.shape
    ks = block_K // 128
    if block_rows % 64 or block_K % 128 or R % block_rows or C % (block_K // 32):
        raise ValueError(f"preshuffle_mx_scales: shape {tuple(scales.shape)} does not tile by "
                         f"{block_rows} rows x {block_K} K (rows % 64, K % 128)")
    x = scales.reshape(R // block_rows, block_rows // 64, 4, 16, C * 32 // block_K, ks, 4)
    return x.permute(0, 4, 5, 1, 6, 3, 2).reshape(-1, 64).contiguous()
