"""BitNet b1.58 (LLaMA architecture with ternary BitLinear projections) on tilelang kernels
(reference: examples/bitnet-1.58b/modeling_bitnet.py:89-420, utils_quant.py:16-31,216-236,
configuration_bitnet.py).

Architecture as the reference: RMSNorm -> q/k/v BitLinear -> RoPE -> causal attention ->
``inner_attn_ln`` RMSNorm -> o_proj BitLinear; RMSNorm -> gate/up BitLinear -> SiLU(gate) * up ->
``ffn_layernorm`` RMSNorm -> down BitLinear.  A BitLinear quantises its input per token to int8
(absmax, 127 levels) and its weight to {-1, 0, 1} with one scale 1/mean|W|.

MI355X execution (``tilelang.ops.bitnet``):

* every BitLinear input is produced by an RMSNorm, so norm + int8 quantisation are ONE kernel
  (``rms_norm_quant``) that writes the int8 row and its scale;
* q|k|v and gate|up are each one fused int8 x int2 GEMM on ``v_mfma_i32_16x16x64_i8`` (weights
  2 bits each in HBM, per-column weight scales in the dequantising epilogue); decode-sized inputs
  (<= 8 rows) take the weight-streaming GEMV kernel instead (no matrix cores, K padded to 256);
* attention uses PyTorch SDPA (the BitNet-specific work is the ternary projections; the flash
  kernels live in examples/flash_attention).

Weights are random (no checkpoint is available offline); ``BitnetConfig.bitnet_3b()`` is the
reference's 3B shape.  ``reference_forward`` is the reference's fp32-simulated BitLinear math,
used by the tests as the numerics oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
from torch import nn

from ..ops import bitnet as K


@dataclass
class BitnetConfig:
    vocab_size: int = 32002
    hidden_size: int = 3200
    intermediate_size: int = 8640
    num_hidden_layers: int = 26
    num_attention_heads: int = 32
    max_position_embeddings: int = 2048
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    dtype: torch.dtype = torch.float16

    @classmethod
    def bitnet_3b(cls):
        return cls()

    @classmethod
    def tiny(cls):
        return cls(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                   max_position_embeddings=256)


class BitLinearGroup(nn.Module):
    """One or more BitLinear projections sharing an input (fused along N)."""

    def __init__(self, in_features, out_features_list, dtype):
        super().__init__()
        self.splits = list(out_features_list)
        self.weights = nn.ParameterList(
            [nn.Parameter(torch.randn(n, in_features, dtype=dtype) * in_features**-0.5) for n in self.splits])
        self.packed: Optional[torch.Tensor] = None
        self.packed_dec: Optional[torch.Tensor] = None
        self.col_scale: Optional[torch.Tensor] = None

    @torch.no_grad()
    def freeze(self):
        """Ternarise + pack the weights (per projection scale, expanded per output column).  Two
        packings: exact K for the prefill MFMA GEMM, K padded to 256 codes (padding = code 1 =
        weight 0) for the decode GEMV."""
        packs, scales = [], []
        for w in self.weights:
            p, s = K.weight_quant_ternary(w)
            packs.append(p)
            scales.append(s.expand(w.shape[0]))
        self.packed = torch.cat(packs, 0).contiguous()
        kp = -(-self.packed.shape[1] // 64) * 64
        self.packed_dec = torch.nn.functional.pad(self.packed, (0, kp - self.packed.shape[1]),
                                                  value=0b01010101).contiguous()
        self.col_scale = torch.cat(scales).float().contiguous()

    def forward(self, xq, sx, dtype):
        if self.packed is None or self.packed.device != xq.device:
            self.freeze()
        rows = xq.numel() // xq.shape[-1]
        wq = self.packed_dec if rows <= 8 else self.packed
        y = K.int2_gemm(xq, wq, sx, self.col_scale, out_dtype=dtype, zero=1)
        return torch.split(y, self.splits, -1) if len(self.splits) > 1 else y


def _rope(x, cos, sin):
    x1, x2 = x[..., :x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return x * cos + torch.cat((-x2, x1), -1) * sin


def rope_tables(head_dim, seq_len, theta, device, dtype):
    inv = 1.0 / (theta**(torch.arange(0, head_dim, 2, dtype=torch.float32, device=device) / head_dim))
    f = torch.outer(torch.arange(seq_len, dtype=torch.float32, device=device), inv)
    emb = torch.cat((f, f), -1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


class BitnetDecoderLayer(nn.Module):

    def __init__(self, cfg: BitnetConfig):
        super().__init__()
        h, i, dt = cfg.hidden_size, cfg.intermediate_size, cfg.dtype
        self.cfg = cfg
        self.input_layernorm = nn.Parameter(torch.ones(h, dtype=dt))
        self.inner_attn_ln = nn.Parameter(torch.ones(h, dtype=dt))
        self.post_attention_layernorm = nn.Parameter(torch.ones(h, dtype=dt))
        self.ffn_layernorm = nn.Parameter(torch.ones(i, dtype=dt))
        self.qkv = BitLinearGroup(h, [h, h, h], dt)
        self.o_proj = BitLinearGroup(h, [h], dt)
        self.gate_up = BitLinearGroup(h, [i, i], dt)
        self.down = BitLinearGroup(i, [h], dt)

    def forward(self, x, cos, sin):
        cfg = self.cfg
        b, s, h = x.shape
        nh = cfg.num_attention_heads
        hd = h // nh
        eps = cfg.rms_norm_eps
        xq, sx = K.rms_norm_quant(x, self.input_layernorm, eps)
        q, k, v = self.qkv(xq, sx, x.dtype)
        q, k, v = (t.view(b, s, nh, hd).transpose(1, 2) for t in (q, k, v))
        q, k = _rope(q, cos, sin), _rope(k, cos, sin)
        a = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
        a = a.transpose(1, 2).reshape(b, s, h)
        aq, sa = K.rms_norm_quant(a, self.inner_attn_ln, eps)
        x = x + self.o_proj(aq, sa, x.dtype)
        xq, sx = K.rms_norm_quant(x, self.post_attention_layernorm, eps)
        g, u = self.gate_up(xq, sx, x.dtype)
        m = torch.nn.functional.silu(g) * u
        mq, sm = K.rms_norm_quant(m, self.ffn_layernorm, eps)
        return x + self.down(mq, sm, x.dtype)


class BitnetForCausalLM(nn.Module):

    def __init__(self, cfg: BitnetConfig):
        super().__init__()
        self.cfg = cfg
        self.embed_tokens = nn.Parameter(torch.randn(cfg.vocab_size, cfg.hidden_size, dtype=cfg.dtype) * 0.02)
        self.layers = nn.ModuleList([BitnetDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = nn.Parameter(torch.ones(cfg.hidden_size, dtype=cfg.dtype))
        self.lm_head = nn.Parameter(torch.randn(cfg.vocab_size, cfg.hidden_size, dtype=cfg.dtype) * 0.02)

    @torch.no_grad()
    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        from ..ops.norm import rms_norm
        cfg = self.cfg
        x = self.embed_tokens[input_ids]
        s = input_ids.shape[1]
        cos, sin = rope_tables(cfg.hidden_size // cfg.num_attention_heads, s, cfg.rope_theta, x.device, x.dtype)
        for layer in self.layers:
            x = layer(x, cos, sin)
        x = rms_norm(x, self.norm, cfg.rms_norm_eps)
        return x @ self.lm_head.t()  # the lm_head is not a BitLinear in the reference

    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, max_new_tokens: int = 8) -> torch.Tensor:
        """Greedy decoding (full recompute per step: a demo of the decode-sized GEMM path)."""
        ids = input_ids
        for _ in range(max_new_tokens):
            nxt = self.forward(ids)[:, -1].argmax(-1, keepdim=True)
            ids = torch.cat([ids, nxt], 1)
        return ids


# ---------------------------------------------------------------------------------------- fp32 oracle


def _ref_rms(x, w, eps):
    xf = x.float()
    y = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype)
    return w * y


def _ref_bitlinear(x, w):
    """utils_quant.BitLinear forward (fp32 simulated): activation_quant(x) @ weight_quant(w)^T."""
    xf = x.float()
    s = 127.0 / xf.abs().amax(-1, keepdim=True).clamp(min=1e-5)
    xq = (xf * s).round().clamp(-128, 127) / s
    wf = w.float()
    sw = 1.0 / wf.abs().mean().clamp(min=1e-5)
    wq = (wf * sw).round().clamp(-1, 1) / sw
    return (xq @ wq.t()).to(x.dtype)


@torch.no_grad()
def reference_layer(layer: BitnetDecoderLayer, x, cos, sin):
    cfg = layer.cfg
    b, s, h = x.shape
    nh, eps = cfg.num_attention_heads, cfg.rms_norm_eps
    hd = h // nh
    n = _ref_rms(x, layer.input_layernorm, eps)
    q, k, v = (_ref_bitlinear(n, w) for w in layer.qkv.weights)
    q, k, v = (t.view(b, s, nh, hd).transpose(1, 2).float() for t in (q, k, v))
    q, k = _rope(q, cos.float(), sin.float()), _rope(k, cos.float(), sin.float())
    sc = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    sc = sc.masked_fill(torch.triu(torch.ones(s, s, dtype=torch.bool, device=x.device), 1), float("-inf"))
    a = (torch.softmax(sc, -1) @ v).transpose(1, 2).reshape(b, s, h).to(x.dtype)
    x = x + _ref_bitlinear(_ref_rms(a, layer.inner_attn_ln, eps), layer.o_proj.weights[0])
    n = _ref_rms(x, layer.post_attention_layernorm, eps)
    g, u = (_ref_bitlinear(n, w) for w in layer.gate_up.weights)
    m = (torch.nn.functional.silu(g.float()) * u.float()).to(x.dtype)
    return x + _ref_bitlinear(_ref_rms(m, layer.ffn_layernorm, eps), layer.down.weights[0])
