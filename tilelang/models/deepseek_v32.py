"""DeepSeek-V3.2 (DSA) inference model on tilelang kernels, tensor/expert parallel over RCCL.

Reference: examples/deepseek_v32/inference/{model,generate,kernel}.py (SURVEY §2.4 / §3.6 -- the
reference's only torch.distributed workload).  Same architecture and parallel decomposition:

* ``ParallelEmbedding`` (vocab split + all-reduce), ``ColumnParallelLinear`` (output split),
  ``RowParallelLinear`` (input split + fp32 all-reduce), vocab-parallel head + all-gather;
* MLA attention with the DSA path: the lightning indexer (fp8 q/k, relu-weighted head sum,
  ``tilelang.ops.dsa.mqa_attn_return_logits``) scores every cached key, the top-k selector
  (``dsa.topk_selector``) keeps ``index_topk`` of them, and the sparse MLA kernel
  (``dsa.sparse_mla_fwd``) attends over the selected rows of the compressed latent cache with
  the up-projection absorbed into the query (576-wide q/k, 512-wide latent values);
* MoE with sigmoid, group-limited routing; routed experts sharded over ranks (EP) and run by
  the grouped-GEMM SwiGLU kernels (``tilelang.ops.moe.expert_ffn``), shared experts as a TP MLP,
  one all-reduce per MoE layer (as the reference);
* RMSNorm / GEMM / fp8 activation quantisation are tilelang kernels (``tilelang.ops``).

MI355X-first choices: one process per GPU (torchrun / ``torch.distributed``, backend ``nccl`` =
RCCL over xGMI); every projection is a tilelang MFMA GEMM; fp8 is OCP e4m3 (gfx950), not fnuz.
``ModelArgs.gemm_impl = "fp8"`` (the reference's ``dtype = "fp8"``) stores every projection weight
in the checkpoint's fp8 format -- OCP e4m3 with one fp32 scale per 128x128 block -- and runs it
as ``act_quant`` (per-token, 128-wide groups; ``scale_fmt="ue8m0"`` for power-of-two scales) +
the block-scaled fp8 GEMM (``tilelang.ops.fp8_gemm``, 2xAcc promotion), as the reference's
``linear`` does (model.py:140-168).  The absorbed MLA up-projection dequantises ``wkv_b`` once
(``weight_dequant``, model.py:514, cached as model.py:625 does) and runs as per-head MFMA GEMMs
(``tilelang.ops.gemm.head_bmm``); routed experts stay on the bf16 grouped-GEMM kernels.
Checkpoints: ``tilelang.models.deepseek_v32_ckpt`` converts HF-named safetensors into per-rank
``model{rank}-mp{world}.safetensors`` shards and loads them (reference convert.py /
generate.py:119).

Simplifications (documented; no real checkpoint is available offline, so tests round-trip
synthetic weights through convert -> load): plain RoPE (no YaRN rescaling), no Hadamard rotation
before the indexer's fp8 cast.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist
from torch import nn

from ..ops import dsa
from ..ops.gemm import head_bmm, linear
from ..ops.moe import expert_ffn
from ..ops.norm import rms_norm
from ..ops.quant import act_quant


@dataclass
class ModelArgs:
    max_batch_size: int = 4
    max_seq_len: int = 4096
    dtype: torch.dtype = torch.bfloat16
    vocab_size: int = 129280
    dim: int = 7168
    inter_dim: int = 18432
    moe_inter_dim: int = 2048
    n_layers: int = 61
    n_dense_layers: int = 3
    n_heads: int = 128
    n_routed_experts: int = 256
    n_shared_experts: int = 1
    n_activated_experts: int = 8
    n_expert_groups: int = 8
    n_limited_groups: int = 4
    score_func: str = "sigmoid"
    route_scale: float = 2.5
    q_lora_rank: int = 1536
    kv_lora_rank: int = 512
    qk_nope_head_dim: int = 128
    qk_rope_head_dim: int = 64
    v_head_dim: int = 128
    index_n_heads: int = 64
    index_head_dim: int = 128
    index_topk: int = 2048
    rope_theta: float = 10000.0
    norm_eps: float = 1e-6
    block_M: int = 128  # MoE row tile
    gemm_impl: str = "bf16"  # "fp8": block-scaled fp8 projection weights (the checkpoint format)
    scale_fmt: Optional[str] = None  # "ue8m0": power-of-two activation scales

    @staticmethod
    def from_json(path: str, **over) -> "ModelArgs":
        import json
        with open(path) as f:
            d = json.load(f)
        known = {k: v for k, v in d.items() if k in ModelArgs.__dataclass_fields__ and k != "dtype"}
        known.update(over)
        return ModelArgs(**known)

    @staticmethod
    def tiny(**over) -> "ModelArgs":
        """A small configuration with the same structure (tests / smoke)."""
        a = ModelArgs(max_batch_size=2, max_seq_len=256, vocab_size=512, dim=256, inter_dim=512, moe_inter_dim=128,
                      n_layers=2, n_dense_layers=1, n_heads=16, n_routed_experts=8, n_shared_experts=1,
                      n_activated_experts=2, n_expert_groups=2, n_limited_groups=1, q_lora_rank=128,
                      kv_lora_rank=128, qk_nope_head_dim=32, qk_rope_head_dim=32, v_head_dim=32, index_n_heads=16,
                      index_head_dim=128, index_topk=64, block_M=64)
        for k, v in over.items():
            setattr(a, k, v)
        return a


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def _all_reduce(t: torch.Tensor) -> torch.Tensor:
    ws, _ = _world()
    if ws > 1:
        dist.all_reduce(t)
    return t


class _Init:
    """Deterministic weights: every full tensor is drawn from a per-parameter seed on the CPU
    and sliced for this rank, so any TP/EP degree sees the same global model."""

    def __init__(self, seed: int):
        self.seed = seed
        self.count = 0

    def full(self, *shape, scale: float, dtype) -> torch.Tensor:
        self.count += 1
        g = torch.Generator(device="cpu").manual_seed(self.seed * 100003 + self.count)
        return (torch.randn(*shape, generator=g) * scale).to(dtype)


class Linear(nn.Module):
    # set by Transformer from ModelArgs.gemm_impl / scale_fmt (the reference's Linear.dtype)
    fp8 = False
    scale_fmt: Optional[str] = None

    def __init__(self, init: _Init, in_features: int, out_features: int, dtype, part_out=1, part_in=1, rank=0):
        super().__init__()
        w = init.full(out_features, in_features, scale=in_features**-0.5, dtype=dtype)
        if part_out > 1:
            n = out_features // part_out
            w = w[rank * n:(rank + 1) * n]
        if part_in > 1:
            n = in_features // part_in
            w = w[:, rank * n:(rank + 1) * n]
        self.scale = None
        if Linear.fp8 and dtype != torch.float32 and w.shape[1] % 128 == 0:
            # the checkpoint format: fp8 e4m3 + one fp32 scale per 128x128 block of this rank's slice
            from ..ops.fp8_gemm import weight_quant
            wq, ws = weight_quant(w.contiguous())
            self.weight = nn.Parameter(wq, requires_grad=False)
            self.scale = nn.Parameter(ws, requires_grad=False)
            self.out_dtype = dtype
        else:
            self.weight = nn.Parameter(w.contiguous(), requires_grad=False)

    def _mm(self, x):
        if self.scale is None:
            return linear(x, self.weight)
        from ..ops.fp8_gemm import fp8_linear
        return fp8_linear(x.to(self.out_dtype), self.weight, self.scale, Linear.scale_fmt == "ue8m0")

    def dequant_weight(self) -> torch.Tensor:
        """The weight in its compute dtype (fp8 blocks rescaled: reference ``weight_dequant``)."""
        if self.scale is None:
            return self.weight
        from ..ops.fp8_gemm import weight_dequant
        return weight_dequant(self.weight, self.scale).to(self.out_dtype)

    def forward(self, x):
        return self._mm(x)


def ColumnParallelLinear(init, in_features, out_features, dtype):
    ws, r = _world()
    assert out_features % ws == 0, f"output features {out_features} must be divisible by world size {ws}"
    return Linear(init, in_features, out_features, dtype, part_out=ws, rank=r)


class RowParallelLinear(Linear):

    def __init__(self, init, in_features, out_features, dtype, reduce_output=True):
        ws, r = _world()
        assert in_features % ws == 0, f"input features {in_features} must be divisible by world size {ws}"
        super().__init__(init, in_features, out_features, dtype, part_in=ws, rank=r)
        self.reduce_output = reduce_output

    def forward(self, x):
        y = self._mm(x)
        if self.reduce_output and _world()[0] > 1:
            y = _all_reduce(y.float()).to(x.dtype)
        return y


class ParallelEmbedding(nn.Module):

    def __init__(self, init, vocab_size, dim, dtype):
        super().__init__()
        ws, r = _world()
        assert vocab_size % ws == 0
        self.part = vocab_size // ws
        self.start = r * self.part
        w = init.full(vocab_size, dim, scale=1.0, dtype=dtype)[self.start:self.start + self.part]
        self.weight = nn.Parameter(w.contiguous(), requires_grad=False)

    def forward(self, tokens):
        ws, _ = _world()
        if ws == 1:
            return self.weight[tokens]
        local = tokens - self.start
        mask = (local < 0) | (local >= self.part)
        y = self.weight[local.clamp(0, self.part - 1)]
        y = y.masked_fill(mask.unsqueeze(-1), 0)
        return _all_reduce(y.float()).to(self.weight.dtype)


class RMSNorm(nn.Module):

    def __init__(self, dim, eps=1e-6, dtype=torch.bfloat16):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, dtype=dtype), requires_grad=False)

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)


def precompute_freqs_cis(rope_dim: int, max_seq_len: int, theta: float) -> torch.Tensor:
    inv = 1.0 / (theta**(torch.arange(0, rope_dim, 2, dtype=torch.float32) / rope_dim))
    t = torch.arange(max_seq_len, dtype=torch.float32)
    return torch.polar(torch.ones(max_seq_len, rope_dim // 2), torch.outer(t, inv))


def apply_rotary_emb(x: torch.Tensor, freqs: torch.Tensor) -> torch.Tensor:
    """x [b, s, ..., rope_dim] (interleaved pairs), freqs [s, rope_dim/2] complex."""
    dt = x.dtype
    xc = torch.view_as_complex(x.float().reshape(*x.shape[:-1], -1, 2))
    f = freqs.view(1, freqs.shape[0], *([1] * (xc.dim() - 3)), freqs.shape[-1])
    return torch.view_as_real(xc * f).flatten(-2).to(dt)


class Indexer(nn.Module):
    """DSA lightning indexer: picks ``index_topk`` cached keys per query token."""

    def __init__(self, init: _Init, args: ModelArgs):
        super().__init__()
        self.args = args
        self.h, self.d = args.index_n_heads, args.index_head_dim
        self.rope = args.qk_rope_head_dim
        self.wq_b = Linear(init, args.q_lora_rank, self.h * self.d, args.dtype)
        self.wk = Linear(init, args.dim, self.d, args.dtype)
        self.k_norm = nn.LayerNorm(self.d)
        self.weights_proj = Linear(init, args.dim, self.h, torch.float32)
        B, S = args.max_batch_size, args.max_seq_len
        self.register_buffer("k_cache", torch.zeros(B, S, self.d, dtype=torch.float8_e4m3fn), persistent=False)
        self.register_buffer("k_scale", torch.zeros(B, S, dtype=torch.float32), persistent=False)

    def forward(self, x, qr, start_pos, freqs):
        b, s, _ = x.shape
        end = start_pos + s
        q = self.wq_b(qr).view(b, s, self.h, self.d)
        q = torch.cat([apply_rotary_emb(q[..., :self.rope], freqs), q[..., self.rope:]], -1)
        k = self.k_norm(self.wk(x).float()).to(x.dtype)
        k = torch.cat([apply_rotary_emb(k[..., :self.rope], freqs), k[..., self.rope:]], -1)
        q8, qs = act_quant(q.contiguous(), group=self.d)              # [b, s, h, d], [b, s, h, 1]
        k8, ks = act_quant(k.contiguous(), group=self.d)
        self.k_cache[:b, start_pos:end] = k8
        self.k_scale[:b, start_pos:end] = ks.squeeze(-1)
        w = self.weights_proj(x.float()) * (self.h**-0.5) * qs.squeeze(-1)
        topk = min(self.args.index_topk, end)
        topk_pad = max(64, (topk + 63) // 64 * 64)
        n_pad = max(256, (end + 255) // 256 * 256)
        idx_all = []
        for bi in range(b):
            ks_ = torch.zeros(s, dtype=torch.int32, device=x.device)
            ke_ = torch.arange(start_pos + 1, end + 1, dtype=torch.int32, device=x.device)
            logits = dsa.for_target("mqa_attn_return_logits", _target(x), s, None, self.h, self.d)(
                q8[bi].reshape(s * self.h, self.d).contiguous(), self.k_cache[bi, :end].contiguous(),
                self.k_scale[bi, :end].contiguous(), w[bi].contiguous().float(), ks_, ke_)
            padded = torch.full((s, n_pad), float("-inf"), device=x.device)
            padded[:, :end] = logits
            # rows with fewer than topk_pad visible keys pick -inf slots: mark them invalid
            idx = dsa.for_target("topk_selector", _target(x), s, n_pad, topk_pad)(padded)
            val = torch.gather(padded, 1, idx.long())
            idx = torch.where(torch.isfinite(val), idx, torch.full_like(idx, end))
            idx_all.append(idx)
        idx = torch.stack(idx_all)
        if _world()[0] > 1:
            dist.broadcast(idx, src=0)  # every rank must attend to the same keys
        return idx


class MLA(nn.Module):

    def __init__(self, init: _Init, args: ModelArgs):
        super().__init__()
        ws, _ = _world()
        self.args = args
        self.n_local_heads = args.n_heads // ws
        self.nope, self.rope, self.vdim = args.qk_nope_head_dim, args.qk_rope_head_dim, args.v_head_dim
        self.qk_dim = self.nope + self.rope
        self.kv_lora = args.kv_lora_rank
        dt = args.dtype
        self.wq_a = Linear(init, args.dim, args.q_lora_rank, dt)
        self.q_norm = RMSNorm(args.q_lora_rank, args.norm_eps, dt)
        self.wq_b = ColumnParallelLinear(init, args.q_lora_rank, args.n_heads * self.qk_dim, dt)
        self.wkv_a = Linear(init, args.dim, self.kv_lora + self.rope, dt)
        self.kv_norm = RMSNorm(self.kv_lora, args.norm_eps, dt)
        self.wkv_b = ColumnParallelLinear(init, self.kv_lora, args.n_heads * (self.nope + self.vdim), dt)
        self.wo = RowParallelLinear(init, args.n_heads * self.vdim, args.dim, dt)
        self.softmax_scale = self.qk_dim**-0.5
        self.indexer = Indexer(init, args)
        B, S = args.max_batch_size, args.max_seq_len
        self.register_buffer("kv_cache", torch.zeros(B, S, self.kv_lora, dtype=dt), persistent=False)
        self.register_buffer("pe_cache", torch.zeros(B, S, self.rope, dtype=dt), persistent=False)
        self._absorb = None

    def absorbed(self):
        """(W_uk^T [h, kv_lora, nope], W_uv [h, v, kv_lora]) in the compute dtype, dequantised from
        the fp8 ``wkv_b`` ONCE and cached (reference model.py:625 keeps the dequantised weight);
        ``load_model`` drops the cache when it replaces ``wkv_b``."""
        if self._absorb is None:
            w = self.wkv_b.dequant_weight().view(self.n_local_heads, self.nope + self.vdim, self.kv_lora)
            self._absorb = (w[:, :self.nope].transpose(1, 2).contiguous(), w[:, self.nope:].contiguous())
        return self._absorb

    def forward(self, x, start_pos, freqs):
        b, s, _ = x.shape
        end = start_pos + s
        qr = self.q_norm(self.wq_a(x))
        q = self.wq_b(qr).view(b, s, self.n_local_heads, self.qk_dim)
        q_nope, q_pe = q[..., :self.nope], apply_rotary_emb(q[..., self.nope:].contiguous(), freqs)
        kv = self.wkv_a(x)
        latent, k_pe = kv[..., :self.kv_lora], kv[..., self.kv_lora:]
        self.kv_cache[:b, start_pos:end] = self.kv_norm(latent.contiguous())
        self.pe_cache[:b, start_pos:end] = apply_rotary_emb(k_pe.contiguous().unsqueeze(2), freqs).squeeze(2)
        # absorb W_uk into the query: q_lat[h] = q_nope[h] @ W_uk[h]  (one per-head MFMA GEMM)
        w_uk_t, w_uv = self.absorbed()
        q_lat = head_bmm(q_nope.contiguous(), w_uk_t)                           # [b, s, h, 512]
        qf = torch.cat([q_lat, q_pe], -1).contiguous()                          # [b, s, h, 576]
        kvf = torch.cat([self.kv_cache[:b, :end], self.pe_cache[:b, :end]], -1).unsqueeze(2).contiguous()
        idx = self.indexer(x, qr, start_pos, freqs).unsqueeze(2).contiguous()    # [b, s, 1, topk]
        kern = dsa.for_target("sparse_mla_fwd", _target(x), b, s, None, self.n_local_heads, self.kv_lora, self.rope,
                              idx.shape[-1], 1, self.softmax_scale, 64, None, _tdt(x.dtype))
        o_lat, _ = kern(qf, kvf, idx)                                             # [b, s, h, 512]
        o = head_bmm(o_lat.contiguous(), w_uv)                                  # [b, s, h, 128]
        return self.wo(o.reshape(b, s, -1))


def _target(x: torch.Tensor) -> str:
    return "cpu" if x.device.type == "cpu" else "hip"


def _tdt(dt):
    return {torch.float16: "float16", torch.bfloat16: "bfloat16"}[dt]


class MLP(nn.Module):

    def __init__(self, init, dim, inter_dim, dtype, reduce_output=True):
        super().__init__()
        self.w1 = ColumnParallelLinear(init, dim, inter_dim, dtype)
        self.w3 = ColumnParallelLinear(init, dim, inter_dim, dtype)
        self.w2 = RowParallelLinear(init, inter_dim, dim, dtype, reduce_output=reduce_output)

    def forward(self, x):
        return self.w2((torch.nn.functional.silu(self.w1(x).float()) * self.w3(x).float()).to(x.dtype))


class Gate(nn.Module):
    """Sigmoid scores with group-limited top-k (DeepSeek-V3 routing)."""

    def __init__(self, init, args: ModelArgs):
        super().__init__()
        self.args = args
        self.weight = nn.Parameter(init.full(args.n_routed_experts, args.dim, scale=args.dim**-0.5,
                                             dtype=torch.float32), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(args.n_routed_experts), requires_grad=False)

    def forward(self, x):
        a = self.args
        scores = x.float() @ self.weight.t()
        scores = scores.sigmoid() if a.score_func == "sigmoid" else scores.softmax(-1)
        orig = scores
        scores = scores + self.bias
        if a.n_expert_groups > 1:
            g = scores.view(x.shape[0], a.n_expert_groups, -1)
            gs = g.topk(2, -1).values.sum(-1) if a.score_func == "sigmoid" else g.amax(-1)
            keep = gs.topk(a.n_limited_groups, -1).indices
            mask = torch.ones_like(gs, dtype=torch.bool).scatter_(1, keep, False)
            scores = g.masked_fill(mask.unsqueeze(-1), float("-inf")).flatten(1)
        ids = scores.topk(a.n_activated_experts, -1).indices
        w = orig.gather(1, ids)
        if a.score_func == "sigmoid":
            w = w / w.sum(-1, keepdim=True)
        return ids, w * a.route_scale


class MoE(nn.Module):

    def __init__(self, init, args: ModelArgs):
        super().__init__()
        ws, r = _world()
        self.args = args
        assert args.n_routed_experts % ws == 0
        self.n_local = args.n_routed_experts // ws
        self.first = r * self.n_local
        self.gate = Gate(init, args)
        E, H, F = args.n_routed_experts, args.dim, args.moe_inter_dim
        w1 = init.full(E, 2 * F, H, scale=H**-0.5, dtype=args.dtype)  # [gate | up]
        w2 = init.full(E, H, F, scale=F**-0.5, dtype=args.dtype)
        self.w1 = nn.Parameter(w1[self.first:self.first + self.n_local].contiguous(), requires_grad=False)
        self.w2 = nn.Parameter(w2[self.first:self.first + self.n_local].contiguous(), requires_grad=False)
        self.shared = MLP(init, H, args.n_shared_experts * F, args.dtype, reduce_output=False)

    def forward(self, x):
        shp = x.shape
        x = x.reshape(-1, shp[-1])
        ids, w = self.gate(x)
        k = ids.shape[1]
        tok = torch.arange(x.shape[0], device=x.device).repeat_interleave(k)
        flat = ids.reshape(-1)
        local = (flat >= self.first) & (flat < self.first + self.n_local)
        y = torch.zeros(x.shape[0], shp[-1], dtype=torch.float32, device=x.device)
        if bool(local.any()):
            sel = torch.nonzero(local).squeeze(1)
            out = expert_ffn(x[tok[sel]], flat[sel] - self.first, self.w1, self.w2, self.args.block_M)
            y.index_add_(0, tok[sel], out.float() * w.reshape(-1)[sel, None])
        y = y + self.shared(x).float()
        return _all_reduce(y).to(x.dtype).reshape(shp)


class Block(nn.Module):

    def __init__(self, init, layer_id: int, args: ModelArgs):
        super().__init__()
        self.attn_norm = RMSNorm(args.dim, args.norm_eps, args.dtype)
        self.attn = MLA(init, args)
        self.ffn_norm = RMSNorm(args.dim, args.norm_eps, args.dtype)
        self.ffn = MLP(init, args.dim, args.inter_dim, args.dtype) if layer_id < args.n_dense_layers else \
            MoE(init, args)

    def forward(self, x, start_pos, freqs):
        x = x + self.attn(self.attn_norm(x), start_pos, freqs)
        return x + self.ffn(self.ffn_norm(x))


class Transformer(nn.Module):

    def __init__(self, args: ModelArgs, seed: int = 0, device="cuda"):
        super().__init__()
        init = _Init(seed)
        self.args = args
        if args.gemm_impl not in ("bf16", "fp8"):
            raise ValueError(f"gemm_impl must be 'bf16' or 'fp8', got {args.gemm_impl!r}")
        Linear.fp8 = args.gemm_impl == "fp8"
        Linear.scale_fmt = args.scale_fmt
        self.embed = ParallelEmbedding(init, args.vocab_size, args.dim, args.dtype)
        self.layers = nn.ModuleList([Block(init, i, args) for i in range(args.n_layers)])
        self.norm = RMSNorm(args.dim, args.norm_eps, args.dtype)
        Linear.fp8 = False  # the output head stays in the compute dtype (as the reference)
        self.head = ColumnParallelLinear(init, args.dim, args.vocab_size, args.dtype)
        self.register_buffer("freqs_cis", precompute_freqs_cis(args.qk_rope_head_dim, args.max_seq_len,
                                                                args.rope_theta), persistent=False)
        self.to(device)

    @torch.inference_mode()
    def forward(self, tokens: torch.Tensor, start_pos: int = 0) -> torch.Tensor:
        s = tokens.shape[1]
        freqs = self.freqs_cis[start_pos:start_pos + s]
        h = self.embed(tokens)
        for layer in self.layers:
            h = layer(h, start_pos, freqs)
        h = self.norm(h)[:, -1]
        logits = self.head(h).float()
        ws, _ = _world()
        if ws > 1:
            parts = [torch.empty_like(logits) for _ in range(ws)]
            dist.all_gather(parts, logits)
            logits = torch.cat(parts, -1)
        return logits


@torch.inference_mode()
def generate(model: Transformer, prompt_tokens, max_new_tokens: int, temperature: float = 0.0, eos_id: int = -1):
    """Greedy / temperature sampling with the latent + indexer KV caches (reference generate.py)."""
    dev = model.freqs_cis.device
    prompt_lens = [len(t) for t in prompt_tokens]
    assert max(prompt_lens) + max_new_tokens <= model.args.max_seq_len
    assert len(prompt_tokens) <= model.args.max_batch_size
    total = max(prompt_lens) + max_new_tokens
    tokens = torch.full((len(prompt_tokens), total), -1, dtype=torch.long, device=dev)
    for i, t in enumerate(prompt_tokens):
        tokens[i, :len(t)] = torch.tensor(t, dtype=torch.long, device=dev)
    prev = 0
    finished = torch.zeros(len(prompt_tokens), dtype=torch.bool, device=dev)
    prompt_mask = tokens != -1
    for cur in range(min(prompt_lens), total):
        logits = model.forward(tokens[:, prev:cur].clamp(min=0), prev)
        if temperature > 0:
            probs = torch.softmax(logits / temperature, -1)
            nxt = torch.multinomial(probs, 1).squeeze(1)
        else:
            nxt = logits.argmax(-1)
        if _world()[0] > 1:
            dist.broadcast(nxt, src=0)
        nxt = torch.where(prompt_mask[:, cur], tokens[:, cur], nxt)
        tokens[:, cur] = nxt
        finished |= (~prompt_mask[:, cur]) & (nxt == eos_id)
        prev = cur
        if bool(finished.all()):
            break
    return [tokens[i, prompt_lens[i]:prompt_lens[i] + max_new_tokens].tolist() for i in range(len(prompt_tokens))]
