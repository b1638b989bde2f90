"""Mixture-of-Experts FFN layer on the mesh (BASELINE config 5: grouped-GEMM MoE, 8 experts,
1/2/4/8 MI355X over xGMI).

Per layer: router (softmax top-k) -> dispatch -> SwiGLU experts (tilelang grouped GEMMs,
``tilelang.ops.moe``) -> weighted combine.  Parallel modes over the active mesh:

* ``"local"`` — all experts on this rank (single GPU, or plain data parallel);
* ``"ep"``    — expert parallel: rank r owns experts ``[r*E/W, (r+1)*E/W)``; tokens travel to
                their experts and back with two variable-size all-to-alls (RCCL over xGMI,
                ``parallel.collectives.all_to_all_v``) — the reference DeepSeek-V3.2
                example's EP (``examples/deepseek_v32/inference/model.py:787-850``) uses an
                all-reduce of the full output instead, moving W x more bytes;
* ``"tp"``    — tensor parallel ("mesh cross-GPU tiles"): every rank holds 1/W of every
                expert's FFN width, the down-projection's fp32 output tiles are summed across
                the mesh INSIDE the GEMM kernel (``T.comm.all_reduce_tile``), so the reduction
                of one tile overlaps the MMA of the next on the same GPU.

Weights are random-initialised (no checkpoints are available); ``moe_reference`` is the
plain PyTorch fp32 definition the kernels are tested against.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import os

import torch



@dataclass
class MoEConfig:
    hidden: int = 4096
    ffn: int = 14336
    n_experts: int = 8
    topk: int = 2
    dtype: torch.dtype = torch.bfloat16
    block_M: int = 128
    gemm_cfg: Optional[dict] = None  # expert GEMM tile: block_N, block_K, num_stages, threads


def route(x: torch.Tensor, gate_w: torch.Tensor, topk: int):
    """softmax(x Wg^T) top-k with renormalised weights -> (expert ids [T, k], weights [T, k]).

    On the GPU / CPU target this is the tilelang router kernel (``ops.moe.route``); this
    PyTorch definition is the reference it is tested against."""
    logits = torch.nn.functional.linear(x, gate_w).float()
    probs = torch.softmax(logits, -1)
    w, ids = torch.topk(probs, topk, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return ids, w


def moe_reference(x, gate_w, w1, w2, topk, routing=None):
    """fp32 PyTorch definition (w1: [E, 2F, H] = [gate | up], w2: [E, H, F]).  ``routing``:
    (ids, weights) to use instead of ``route`` -- a kernel's own choice between experts whose
    16-bit logits tie exactly (see ``routing_equivalent``)."""
    ids, wts = route(x, gate_w, topk) if routing is None else (routing[0].long(), routing[1].float())
    xf = x.float()
    out = torch.zeros_like(xf)
    F = w1.shape[1] // 2
    for e in range(w1.shape[0]):
        tok, slot = torch.nonzero(ids == e, as_tuple=True)
        if tok.numel() == 0:
            continue
        h = xf[tok] @ w1[e].float().t()
        a = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
        out.index_add_(0, tok, (a @ w2[e].float().t()) * wts[tok, slot, None])
    return out


def routing_equivalent(x, gate_w, topk, ids, w, atol=1e-6) -> bool:
    """True when (ids, w) is a valid top-k of ``route``'s probabilities: same weights, and every
    expert that differs from the reference choice has exactly the probability of the expert it
    replaces (an exact tie of the 16-bit logits, broken the other way)."""
    rid, rw = route(x, gate_w, topk)
    if not torch.allclose(w.float(), rw.float(), atol=atol, rtol=1e-5):
        return False
    probs = torch.softmax(torch.nn.functional.linear(x, gate_w).float(), -1)
    diff = ids.long() != rid
    if not diff.any():
        return True
    got = probs.gather(1, ids.long())
    want = probs.gather(1, rid)
    return bool(torch.allclose(got[diff], want[diff], atol=atol, rtol=1e-5))


def init_moe_weights(cfg: MoEConfig, seed: int = 0):
    """Full (gate [E, H], w1 [E, 2F, H], w2 [E, H, F]) on the CPU, deterministic in ``seed``."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    E, H, F = cfg.n_experts, cfg.hidden, cfg.ffn

    def rnd(*shape, scale):
        return (torch.randn(*shape, generator=g) * scale).to(cfg.dtype)

    return rnd(E, H, scale=H ** -0.5), rnd(E, 2 * F, H, scale=H ** -0.5), rnd(E, H, F, scale=F ** -0.5)


class MoELayer(torch.nn.Module):

    def __init__(self, cfg: MoEConfig, parallel: str = "local", mesh=None, device="cuda", seed: int = 0):
        super().__init__()
        from ..parallel.mesh import current_mesh
        self.cfg = cfg
        self.parallel = parallel
        self.mesh = mesh or (current_mesh() if parallel != "local" else None)
        W = self.mesh.world if self.mesh is not None else 1
        E, H, F = cfg.n_experts, cfg.hidden, cfg.ffn
        if parallel == "ep" and E % W:
            raise ValueError(f"{E} experts do not split over {W} ranks")
        if parallel == "tp" and F % W:
            raise ValueError(f"ffn {F} does not split over {W} ranks")
        # full weights are generated identically on every rank, then sliced
        gate_w, w1, w2 = init_moe_weights(cfg, seed)
        self.gate_w = gate_w.to(device)
        if parallel == "ep":
            r = self.mesh.rank
            n = E // W
            self.local_experts = range(r * n, (r + 1) * n)
            w1, w2 = w1[r * n:(r + 1) * n], w2[r * n:(r + 1) * n]
        elif parallel == "tp":
            r = self.mesh.rank
            f = F // W
            w1 = torch.cat([w1[:, r * f:(r + 1) * f], w1[:, F + r * f:F + (r + 1) * f]], 1)
            w2 = w2[:, :, r * f:(r + 1) * f]
        # kernel layout: gate/up rows interleaved so the SwiGLU activation fuses into GEMM-1
        from ..ops.moe import swiglu_interleave
        self.w1 = swiglu_interleave(w1.contiguous()).to(device)
        self.w2 = w2.contiguous().to(device)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops import moe as K
        cfg = self.cfg
        ids, wts = K.route(x, self.gate_w, cfg.topk)
        if self.parallel in ("local", "tp"):
            y, dest = K.expert_ffn_padded(x, ids, cfg.topk, self.w1, self.w2, cfg.block_M,
                                          reduce_mesh="all" if self.parallel == "tp" else None, cfg=cfg.gemm_cfg,
                                          w1_interleaved=True)
            return K.combine(y, dest, wts)
        if self._device_ep():
            return self._ep_device(x, ids, wts)
        y = self._ep(x, ids)
        return K.combine(y, torch.arange(y.shape[0], device=x.device, dtype=torch.int32), wts)

    def _device_ep(self) -> bool:
        """Process meshes exchange tokens with the device protocol (ops/ep.py: tl/ep.h over IPC on
        GPUs, tl/ep_cpu.h over /dev/shm on CPU gloo meshes); virtual meshes use the host collectives."""
        from ..parallel.mesh import ProcessMesh
        return isinstance(self.mesh, ProcessMesh) and self.ep_mode == "device"

    # "device" (ops/ep.py, no host sync) or "host" (RCCL all_to_all_v); TL_EP_MODE overrides
    ep_mode = os.environ.get("TL_EP_MODE", "device")

    def _ep_device(self, x, ids, wts):
        """Expert parallel without host synchronisation: rows go straight into the owners'
        symmetric buffers (tl/ep.h), the local experts run on the received row table (empty
        slots carry expert id -1), and results come back the same way."""
        from ..ops import moe as K
        from ..ops.ep import EPExchange
        key = (x.shape[0], x.shape[1], x.dtype)
        ex = self.__dict__.get("_exchange")
        if ex is None or ex[0] != key:
            ex = (key, EPExchange(self.mesh, x.shape[0], x.shape[1], self.cfg.topk, self.cfg.n_experts, x.dtype))
            self._exchange = ex
        xc = ex[1]
        rows, rids, rcnt, ret_index = xc.dispatch(x, ids)
        y_pad, ydest = K.expert_ffn_padded(rows, rids, 1, self.w1, self.w2, self.cfg.block_M, cfg=self.cfg.gemm_cfg,
                                           w1_interleaved=True)
        back = xc.combine_rows(y_pad, ydest, rcnt)
        return K.combine(back, ret_index, wts)

    def _ep(self, x, ids):
        """Expert parallel over host collectives: (token, expert) pairs travel to the expert's
        rank and back (two variable-size all-to-alls; one host sync for the split sizes)."""
        from ..ops import moe as K
        from ..parallel import collectives as C
        m = self.mesh
        W = m.world
        n = self.cfg.n_experts // W
        flat_ids = ids.reshape(-1).long()
        dest_rank = torch.div(flat_ids, n, rounding_mode="floor")
        order = torch.argsort(dest_rank, stable=True)
        send_counts = torch.bincount(dest_rank, minlength=W)
        tok = torch.div(order, self.cfg.topk, rounding_mode="floor")
        payload = x[tok]
        local_e = (flat_ids[order] - dest_rank[order] * n).to(payload.dtype).unsqueeze(1)
        # expert id rides along as one extra column (exact in bf16/fp32 for < 256 experts)
        recv, rc = C.all_to_all_v(torch.cat([payload, local_e], 1), send_counts)
        recv_rows, recv_e = recv[:, :-1].contiguous(), recv[:, -1].round().to(torch.int32)
        y_pad, dest = K.expert_ffn_padded(recv_rows, recv_e, 1, self.w1, self.w2, self.cfg.block_M,
                                          cfg=self.cfg.gemm_cfg, w1_interleaved=True)
        y_local = y_pad[dest.long()]
        y_back, _ = C.all_to_all_v(y_local, rc)
        y = torch.empty_like(y_back)
        y[order] = y_back
        return y
