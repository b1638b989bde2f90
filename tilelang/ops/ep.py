"""Expert-parallel token exchange over xGMI with no host synchronisation (``tl/ep.h``).

``EPExchange(mesh, ...)`` moves a step's routed rows to the ranks that own their experts and the
expert results back, entirely from device kernels: senders store rows straight into the
receivers' symmetric IPC buffers at slots they compute themselves, and receivers learn the
counts from flag words — so, unlike a host ``all_to_all_v`` (split sizes on the host: one
device->host sync per layer), the MoE layer enqueues without ever waiting for the GPU.

Reference counterpart: the DeepSeek-V3.2 demo's expert parallelism
(``examples/deepseek_v32/inference/model.py:787-850``, local experts + ``dist.all_reduce``).

Per step (``epoch`` e, the same on every rank):
  dispatch  -> rows in every owner's RECV[e & 1] ([W*cap, H], slot order per source)
  recv_wait -> local expert id per receive slot (-1 = empty)           [FFN on RECV rows]
  ret       -> expert rows back into every source's RET[e & 1]
  ret_wait  -> pair j's result is RET row ``ret_index[j]``              [combine]
``cap`` = tokens * min(topk, experts per rank): the most pairs one rank can route to another,
so no capacity factor and no dropped tokens.
"""
from __future__ import annotations

import functools

import torch

import tilelang
import tilelang.language as T

_CTRL = 4096


def _flags():
    """hipcc flags of the exchange kernels: ``TL_EP_TIMEOUT_S`` (seconds) overrides the wall-clock
    budget of every bounded wait (tl/ep.h TL_EP_TIMEOUT_TICKS, 100 MHz ticks; default 20 s)."""
    import os
    s = os.environ.get("TL_EP_TIMEOUT_S")
    return [f"-DTL_EP_TIMEOUT_TICKS={int(float(s) * 1e8)}ull"] if s else []


def _tdt(dtype: torch.dtype) -> str:
    return {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[dtype]


def layout_bytes(W: int, cap: int, row_bytes: int):
    """(eids offset, recv offset, ret offset, total) of the symmetric buffer (tl/ep.h Layout)."""
    eids = _CTRL
    recv = (_CTRL + 2 * W * cap * 4 + 4095) & ~4095
    ret = recv + 2 * W * cap * row_bytes
    return eids, recv, ret, ret + 2 * W * cap * row_bytes


def _blocks(target: str, n: int) -> int:
    # the CPU target runs blocks one after another: tl/ep_cpu.h does a whole grid's work in one
    return 1 if target == "cpu" else n


@functools.lru_cache(maxsize=None)
def dispatch_kernel(n_tok: int, H: int, topk: int, W: int, n_loc: int, cap: int, dtype: str, blocks: int = 128,
                    target: str = "hip"):
    P = n_tok * topk
    blocks = _blocks(target, blocks)
    eb = {"float16": 2, "bfloat16": 2, "float32": 4}[dtype]

    @T.prim_func
    def ep_dispatch(x: T.Tensor((n_tok, H), dtype), ids: T.Tensor((P, ), "int32"), ret_index: T.Tensor((P, ), "int32"),
                    ws: T.int64, me: T.int32, epoch: T.int32, err: T.int64):
        with T.Kernel(blocks, threads=256) as bx:
            T.evaluate(T.call_extern("void", f"tl::ep::dispatch<{W}>", T.address_of(x[0, 0]), T.address_of(ids[0]),
                                     T.address_of(ret_index[0]), ws, me, epoch, err, P, topk, n_loc, cap, H * eb))

    return tilelang.compile(ep_dispatch, target=target, compile_flags=_flags())


@functools.lru_cache(maxsize=None)
def recv_wait_kernel(W: int, cap: int, row_bytes: int, blocks: int = 16, target: str = "hip"):
    blocks = _blocks(target, blocks)

    @T.prim_func
    def ep_recv_wait(ids_out: T.Tensor((W * cap, ), "int32"), cnt_out: T.Tensor((W, ), "int32"), ws: T.int64,
                     me: T.int32, epoch: T.int32, err: T.int64):
        with T.Kernel(blocks, threads=256) as bx:
            T.evaluate(T.call_extern("void", f"tl::ep::recv_wait<{W}>", T.address_of(ids_out[0]),
                                     T.address_of(cnt_out[0]), ws, me, epoch, err, cap, row_bytes))

    return tilelang.compile(ep_recv_wait, target=target, compile_flags=_flags())


@functools.lru_cache(maxsize=None)
def ret_kernel(rows: int, H: int, W: int, cap: int, dtype: str, blocks: int = 128, target: str = "hip"):
    blocks = _blocks(target, blocks)
    eb = {"float16": 2, "bfloat16": 2, "float32": 4}[dtype]

    @T.prim_func
    def ep_ret(y: T.Tensor((rows, H), dtype), ydest: T.Tensor((W * cap, ), "int32"), cnt: T.Tensor((W, ), "int32"),
               ws: T.int64, me: T.int32, epoch: T.int32, err: T.int64):
        with T.Kernel(blocks, threads=256) as bx:
            T.evaluate(T.call_extern("void", f"tl::ep::ret<{W}>", T.address_of(y[0, 0]), T.address_of(ydest[0]),
                                     T.address_of(cnt[0]), ws, me, epoch, err, cap, H * eb))

    return tilelang.compile(ep_ret, target=target, compile_flags=_flags())


@functools.lru_cache(maxsize=None)
def ret_wait_kernel(W: int, target: str = "hip"):

    @T.prim_func
    def ep_ret_wait(flag: T.Tensor((1, ), "int32"), ws: T.int64, me: T.int32, epoch: T.int32, err: T.int64):
        with T.Kernel(1, threads=64) as bx:
            T.evaluate(T.call_extern("void", f"tl::ep::ret_wait<{W}>", ws, me, epoch, err))

    return tilelang.compile(ep_ret_wait, target=target, compile_flags=_flags())


class EPExchange:
    """Device-driven EP exchange for one MoE layer shape on a ``ProcessMesh``: a GPU mesh runs
    tl/ep.h over IPC, a CPU (gloo) mesh runs the same protocol from tl/ep_cpu.h over /dev/shm."""

    def __init__(self, mesh, n_tok: int, H: int, topk: int, n_experts: int, dtype: torch.dtype, key: str = "ep"):
        W = mesh.world
        if n_experts % W:
            raise ValueError(f"{n_experts} experts do not split over {W} ranks")
        self.mesh, self.W, self.n_tok, self.H, self.topk = mesh, W, n_tok, H, topk
        self.n_loc = n_experts // W
        self.cap = n_tok * min(topk, self.n_loc)
        self.dtype = dtype
        self.row_bytes = H * torch.empty((), dtype=dtype).element_size()
        if self.row_bytes % 16:
            raise ValueError("EP rows must be a multiple of 16 bytes")
        self.eids_off, self.recv_off, self.ret_off, total = layout_bytes(W, self.cap, self.row_bytes)
        self.buf = mesh.symmetric_buffer(f"{key}:{W}x{self.cap}x{self.row_bytes}", total)
        self.epoch = 0
        dt = _tdt(dtype)
        self.target = "cpu" if mesh.device.type == "cpu" else "hip"
        self.k_dispatch = dispatch_kernel(n_tok, H, topk, W, self.n_loc, self.cap, dt, target=self.target)
        self.k_recv = recv_wait_kernel(W, self.cap, self.row_bytes, target=self.target)
        self.k_ret_wait = ret_wait_kernel(W, target=self.target)
        self._dummy = torch.zeros(1, dtype=torch.int32, device=mesh.device)

    def _args(self):
        return (int(self.buf.table.data_ptr()), int(self.mesh.rank), int(self.epoch), int(self.mesh.err.data_ptr()))

    def _watch(self, label):
        if self.target == "cpu":  # the CPU kernels have returned: read the error word now
            e = int(self.mesh.err.item())
            if e:
                self.mesh.err.zero_()
                raise self.mesh.error_decoder(f"{label} (EP rank {self.mesh.rank})", e)
            return
        from ..runtime import errors
        errors.record(self.mesh.err, f"{label} (EP rank {self.mesh.rank})", self.mesh.error_decoder)

    def recv_rows(self, parity: int) -> torch.Tensor:
        W, cap, H = self.W, self.cap, self.H
        per = W * cap * self.row_bytes
        return self.buf.view(self.recv_off + parity * per, (W * cap, H), self.dtype)

    def ret_rows(self, parity: int) -> torch.Tensor:
        W, cap, H = self.W, self.cap, self.H
        per = W * cap * self.row_bytes
        return self.buf.view(self.ret_off + parity * per, (W * cap, H), self.dtype)

    def dispatch(self, x: torch.Tensor, ids: torch.Tensor):
        """Send rows; returns (recv rows [W*cap, H], local expert ids [W*cap] (-1 empty),
        recv counts [W], ret_index [P])."""
        if self.target != "cpu":
            from ..runtime import errors
            errors.poll()
        self.epoch += 1
        p = self.epoch & 1
        flat = ids.reshape(-1).to(torch.int32).contiguous()
        ret_index = torch.empty(flat.numel(), dtype=torch.int32, device=x.device)
        self.k_dispatch(x.contiguous(), flat, ret_index, *self._args())
        rids = torch.empty(self.W * self.cap, dtype=torch.int32, device=x.device)
        rcnt = torch.empty(self.W, dtype=torch.int32, device=x.device)
        self.k_recv(rids, rcnt, *self._args())
        self._watch("ep dispatch")
        return self.recv_rows(p), rids, rcnt, ret_index

    def combine_rows(self, y: torch.Tensor, ydest: torch.Tensor, rcnt: torch.Tensor) -> torch.Tensor:
        """Return expert results; returns the RET row table [W*cap, H] (pair j: row ret_index[j])."""
        k = ret_kernel(y.shape[0], self.H, self.W, self.cap, _tdt(self.dtype), target=self.target)
        k(y.contiguous(), ydest.to(torch.int32).contiguous(), rcnt, *self._args())
        self.k_ret_wait(self._dummy, *self._args())
        self._watch("ep return")
        return self.ret_rows(self.epoch & 1)
