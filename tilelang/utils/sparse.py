"""2:4 structured-sparsity helpers for ``T.gemm_sp`` (reference ``tilelang/utils/sparse.py``).

The reference compresses with CUTLASS (sm90) or ``torch.sparse.to_sparse_semi_structured`` (sm80)
and its metadata layout is an NVIDIA ``mma.sp`` format.  gfx950's ``v_smfmac`` consumes a simpler
format, produced here with plain tensor ops (CPU or GPU):

* ``A_sparse [M, K/2]``: the two kept values of each group of 4 along K, in K order;
* ``E [M, K/16]`` int16: word ``c`` covers original K ``[16c, 16c+16)`` (4 groups, 8 kept
  values); bits ``[2v+1:2v]`` hold the in-group position (0..3) of kept value ``v``.

A group with fewer than two non-zeros keeps explicit zeros (any positions are valid then).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

E_FACTOR = 16          # original K elements per metadata word
E_DTYPE = torch.int16


def _check(A: torch.Tensor):
    if A.dim() != 2:
        raise ValueError(f"2:4 compression expects a 2-D tensor, got shape {tuple(A.shape)}")
    if A.shape[1] % E_FACTOR:
        raise ValueError(f"2:4 compression needs K % {E_FACTOR} == 0, got K={A.shape[1]}")


def compress(A: torch.Tensor, transposed: bool = False, block_k: Optional[int] = None, arch: Optional[str] = None,
             **kwargs) -> Tuple[torch.Tensor, torch.Tensor]:
    """Compress a 2:4-sparse ``A [M, K]`` (``[K, M]`` with ``transposed``) into ``(A_sparse, E)``.

    With ``transposed`` the input is ``[K, M]`` and ``A_sparse`` is returned as ``[K/2, M]``
    (the ``T.gemm_sp(..., transpose_A=True)`` operand); ``E`` is always ``[M, K/16]``.
    ``block_k`` / ``arch`` are accepted for API parity: the gfx950 format does not depend on the
    tile size.  Raises if a group of 4 holds more than two non-zeros."""
    del block_k, arch, kwargs
    At = A.t() if transposed else A
    _check(At)
    M, K = At.shape
    g = At.reshape(M, K // 4, 4)
    nz = g != 0
    if bool((nz.sum(-1) > 2).any()):
        raise ValueError("tensor is not 2:4 sparse: some group of 4 along K has more than 2 non-zeros")
    # rank positions: non-zeros first (stable, by position), pad with the lowest zero positions
    pos = torch.arange(4, device=A.device).expand(M, K // 4, 4)
    key = (~nz).to(torch.int64) * 4 + pos
    order = key.argsort(dim=-1, stable=True)[..., :2]
    order, _ = order.sort(dim=-1)
    vals = torch.gather(g, -1, order)                                   # [M, K/4, 2]
    A_sp = vals.reshape(M, K // 2)
    codes = order.reshape(M, K // 16, 8).to(torch.int32)                # 8 positions per word
    shifts = (2 * torch.arange(8, device=A.device, dtype=torch.int32))
    word = (codes << shifts).sum(-1)                                    # < 2^16
    E = torch.where(word >= 32768, word - 65536, word).to(E_DTYPE)
    if transposed:
        A_sp = A_sp.t().contiguous()
    return A_sp.contiguous(), E.contiguous()


def decompress(A_sp: torch.Tensor, E: torch.Tensor, transposed: bool = False) -> torch.Tensor:
    """Inverse of :func:`compress`: the dense ``[M, K]`` (``[K, M]`` with ``transposed``) tensor."""
    As = A_sp.t() if transposed else A_sp
    M, K2 = As.shape
    K = 2 * K2
    word = E.to(torch.int32) & 0xFFFF
    shifts = 2 * torch.arange(8, device=E.device, dtype=torch.int32)
    codes = ((word.unsqueeze(-1) >> shifts) & 3).reshape(M, K // 4, 2).to(torch.int64)
    out = torch.zeros(M, K // 4, 4, dtype=As.dtype, device=As.device)
    out.scatter_(-1, codes, As.reshape(M, K // 4, 2))
    out = out.reshape(M, K)
    return out.t().contiguous() if transposed else out


def randn_semi_sparse(M: int, K: int, dtype=torch.float16, device="cuda", transposed: bool = False):
    """Random ``[M, K]`` tensor with 2:4 sparsity along K (``[K, M]`` if ``transposed``)."""
    t = torch.randn((M, K), dtype=torch.float, device=device).view(M, -1, 4)
    drop = t.abs().topk(2, dim=-1, largest=False).indices
    t.scatter_(-1, drop, 0)
    t = t.view(M, K)
    if transposed:
        t = t.t().contiguous()
    return t.to(dtype)


def randint_semi_sparse(M: int, K: int, low: int, high: int, dtype=torch.int32, device="cuda",
                        transposed: bool = False):
    """Random integer ``[M, K]`` tensor with 2:4 sparsity along K."""
    t = torch.randint(low, high, (M, K), dtype=torch.int32, device=device).view(M, -1, 4)
    drop = torch.rand(t.shape, device=device).topk(2, dim=-1).indices
    t.scatter_(-1, drop, 0)
    t = t.view(M, K)
    if transposed:
        t = t.t().contiguous()
    return t.to(dtype)
