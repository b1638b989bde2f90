"""Tensor supply for profiling / checking (reference ``tilelang/utils/tensor.py:24-309``)."""
from __future__ import annotations

from enum import Enum

from ..ir import dtypes as _dt


class TensorSupplyType(Enum):
    Integer = 1
    Uniform = 2
    Normal = 3
    Randn = 4
    Zero = 5
    One = 6
    Auto = 7


def get_tensor_supply(supply_type: TensorSupplyType = TensorSupplyType.Auto):

    def supply(shape, dtype, device="cuda"):
        import torch
        dt = _dt.as_dtype(dtype)
        tdt = _dt.to_torch(dt)
        shape = [int(s) for s in shape]
        st = supply_type
        if st == TensorSupplyType.Auto:
            st = TensorSupplyType.Normal if dt.is_float else TensorSupplyType.Integer
        if dt.is_fp8:
            return (torch.randn(shape, device=device) * 0.5).clamp(-8, 8).to(tdt)
        if st == TensorSupplyType.Integer:
            if dt.is_bool:
                return torch.randint(0, 2, shape, device=device).bool()
            if dt.is_float:
                return torch.randint(-2, 3, shape, device=device).to(tdt)
            hi = 3 if dt.bits > 1 else 2
            return torch.randint(-2 if dt.kind == "int" else 0, hi, shape, device=device).to(tdt)
        if st == TensorSupplyType.Uniform:
            return torch.empty(shape, device=device, dtype=tdt).uniform_(-1.0, 1.0)
        if st in (TensorSupplyType.Normal, TensorSupplyType.Randn):
            return torch.randn(shape, device=device).to(tdt)
        if st == TensorSupplyType.Zero:
            return torch.zeros(shape, device=device, dtype=tdt)
        if st == TensorSupplyType.One:
            return torch.ones(shape, device=device, dtype=tdt)
        raise ValueError(st)

    return supply


def torch_assert_close(a, b, rtol=1e-2, atol=1e-2, max_mismatched_ratio=0.001, verbose=False, base_name="LHS",
                       ref_name="RHS"):
    """Allclose with a tolerated fraction of mismatches (reference tensor.py:217)."""
    import torch
    a = a.float()
    b = b.float()
    if a.shape != b.shape:
        raise AssertionError(f"shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    diff = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (diff > tol) | torch.isnan(a) != torch.isnan(b)
    n_bad = int(bad.sum().item())
    ratio = n_bad / max(1, a.numel())
    if ratio > max_mismatched_ratio:
        raise AssertionError(f"{base_name} vs {ref_name}: {n_bad} / {a.numel()} elements ({ratio:.4%}) exceed "
                             f"atol={atol} rtol={rtol}; max abs diff {diff.max().item():.4g}")
    return True
