"""Test helpers (reference: tilelang/testing/__init__.py): device requirement decorators,
seeding, ``main()`` -> pytest, and a tolerance-reporting ``torch_assert_close``."""
from __future__ import annotations

import functools
import os
import random
import sys

import pytest


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def _gfx_arch() -> str:
    try:
        import torch
        return torch.cuda.get_device_properties(0).gcnArchName.split(":")[0]
    except Exception:  # noqa: BLE001
        return ""


def requires_rocm(fn=None):
    """Skip unless a ROCm GPU is visible."""
    dec = pytest.mark.skipif(not _gpu_available(), reason="needs a ROCm GPU")
    return dec(fn) if fn is not None else dec


def requires_gfx950(fn=None):
    """Skip unless the visible GPU is an MI355X-class gfx950."""
    dec = pytest.mark.skipif(not _gpu_available() or _gfx_arch() != "gfx950", reason="needs gfx950 (MI355X)")
    return dec(fn) if fn is not None else dec


def requires_multi_gpu(n: int = 2):
    try:
        import torch
        ok = torch.cuda.device_count() >= n
    except Exception:  # noqa: BLE001
        ok = False
    return pytest.mark.skipif(not ok, reason=f"needs >= {n} GPUs")


# the reference's CUDA-flavoured names map onto the ROCm checks
requires_cuda = requires_rocm
requires_package = lambda name: pytest.mark.skipif(  # noqa: E731
    __import__("importlib.util").util.find_spec(name) is None, reason=f"needs package {name}")


def set_random_seed(seed: int = 42) -> None:
    random.seed(seed)
    try:
        import numpy as np
        np.random.seed(seed)
    except Exception:  # noqa: BLE001
        pass
    try:
        import torch
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
    except Exception:  # noqa: BLE001
        pass


def torch_assert_close(a, b, rtol=1e-2, atol=1e-2, max_mismatched_ratio=0.0, base_name="a", ref_name="b"):
    """``torch.testing.assert_close`` that tolerates a fraction of mismatched elements and
    reports the worst ones (reference ``torch_assert_close``)."""
    import torch
    a, b = a.float(), b.float()
    bad = ~torch.isclose(a, b, rtol=rtol, atol=atol, equal_nan=True)
    ratio = bad.float().mean().item() if bad.numel() else 0.0
    if ratio > max_mismatched_ratio:
        diff = (a - b).abs()
        idx = diff.flatten().topk(min(5, diff.numel())).indices
        worst = [(int(i), a.flatten()[i].item(), b.flatten()[i].item()) for i in idx]
        raise AssertionError(f"{base_name} vs {ref_name}: {ratio:.4%} mismatched (> {max_mismatched_ratio:.4%}); "
                             f"max abs diff {diff.max().item():.4g}; worst (index, {base_name}, {ref_name}): {worst}")


def main(argv=None):
    """Run the calling test file with pytest (``if __name__ == "__main__": tilelang.testing.main()``)."""
    frame = sys._getframe(1)
    path = frame.f_globals.get("__file__")
    args = [path] if path else []
    args += list(argv if argv is not None else sys.argv[1:])
    sys.exit(pytest.main(args + ["-q"]))


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    return default if v is None else v.lower() in ("1", "true", "yes", "on")


__all__ = ["requires_rocm", "requires_cuda", "requires_gfx950", "requires_multi_gpu", "requires_package",
           "set_random_seed", "torch_assert_close", "main", "env_flag", "functools"]
