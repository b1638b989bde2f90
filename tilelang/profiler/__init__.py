"""Profiler (reference ``tilelang/profiler/__init__.py:21-280``)."""
from __future__ import annotations

from typing import Callable, List, Optional

from ..utils.tensor import TensorSupplyType, get_tensor_supply, torch_assert_close
from .bench import do_bench


class Profiler:

    def __init__(self, kernel, supply_type: TensorSupplyType = TensorSupplyType.Auto):
        self.kernel = kernel
        self.supply_type = supply_type
        self.supply = get_tensor_supply(supply_type)
        self._inputs = None

    # the kernel's non-output buffer/scalar parameters
    def _input_params(self):
        from ..ir.buffer import Buffer
        out = []
        for i, p in enumerate(self.kernel.func.params):
            if i in (self.kernel.out_idx or []):
                continue
            out.append(p)
        return out

    def _get_inputs(self, with_output=False):
        from ..ir.buffer import Buffer
        from ..ir.expr import as_int
        if self._inputs is None:
            dev = "cpu" if self.kernel.artifact.is_cpu else "cuda"
            ins = []
            for p in self._input_params():
                if isinstance(p, Buffer):
                    shape = [as_int(s) for s in p.shape]
                    if any(s is None for s in shape):
                        raise ValueError(f"cannot synthesise input {p.name} with dynamic shape {p.shape}; pass "
                                         f"input_tensors")
                    ins.append(self.supply(shape, p.dtype, dev))
                else:
                    ins.append(1)
            self._inputs = ins
        return self._inputs

    def run_once(self, func: Optional[Callable] = None):
        ins = self._get_inputs()
        return (func or self.kernel)(*ins)

    def assert_allclose(self, reference_program: Callable, input_tensors=None, atol: float = 1e-2,
                        rtol: float = 1e-2, max_mismatched_ratio: float = 0.01):
        ins = input_tensors or self._get_inputs()
        out = self.kernel(*ins)
        ref = reference_program(*ins)
        outs = out if isinstance(out, (list, tuple)) else [out]
        refs = ref if isinstance(ref, (list, tuple)) else [ref]
        for o, r in zip(outs, refs):
            torch_assert_close(o, r, rtol=rtol, atol=atol, max_mismatched_ratio=max_mismatched_ratio)

    def assert_consistent(self, repeat: int = 10):
        """Run several times and require bit-identical outputs (catches races)."""
        import torch
        ins = self._get_inputs()
        first = self.kernel(*ins)
        firsts = first if isinstance(first, (list, tuple)) else [first]
        for _ in range(repeat):
            o = self.kernel(*ins)
            os_ = o if isinstance(o, (list, tuple)) else [o]
            for a, b in zip(firsts, os_):
                if not torch.equal(a, b):
                    raise AssertionError("kernel outputs differ between runs (race or uninitialised data)")

    def do_bench(self, func: Optional[Callable] = None, warmup: int = 25, rep: int = 100, n_warmup: int = 0,
                 n_repeat: int = 0, input_tensors: Optional[List] = None, backend: str = "event",
                 quantiles=None, return_mode: str = "mean"):
        fn = func or self.kernel
        if func is not None and _takes_no_args(func):
            # ``profiler.do_bench(lambda: kernel(a, b))``: a closure over its own inputs
            ins = []
        else:
            ins = input_tensors or self._get_inputs()
        if self.kernel.artifact.is_cpu:
            import time
            fn(*ins)
            t = time.perf_counter()
            n = max(1, n_repeat or 3)
            for _ in range(n):
                fn(*ins)
            return (time.perf_counter() - t) / n * 1e3
        return do_bench(lambda: fn(*ins), warmup=warmup, rep=rep, _n_warmup=n_warmup, _n_repeat=n_repeat,
                        backend=backend, quantiles=quantiles, return_mode=return_mode)


def _takes_no_args(fn) -> bool:
    import inspect
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return False
    return all(p.default is not inspect.Parameter.empty or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD)
               for p in sig.parameters.values())


__all__ = ["Profiler", "do_bench"]
