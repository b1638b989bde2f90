"""Math-precision probe for gfx950 (reference ``maint/precision/compare_ops.py`` +
``cuda_ops.cu:125-171``): every transcendental / division the DSL exposes, computed by

  * TileLang (precise: OCML / correctly-rounded paths, the default),
  * TileLang fast math (``tl.enable_fast_math``: ``v_exp_f32`` / ``v_log_f32`` / ``v_sin_f32`` ...
    hardware transcendentals, what the attention kernels use),
  * PyTorch on the same device,

and compared element-wise against a float64 reference of the same float32 inputs (max / mean
absolute and relative error, plus max ULP distance in float32).  ``python -m
tilelang.tools.precision --out docs/PRECISION.md`` writes the table; on a CPU-only machine the
CPU target is probed instead (fast math is then the same code as precise).
"""
from __future__ import annotations

import argparse
import math
from typing import Dict, Tuple

import torch

import tilelang
import tilelang.language as T

# op -> (input low, input high, torch fp64 reference, DSL expression builder)
OPS = {
    "div": (-100.0, 100.0, lambda x, y: x / y, lambda a, b: a / b),
    "reciprocal": (0.01, 100.0, lambda x, y: 1.0 / x, lambda a, b: T.rcp(a)),
    "exp": (-10.0, 10.0, lambda x, y: torch.exp(x), lambda a, b: T.exp(a)),
    "exp2": (-20.0, 20.0, lambda x, y: torch.exp2(x), lambda a, b: T.exp2(a)),
    "log": (0.001, 1000.0, lambda x, y: torch.log(x), lambda a, b: T.log(a)),
    "log2": (0.001, 1000.0, lambda x, y: torch.log2(x), lambda a, b: T.log2(a)),
    "sin": (-math.pi, math.pi, lambda x, y: torch.sin(x), lambda a, b: T.sin(a)),
    "cos": (-math.pi, math.pi, lambda x, y: torch.cos(x), lambda a, b: T.cos(a)),
    "sqrt": (0.0, 100.0, lambda x, y: torch.sqrt(x), lambda a, b: T.sqrt(a)),
    "rsqrt": (0.01, 100.0, lambda x, y: torch.rsqrt(x), lambda a, b: T.rsqrt(a)),
    "tanh": (-5.0, 5.0, lambda x, y: torch.tanh(x), lambda a, b: T.tanh(a)),
}

_TORCH32 = {
    "div": lambda x, y: x / y, "reciprocal": torch.reciprocal, "exp": torch.exp, "exp2": torch.exp2,
    "log": torch.log, "log2": torch.log2, "sin": torch.sin, "cos": torch.cos, "sqrt": torch.sqrt,
    "rsqrt": torch.rsqrt, "tanh": torch.tanh,
}


def _kernel(op: str, n: int, fast: bool, target: str):
    build = OPS[op][3]

    @T.prim_func
    def probe(A: T.Tensor((n, ), "float32"), Bv: T.Tensor((n, ), "float32"), C: T.Tensor((n, ), "float32")):
        with T.Kernel(T.ceildiv(n, 1024), threads=256) as bx:
            for i in T.Parallel(1024):
                C[bx * 1024 + i] = build(A[bx * 1024 + i], Bv[bx * 1024 + i])

    cfg = {"tl.enable_fast_math": True} if fast else {"tl.disable_fast_math": True}
    return tilelang.compile(probe, out_idx=[2], target=target, pass_configs=cfg)


def _inputs(op: str, n: int, device, seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    lo, hi = OPS[op][0], OPS[op][1]
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.rand(n, generator=g, dtype=torch.float64) * (hi - lo) + lo
    y = torch.rand(n, generator=g, dtype=torch.float64) * 99.0 + 1.0  # divisors in [1, 100)
    y = torch.where(torch.rand(n, generator=g) < 0.5, -y, y)
    return x.float().to(device), y.float().to(device)


def _ulp32(x: torch.Tensor) -> torch.Tensor:
    """Spacing of float32 at |x| (as float64)."""
    ax = x.abs().float().clamp_min(torch.finfo(torch.float32).tiny)
    return (torch.nextafter(ax, torch.full_like(ax, float("inf"))) - ax).double()


def error_stats(out: torch.Tensor, ref: torch.Tensor) -> Dict[str, float]:
    o = out.double().cpu()
    r = ref.double().cpu()
    ok = torch.isfinite(r) & torch.isfinite(o)
    ae = (o - r).abs()[ok]
    re = ae / r.abs()[ok].clamp_min(1e-30)
    ulp = ae / _ulp32(r[ok])
    return dict(max_abs=float(ae.max()), mean_abs=float(ae.mean()), max_rel=float(re.max()),
                mean_rel=float(re.mean()), max_ulp=float(ulp.max()), nonfinite=int((~ok).sum()))


def run(device: str = "cuda", n: int = 1 << 20, seed: int = 0, ops=None) -> Dict[str, Dict[str, Dict[str, float]]]:
    target = "cpu" if device == "cpu" else "hip"
    res = {}
    for op in (ops or OPS):
        x, y = _inputs(op, n, device, seed)
        ref = OPS[op][2](x.double().cpu(), y.double().cpu())
        rows = {}
        rows["TileLang (precise)"] = error_stats(_kernel(op, n, False, target)(x, y), ref)
        rows["TileLang (fast math)"] = error_stats(_kernel(op, n, True, target)(x, y), ref)
        f = _TORCH32[op]
        rows["PyTorch"] = error_stats(f(x, y) if op == "div" else f(x), ref)
        res[op] = rows
    return res


def to_markdown(res, device_name: str) -> str:
    out = [f"# Math precision on {device_name}", "",
           "float32 inputs, errors against a float64 reference of the same inputs "
           "(`python -m tilelang.tools.precision`; reference counterpart `maint/precision/README.md`).", ""]
    for op, rows in res.items():
        lo, hi = OPS[op][0], OPS[op][1]
        out += [f"### {op}  (x in [{lo:g}, {hi:g}])", "",
                "| Implementation | Max Abs Error | Mean Abs Error | Max Rel Error | Mean Rel Error | Max ULP |",
                "|---|---|---|---|---|---|"]
        for name, s in rows.items():
            out.append(f"| {name} vs Double | {s['max_abs']:.3e} | {s['mean_abs']:.3e} | {s['max_rel']:.3e} | "
                       f"{s['mean_rel']:.3e} | {s['max_ulp']:.1f} |")
        out.append("")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = run(a.device, a.n)
    name = torch.cuda.get_device_name() + " (gfx950)" if a.device != "cpu" else "the CPU target"
    md = to_markdown(res, name)
    print(md)
    if a.out:
        with open(a.out, "w") as f:
            f.write(md + "\n")


if __name__ == "__main__":
    main()
