"""Shared plumbing of the benchmark harness (benchmarks/*/benchmark_*.py): one process per table,
every candidate config compiled, checked against an fp32 definition and timed with do_bench
(cold caches; ``flush_mode="write"`` -- the reference's zero-fill flush -- so the H800 column of
the reference README is compared like for like), the best config per row kept.

Each script prints a markdown table (MI355X | H800 reference | ratio | vendor library) and writes
``<out>/<name>.json``; ``benchmarks/run_all.sh`` runs every table on the GPU box.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Callable, Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "examples", "gemm"), os.path.join(ROOT, "examples", "gemm_fp8"),
          os.path.join(ROOT, "examples", "linear_attention"), os.path.join(ROOT, "examples", "blocksparse_attention"),
          os.path.join(ROOT, "examples", "flash_attention")):
    if p not in sys.path:
        sys.path.insert(0, p)


def bench(fn: Callable, warmup: int = 10, rep: int = 50) -> float:
    """Cold-cache mean latency in ms (write flush, as the reference's do_bench)."""
    from tilelang.profiler import do_bench
    return do_bench(fn, warmup=warmup, rep=rep, flush_mode="write")


def tune(name: str, configs: List[dict], build: Callable[[dict], Callable], check: Callable[[Callable], None],
         warmup: int = 10, rep: int = 50, log=print) -> Dict:
    """Compile/check/time every config; returns {"config", "ms", "all": [...]} of the fastest."""
    best = {"config": None, "ms": float("inf"), "all": []}
    for cfg in configs:
        t0 = time.time()
        try:
            fn = build(cfg)
            check(fn)
            ms = bench(fn, warmup, rep)
        except Exception as e:  # noqa: BLE001 - a config that does not compile / fit / check is skipped
            best["all"].append({"config": cfg, "error": f"{type(e).__name__}: {str(e)[:160]}"})
            log(f"  [{name}] {cfg}: FAILED {type(e).__name__}: {str(e)[:160]}")
            continue
        best["all"].append({"config": cfg, "ms": ms})
        log(f"  [{name}] {cfg}: {ms:.4f} ms ({time.time() - t0:.1f}s)")
        if ms < best["ms"]:
            best["ms"], best["config"] = ms, cfg
    return best


def table(title: str, header: List[str], rows: List[List], out_dir: Optional[str], name: str, extra=None):
    lines = [f"### {title}", "", "| " + " | ".join(header) + " |", "|" + "---|" * len(header)]
    for r in rows:
        lines.append("| " + " | ".join(str(x) for x in r) + " |")
    text = "\n".join(lines)
    print(text, flush=True)
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"{name}.md"), "w") as f:
            f.write(text + "\n")
        with open(os.path.join(out_dir, f"{name}.json"), "w") as f:
            json.dump({"title": title, "header": header, "rows": rows, "extra": extra}, f, indent=1, default=str)
    return text


def out_dir_arg(default="gpurun_out/benchmarks"):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=default)
    ap.add_argument("--quick", action="store_true", help="first config only (smoke)")
    ap.add_argument("--rows", default=None, help="comma-separated subset of the table's rows")
    return ap.parse_args()
