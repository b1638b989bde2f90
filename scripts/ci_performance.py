#!/usr/bin/env python3
"""Performance regression check between two revisions (reference: maint/scripts/ci_performance.py).

The reference runs its ``performance.py`` under two virtualenvs and prints the two latency /
TFLOPS lines side by side.  Here the unit of comparison is the headline ``bench.py`` JSON line
(aggregate TFLOPS plus the per-phase GEMM / attention / MoE rates) on ONE MI355X:

    python scripts/ci_performance.py --base origin/main              # base ref vs the working tree
    python scripts/ci_performance.py --base HEAD~5 --repeats 3 --max-regression 3

* the base revision is checked out with ``git worktree`` into a scratch directory and its native
  extensions are built there (``setup.py build_ext --inplace``), so the two trees never share a
  ``.so`` or a kernel cache entry (``TILELANG_CACHE_DIR`` is per tree);
* every run happens in its own child process, base and current interleaved (A B A B ...) so that
  clock / thermal drift over the job hits both sides equally; the median of ``--repeats`` runs is
  reported;
* exit status 1 when any tracked rate of the current tree is more than ``--max-regression`` percent
  below the base (the CI job fails), 0 otherwise.  ``--json`` writes the table for the PR bot.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACKED = ("value", "gemm_tflops", "attn_tflops", "moe_tflops_per_gpu")


def parse_bench(stdout: str) -> dict:
    """The last JSON object line that names the metric (bench.py prints exactly one)."""
    for line in reversed(stdout.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise ValueError("no bench JSON line in output:\n" + stdout[-2000:])


def run_bench(tree: str, bench_args, timeout: int) -> dict:
    env = dict(os.environ)
    env["TILELANG_CACHE_DIR"] = os.path.join(tree, ".tl_cache_ci")
    env["PYTHONPATH"] = tree + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "bench.py", *bench_args], cwd=tree, env=env, capture_output=True, text=True,
                       timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"bench.py failed in {tree} (rc {r.returncode}):\n{r.stderr[-3000:]}")
    return parse_bench(r.stdout)


def prepare_base(ref: str, scratch: str) -> str:
    path = os.path.join(scratch, "base")
    subprocess.run(["git", "worktree", "add", "--detach", path, ref], cwd=ROOT, check=True, capture_output=True)
    r = subprocess.run([sys.executable, "setup.py", "build_ext", "--inplace"], cwd=path, capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"building {ref} failed:\n{r.stderr[-3000:]}")
    return path


def summarize(runs):
    out = {}
    for key in TRACKED:
        vals = [r[key] for r in runs if isinstance(r.get(key), (int, float))]
        out[key] = statistics.median(vals) if vals else None
    out["ms_per_step"] = statistics.median(r["ms_per_step"] for r in runs)
    return out


def compare(base: dict, cur: dict, max_regression: float):
    rows, regressed = [], []
    for key in TRACKED + ("ms_per_step",):
        b, c = base.get(key), cur.get(key)
        if b is None or c is None:
            rows.append([key, b, c, None])
            continue
        higher_better = key != "ms_per_step"
        delta = (c - b) / b * 100.0 * (1 if higher_better else -1)
        rows.append([key, round(b, 2), round(c, 2), round(delta, 2)])
        if key in TRACKED and delta < -max_regression:
            regressed.append(key)
    return rows, regressed


def format_table(rows) -> str:
    headers = ["rate", "base", "current", "change %"]
    try:
        from tabulate import tabulate
        return tabulate(rows, headers=headers, tablefmt="github", numalign="decimal")
    except ImportError:  # pragma: no cover - tabulate ships in the image
        lines = [" | ".join(headers)] + [" | ".join(str(x) for x in r) for r in rows]
        return "\n".join(lines)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--base", default="origin/main", help="git revision to compare against")
    p.add_argument("--repeats", type=int, default=3)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--max-regression", type=float, default=3.0, help="percent")
    p.add_argument("--timeout", type=int, default=900)
    p.add_argument("--json", help="write the comparison here")
    p.add_argument("--extra", nargs=argparse.REMAINDER, default=[], help="more bench.py arguments")
    a = p.parse_args(argv)
    bench_args = ["--steps", str(a.steps), "--warmup", str(a.warmup), *a.extra]
    scratch = tempfile.mkdtemp(prefix="tl_ci_perf_")
    base_tree = None
    try:
        base_tree = prepare_base(a.base, scratch)
        base_runs, cur_runs = [], []
        for i in range(a.repeats):
            base_runs.append(run_bench(base_tree, bench_args, a.timeout))
            cur_runs.append(run_bench(ROOT, bench_args, a.timeout))
            print(f"repeat {i}: base {base_runs[-1]['value']:.1f} current {cur_runs[-1]['value']:.1f} "
                  f"{cur_runs[-1]['unit']}", flush=True)
        rows, regressed = compare(summarize(base_runs), summarize(cur_runs), a.max_regression)
        print(format_table(rows))
        if a.json:
            with open(a.json, "w") as f:
                json.dump(dict(base=a.base, rows=rows, regressed=regressed, base_runs=base_runs, current_runs=cur_runs),
                          f, indent=1)
        if regressed:
            print(f"REGRESSION > {a.max_regression}% in: {', '.join(regressed)}")
            return 1
        return 0
    finally:
        if base_tree is not None:
            subprocess.run(["git", "worktree", "remove", "--force", base_tree], cwd=ROOT, capture_output=True)
        shutil.rmtree(scratch, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
