"""Child process of a process-parallel autotune compile:
``python -m tilelang.autotuner.compile_worker <job.pkl>``.

Lowering is Python (GIL-bound): a thread pool overlaps the hipcc subprocesses but runs the passes of
all configs one after another.  ``AutoTuner.run`` with ``compile_backend="process"`` (or
``TILELANG_AUTOTUNE_COMPILE=process``) splits the configs over worker processes that each lower +
compile their share and store the kernels in the disk kernel cache (``cache/kernel_cache.py``,
keyed on the printed program); the parent's own compile of every config is then a cache hit (no
lowering, no hipcc).  Errors are reported back per config; the parent's compile re-raises them
with the usual message.
"""
from __future__ import annotations

import json
import os
import sys
import traceback


def main(job_path: str) -> int:
    import cloudpickle
    with open(job_path, "rb") as f:
        job = cloudpickle.load(f)
    errors = {}
    for i, cfg in job["configs"]:
        merged = dict(job["kwargs"])
        merged.update(cfg)
        try:
            job["fn"](*job["args"], **merged)
        except BaseException as e:  # noqa: BLE001 - an invalid config is not fatal
            errors[str(i)] = f"{type(e).__name__}: {e}"[:500]
            if os.environ.get("TILELANG_AUTOTUNE_DEBUG"):
                traceback.print_exc()
    out = job_path + ".result.json"
    with open(out + ".tmp", "w") as f:
        json.dump({"errors": errors}, f)
    os.replace(out + ".tmp", out)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
