"""Child process of an isolated autotune run: ``python -m tilelang.autotuner.worker <job dir>``.

The parent (``AutoTuner.run`` with ``isolate=True``) writes ``job.pkl`` (cloudpickle: the kernel
factory, its arguments, one config, the check program) and ``inputs.pt`` (host copies of the
inputs, ``torch.save`` of plain tensors), starts this module in a NEW SESSION and kills the whole
process group when the config exceeds its wall-clock budget -- so a config whose kernel never
returns costs one budget, not the tuning run (the in-process ``run_with_timeout`` can only
interrupt Python, never a launch that does not return).  The result goes to ``result.json``.
"""
from __future__ import annotations

import json
import os
import sys
import traceback


def main(d: str) -> int:
    res = {}
    try:
        import cloudpickle
        import torch
        with open(os.path.join(d, "job.pkl"), "rb") as f:
            job = cloudpickle.load(f)
        host = torch.load(os.path.join(d, "inputs.pt"), weights_only=True)
        merged = dict(job["kwargs"])
        merged.update(job["cfg"])
        kernel = job["fn"](*job["args"], **merged)
        dev = "cpu" if kernel.artifact.is_cpu else "cuda"
        inputs = [t.to(dev) if isinstance(t, torch.Tensor) else t for t in host]
        prof = kernel.get_profiler(job.get("supply_type"))
        if job.get("manual_check_prog") is not None:
            job["manual_check_prog"](kernel(*inputs), *inputs)
        elif job.get("ref_prog") is not None:
            prof.assert_allclose(job["ref_prog"], inputs, job["atol"], job["rtol"], job["max_mismatched_ratio"])
        res["latency"] = prof.do_bench(None, job["warmup"], job["rep"], input_tensors=inputs)
    except BaseException as e:  # noqa: BLE001
        res["error"] = f"{type(e).__name__}: {e}"
        res["trace"] = traceback.format_exc()[-2000:]
    with open(os.path.join(d, "result.json.tmp"), "w") as f:
        json.dump(res, f)
    os.replace(os.path.join(d, "result.json.tmp"), os.path.join(d, "result.json"))
    return 0 if "latency" in res else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
