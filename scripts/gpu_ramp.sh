#!/bin/bash
# Clock-ramp study of the headline step: bench.py at the driver's --steps 20 --warmup 5 with
# different pre-warm lengths (per-step device times in the JSON), each run its own process.
set -u
OUT=${1:-gpurun_out/ramp}
mkdir -p $OUT
export PYTHONPATH=$PWD:${PYTHONPATH:-}
for pw in 0 0 100 300 1000; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --prewarm-ms $pw > $OUT/bench_pw$pw.log 2>&1 || exit $?
  python - $OUT/bench_pw$pw.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["prewarm_ms"], d["value"], d["ms_per_step"], d["step_ms_first"], d["step_ms_median"], d["step_ms_last"],
      d["gemm_tflops"], d["attn_tflops"], d["moe_tflops_per_gpu"], d["gemm_vendor_tflops"])
PY
done
