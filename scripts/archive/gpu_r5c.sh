#!/bin/bash
# driver-config bench (x2) + MALL flush probe + rocprofv3 kernel stats of the bench
set -u
OUT=${1:-gpurun_out/r5c}
mkdir -p $OUT
export PYTHONPATH=$PWD:${PYTHONPATH:-}
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || exit $?
  python - $OUT/bench_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print({k: d[k] for k in ("value", "ms_per_step", "step_ms_first", "step_ms_median", "step_ms_last", "gemm_tflops",
                         "gemm_vendor_tflops", "attn_tflops", "moe_tflops_per_gpu", "prewarm_ms")})
PY
done
timeout -k 10 300 python -u scripts/mall_flush_probe.py > $OUT/mall.log 2>&1; echo "mall rc=$?"; cat $OUT/mall.log | grep copy
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$OUT/prof.log 2>&1; echo "rocprof rc=$?"
