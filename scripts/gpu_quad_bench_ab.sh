#!/bin/bash
# same-box A/B of the headline bench: round-5 start configuration (NN GEMM, no quad loops) vs now
# (NT GEMM + quad loops in the GEMM and the MoE expert GEMMs), alternating, driver configuration
set -u
OUT=${1:-gpurun_out/quad_bench_ab}
mkdir -p $OUT
export PYTHONPATH=$PWD:${PYTHONPATH:-}
for i in 1 2; do
  TL_GEMM_QUAD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --gemm-nn > $OUT/old_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/new_$i.log 2>&1 || exit $?
done
python - $OUT <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(os.path.basename(f), {k: d[k] for k in ("value", "ms_per_step", "gemm_tflops", "gemm_vendor_tflops",
                                                  "attn_tflops", "moe_tflops_per_gpu", "gemm_layout")})
PY
