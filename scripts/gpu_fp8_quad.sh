#!/bin/bash
# fp8 quad loop: numerics (fp8 + fp16 regression) and the same-process A/B against the generic
# pipeline and hipBLASLt _scaled_mm.  Usage: bash scripts/gpu_fp8_quad.sh gpurun_out/fp8q
set -o pipefail
OUT=${1:-gpurun_out/fp8q}
mkdir -p "$OUT"
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm_phased.py -k "quad" > "$OUT/tests.log" 2>&1 &&
timeout -k 10 500 python -u scripts/gemm_quad_ab.py --dtype float8_e4m3fn --check 256,256,128 512,256,8320 1024,512,384 \
  --shapes 8192,8192,1024 8192,8192,2048 8192,8192,4096 8192,8192,8192 > "$OUT/ab.log" 2>&1
