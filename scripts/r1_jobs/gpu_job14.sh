#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job14.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 400 python -u scripts/gpu_sweep_smla.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/dequantize_gemm/example_dequant_gemm_mxfp4.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/dequantize_gemm/example_dequant_gemm_mxfp4.py --m 4096 >> $O 2>&1
tail -12 $O
