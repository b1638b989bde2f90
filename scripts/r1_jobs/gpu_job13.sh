#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job13.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py tests/test_gpu_examples.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -k "sink or paged or grouped or mxfp4 or nsa or block_sparse" >> $O 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gpu_sweep.py sink '{}' '{"lazy_rescale":false}' '{"causal":false}' >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/deepseek_mla/example_mla_decode_paged.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/grouped_gemm/example_grouped_gemm_bwd.py --batch_sizes 1024,2048,512,4096 >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/dequantize_gemm/example_dequant_gemm_mxfp4.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/dequantize_gemm/example_dequant_gemm_mxfp4.py --m 4096 >> $O 2>&1
grep -v "^tests/\|PASSED" $O | tail -22
