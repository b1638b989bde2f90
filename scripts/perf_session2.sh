#!/bin/bash
# Round-2 session-2: A/B of FA compile flags + young-half priority, MoE padded-tile skip, perf of the
# new examples (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
run() { local name=$1; shift; echo "=== $name" >> gpurun_out/perf2.log; timeout -k 10 300 "$@" >> gpurun_out/perf2.log 2>&1 || { echo "FAILED $name rc=$?" >> gpurun_out/perf2.log; tail -20 gpurun_out/perf2.log; exit 1; }; }
: > gpurun_out/perf2.log
run moe_skip python scripts/prof_moe.py 20 --skip-ab
run flags python scripts/flag_sweep.py
run tests python -u -m pytest tests/test_bitnet.py tests/test_moe.py -m gpu -x -v --timeout 120 --timeout-method thread
run bitnet python examples/bitnet-1.58b/tilelang_bitnet_158_int8xint2.py
run varlen_logits python examples/flash_decoding/example_gqa_decode_varlen_logits.py --batch_size 1 --k_seqlen 8192
run varlen_logits_b16 python examples/flash_decoding/example_gqa_decode_varlen_logits.py --batch_size 16 --k_seqlen 8192 --test_varlen
run varlen_logits_paged python examples/flash_decoding/example_gqa_decode_varlen_logits.py --batch_size 16 --k_seqlen 8192 --paged
run mha_inference python examples/flash_decoding/example_mha_inference.py
run nsa_varlen python examples/deepseek_nsa/example_nsa_fwd_varlen.py
run nsa_decode python examples/deepseek_nsa/example_nsa_decode.py
run w4a8 python examples/dequantize_gemm/example_dequant_gemm_w4a8.py --m 4096 --n 4096 --k 4096
run gemv_int4 python examples/dequantize_gemm/example_dequant_gemv_fp16xint4.py
run grouped_mxfp4 python examples/dequantize_gemm/example_dequant_groupedgemm_bf16_mxfp4.py --m 4096 --n 4096 --k 4096 --topk 4 --E 32
grep -v "^tests/\|PASSED\|^$" gpurun_out/perf2.log | tail -80
