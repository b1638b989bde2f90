#!/bin/bash
# Perf of kernels whose copies became LDS-DMA + bench with the extended result guard (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
: > gpurun_out/perf3.log
run() { local name=$1; shift; echo "=== $name" >> gpurun_out/perf3.log; timeout -k 10 240 "$@" >> gpurun_out/perf3.log 2>&1 || { echo "FAILED $name"; tail -20 gpurun_out/perf3.log; exit 1; }; }
run fa_bwd python examples/flash_attention/example_mha_bwd.py
run fa_bwd_causal python examples/flash_attention/example_mha_bwd.py --causal
run sink_window python examples/attention_sink/example_gqa_sink_fwd_bhsd.py --window_size 128
run sink_causal python examples/attention_sink/example_gqa_sink_fwd_bhsd.py
run gqa_decode python examples/flash_decoding/example_gqa_decode.py
run mla_paged python examples/deepseek_mla/example_mla_decode_paged.py
run bench python bench.py --steps 20 --warmup 5
grep -v "amdgpu.ids" gpurun_out/perf3.log
