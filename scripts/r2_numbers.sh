#!/bin/bash
# Round-2 example numbers on one MI355X (each example's own main(): correctness check + timing).
set -u
cd "$(dirname "$0")/.."
export PYTHONPATH=$(pwd)${PYTHONPATH:+:$PYTHONPATH}
OUT=gpurun_out/r2_numbers.log
: > $OUT
run() {  # name, dir, script args...
  local name=$1 dir=$2; shift 2
  echo "=== $name" >> $OUT
  (cd examples/$dir && timeout -k 10 240 python -u "$@" >> ../../$OUT 2>&1) || echo "FAILED rc=$?" >> $OUT
}
run sink_gqa_causal attention_sink example_gqa_sink_fwd_bhsd.py
run fa_persistent amd example_amd_flash_attn_fwd.py --heads 64 --seq_len 4096
run fa_persistent_causal amd example_amd_flash_attn_fwd.py --heads 64 --seq_len 4096 --is_causal
run gdn_bwd gdn example_gdn_bwd.py --seq 8192 --heads 16
run nsa_bwd deepseek_nsa example_nsa_bwd.py
run linear_attn_bwd linear_attention example_linear_attn_bwd.py
run varlen_bwd flash_attention example_mha_bwd_varlen.py
run minference minference example_vertical_slash_sparse_attn.py
run intrinsics_gemm gemm example_gemm_intrinsics.py
grep -v amdgpu.ids $OUT
