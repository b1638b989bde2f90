#!/bin/bash
# Fresh numbers for the secondary kernels' example mains, default build and with the pipelined
# loops unrolled (TL_PIPELINE_UNROLL=2), each step under its own time limit.
#   bash scripts/secondary_sweep.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/secondary}
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
for u in 0 2; do
  for ex in deepseek_v32/sparse_mla_bwd.py deepseek_nsa/example_nsa_fwd.py deepseek_nsa/example_nsa_bwd.py \
            flash_attention/example_mha_bwd_varlen.py linear_attention/example_linear_attn_fwd.py gdn/example_gdn.py; do
    n=$(basename $ex .py)
    TL_PIPELINE_UNROLL=$u timeout -k 10 240 python -u examples/$ex > $OUT/${n}_u$u.log 2>&1 || { echo "$n u$u rc=$?"; tail -3 $OUT/${n}_u$u.log; exit 1; }
    echo "u$u $(grep -hE 'ms|TFLOPS' $OUT/${n}_u$u.log | grep -v amdgpu | tail -2 | tr '\n' ' ')"
  done
done
