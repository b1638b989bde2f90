#!/bin/bash
# Example mains (their own timing lines) built as they are and with an A/B switch set (default
# TL_PIPELINE_UNROLL=2: every pipelined main loop unrolled; SWITCH=TL_GEMM_RS_PIPE VAL=4 ...), one
# example after the other, each under its own time limit.
#   [SWITCH=NAME VAL=v] bash scripts/unroll_sweep_examples.sh out_dir example.py [example.py ...]
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
for ex in "$@"; do
  n=$(basename $ex .py)
  SW=${SWITCH:-TL_PIPELINE_UNROLL}
  for u in 0 ${VAL:-2}; do
    if [ $u = 0 ]; then unset $SW; else export $SW=$u; fi
    timeout -k 10 150 python -u $ex > $OUT/${n}_u$u.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$n u$u rc=$rc: $(tail -1 $OUT/${n}_u$u.log | cut -c1-150)"; [ $rc -ge 124 ] && exit $rc; continue; fi
    echo "$n u$u: $(grep -hE '[0-9] ?ms|TFLOPS|TF\b|GB/s' $OUT/${n}_u$u.log | grep -v amdgpu | tail -3 | cut -c1-160 | tr '\n' ' ')"
  done
  unset $SW
done
