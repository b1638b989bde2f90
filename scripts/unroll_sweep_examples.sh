#!/bin/bash
# Example mains (their own timing lines) built as they are and with every pipelined main loop
# unrolled (TL_PIPELINE_UNROLL=2), one example after the other, each under its own time limit.
#   bash scripts/unroll_sweep_examples.sh out_dir example.py [example.py ...]
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
for ex in "$@"; do
  n=$(basename $ex .py)
  for u in 0 2; do
    TL_PIPELINE_UNROLL=$u timeout -k 10 150 python -u $ex > $OUT/${n}_u$u.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$n u$u rc=$rc: $(tail -1 $OUT/${n}_u$u.log | cut -c1-150)"; [ $rc -ge 124 ] && exit $rc; continue; fi
    echo "$n u$u: $(grep -hE '[0-9] ?ms|TFLOPS|TF\b|GB/s' $OUT/${n}_u$u.log | grep -v amdgpu | tail -3 | cut -c1-160 | tr '\n' ' ')"
  done
done
