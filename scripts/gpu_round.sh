#!/bin/bash
# One GPU session: gpu tests, bench (N=1), rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; stop at the first fault/abort/timeout.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (not a GPU fault)
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
ok_rc $rc || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  ROOT=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o bench \
     --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/prof.log 2>&1)
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
fi
