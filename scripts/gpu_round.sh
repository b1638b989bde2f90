#!/bin/bash
# One GPU session: gpu tests, bench (N=1), rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; stop at the first fault/abort/timeout.
#   TESTS=<pytest path/-k args>  (default: tests)     PROFILE=0|1 (default 1)    BENCH=0|1 (default 1)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (not a GPU fault)
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -v -m gpu -x --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $OUT/pytest_gpu.log | tail -5
ok_rc $rc || exit $rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-1}" = "1" ]; then
  ROOT=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o bench \
     --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 5 > $ROOT/$OUT/prof.log 2>&1)
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
fi
