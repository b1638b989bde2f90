#!/bin/bash
# Round-end rehearsal on the GPU box (gpurun): the GPU test tier, smoke(), bench.py and a
# rocprofv3 kernel-stats profile of the bench, each step under its own time limit; stops at the
# first failing step.   bash scripts/gpu_suite.sh [out_dir]
set -u
OUT=${1:-gpurun_out/suite}
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -6
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep metric $OUT/bench.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o bench --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$OUT/prof.log 2>&1; echo "rocprof rc=$?"
