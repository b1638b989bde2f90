#!/bin/bash
set -u
mkdir -p gpurun_out/s3h
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_backward_kernels.py -v -m gpu -k nsa --timeout 120 --timeout-method thread > gpurun_out/s3h/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s3h/t.log | tail -3
[ $rc -eq 0 ] || { tail -30 gpurun_out/s3h/t.log; exit 1; }
cd $R/examples/deepseek_nsa && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s3h/nsa -o nsa --output-format csv -- python3 example_nsa_bwd.py > $R/gpurun_out/s3h/nsa.log 2>&1 || { tail -20 $R/gpurun_out/s3h/nsa.log; exit 1; }
cd $R; grep TFLOPS gpurun_out/s3h/nsa.log
python3 - "$(find gpurun_out/s3h/nsa -name '*kernel_stats.csv')" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"  {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
cd $R/examples/deepseek_nsa && timeout -k 10 240 python3 example_nsa_bwd.py 2>&1 | grep TFLOPS
