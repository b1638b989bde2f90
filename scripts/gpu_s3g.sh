#!/bin/bash
set -u
mkdir -p gpurun_out/s3g
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
R=$GRAFT_REPO_ROOT
cd $R/examples/deepseek_nsa && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s3g/nsa -o nsa --output-format csv -- python3 example_nsa_bwd.py > $R/gpurun_out/s3g/nsa.log 2>&1 || { tail -20 $R/gpurun_out/s3g/nsa.log; exit 1; }
cd $R; grep TFLOPS gpurun_out/s3g/nsa.log
python3 - "$(find gpurun_out/s3g/nsa -name '*kernel_stats.csv')" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"  {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
