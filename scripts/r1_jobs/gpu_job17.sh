#!/bin/bash
cd "$(dirname "$0")/.."
ROOT=$(pwd)
export PYTHONPATH=$ROOT
O=$ROOT/gpurun_out/job17
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o smla_bwd --output-format csv -- python3 $ROOT/scripts/prof_smla_bwd.py > $O/prof.log 2>&1 || exit $?
find $O -name "*kernel_stats.csv" -exec cat {} \;
