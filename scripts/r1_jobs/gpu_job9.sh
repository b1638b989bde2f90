#!/bin/bash
cd "$(dirname "$0")/.."
ROOT=$(pwd)
export PYTHONPATH=$ROOT
O=$ROOT/gpurun_out/job9
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM \
  -d $O/p2 -o p2 --output-format csv -- python3 $ROOT/scripts/prof_smla.py > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_RDREQ_sum \
  -d $O/p3 -o p3 --output-format csv -- python3 $ROOT/scripts/prof_smla.py > $O/p3.log 2>&1 || exit $?
find $O -name "*counter_collection.csv" | head
