#!/bin/bash
# PMC passes of the MX GEMM kernels (fp8 x fp8 and fp4 x fp4), one counter group per run.
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/mx_pmc
mkdir -p $OUT
timeout -k 10 300 python scripts/prof_mx.py e4m3 e4m3 2 > $OUT/warm.log 2>&1 || { tail -5 $OUT/warm.log; exit 1; }
timeout -k 10 300 python scripts/prof_mx.py pt8 pt8 2 > $OUT/warm2.log 2>&1 || { tail -5 $OUT/warm2.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for f in e4m3 pt8; do
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/${f}_p$i -o p --output-format csv -- python3 $ROOT/scripts/prof_mx.py $f $f 5 > $OUT/${f}_p$i.log 2>&1 || { echo "pmc $f p$i failed"; tail -5 $OUT/${f}_p$i.log; exit 1; }
    i=$((i+1))
  done
done
cd $ROOT
for f in e4m3 pt8; do
  python scripts/pmc_summary.py "^(mx_matmul|gemm_fp8)_kernel" $(find $OUT/${f}_p1 $OUT/${f}_p2 -name "*counter_collection.csv") > $OUT/summary_$f.md
  cat $OUT/summary_$f.md
done
