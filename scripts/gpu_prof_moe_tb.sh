#!/bin/bash
# PMC passes (<= 8 SQ counters each, own run) of the MoE layer: tail-balanced expert GEMMs,
# fused router, align, combine.  Also a kernel-trace stats run.
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/moe_tb
mkdir -p $OUT
export PYTHONPATH=$ROOT:${PYTHONPATH:-}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o s -- python3 $ROOT/scripts/prof_moe.py 10 > $OUT/stats.log 2>&1 || { echo "stats failed"; tail -20 $OUT/stats.log; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc_p$i -o p --output-format csv -- python3 $ROOT/scripts/prof_moe.py 5 > $OUT/pmc_p$i.log 2>&1 || { echo "pmc p$i failed"; tail -20 $OUT/pmc_p$i.log; exit 1; }
  i=$((i+1))
done
cd $ROOT
python scripts/pmc_summary.py "moe_" $(find $OUT/pmc_p1 $OUT/pmc_p2 -name "*counter_collection.csv") > $OUT/pmc_summary.md
cat $OUT/pmc_summary.md
find $OUT/stats -name "*kernel_stats.csv" -exec cut -c1-120 {} \; | head -10
