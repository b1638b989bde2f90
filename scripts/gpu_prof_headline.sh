#!/bin/bash
# Headline evidence on one MI355X: bench.py, cold/warm per-kernel times, and PMC passes of the
# bench GEMM and FlashAttention kernels (each pass its own run, <= 8 SQ counters).
#   TAG=<name> (default r2)
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r2}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 python scripts/prof_bench.py both --cold > $OUT/cold_warm.log 2>&1 || { echo "cold failed"; tail -20 $OUT/cold_warm.log; exit 1; }
cat $OUT/cold_warm.log
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for k in gemm fa; do
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc_${k}_p$i -o p --output-format csv -- python3 $ROOT/scripts/prof_bench.py $k 10 > $OUT/pmc_${k}_p$i.log 2>&1 || { echo "pmc $k p$i failed"; tail -20 $OUT/pmc_${k}_p$i.log; exit 1; }
    i=$((i+1))
  done
done
cd $ROOT
for k in gemm fa; do
  python scripts/pmc_summary.py "gemm_kernel|flashattn_kernel|flashattn_pipelined_kernel" $(find $OUT/pmc_${k}_p1 $OUT/pmc_${k}_p2 -name "*counter_collection.csv") > $OUT/pmc_${k}_summary.md
  cat $OUT/pmc_${k}_summary.md
done
