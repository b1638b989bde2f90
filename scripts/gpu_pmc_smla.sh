# PMC passes for the sparse MLA fwd kernel at the reference shape (one counter set per run).
#   bash scripts/gpu_pmc_smla.sh [out_dir]      summaries: python scripts/pmc_summary.py <out_dir>/...
set -o pipefail
OUT=${1:-gpurun_out/pmc_smla}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
C1=SQ_BUSY_CU_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_MFMA
C2=FETCH_SIZE,TCC_HIT_sum
C3=TCC_MISS_sum,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_RD
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C1 -d $R/$OUT/p1 -o p1 --output-format csv -- python3 $R/scripts/prof_smla.py > $R/$OUT/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $C2 -d $R/$OUT/p2 -o p2 --output-format csv -- python3 $R/scripts/prof_smla.py > $R/$OUT/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $C3 -d $R/$OUT/p3 -o p3 --output-format csv -- python3 $R/scripts/prof_smla.py > $R/$OUT/p3.log 2>&1
