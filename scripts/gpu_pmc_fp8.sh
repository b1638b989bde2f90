# PMC passes: the fp8 quad GEMM loop vs hipBLASLt _scaled_mm (8192^3 e4m3)
#   bash scripts/gpu_pmc_fp8.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/pmc_fp8}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C1=SQ_BUSY_CU_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_LDS,SQ_INSTS_MFMA
C2=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS,SQ_INSTS_VALU,TCC_HIT_sum,TCC_MISS_sum
cd /tmp && for w in fp8_nt scaled_mm; do
  timeout -s KILL 120 rocprofv3 --pmc $C1 -d $R/$OUT/${w}_1 -o p --output-format csv -- python3 $R/scripts/pmc_driver.py $w 10 > $R/$OUT/${w}_1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $C2 -d $R/$OUT/${w}_2 -o p --output-format csv -- python3 $R/scripts/pmc_driver.py $w 10 > $R/$OUT/${w}_2.log 2>&1 || exit 1
done
