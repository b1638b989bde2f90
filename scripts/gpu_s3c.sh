#!/bin/bash
# session 3: persistent/staged FA after diagonal-only masking + PMC passes on the bench GEMM and FA
set -u
mkdir -p gpurun_out/pmc_s3
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u scripts/fa_persistent_ab.py > gpurun_out/fa_persistent_ab2.log 2>&1 || { grep -v amdgpu.ids gpurun_out/fa_persistent_ab2.log | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_persistent_ab2.log | grep TF
for w in gemm fa fa32; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc_s3/$w -o p1 -- python3 $R/scripts/pmc_driver.py $w > $R/gpurun_out/pmc_s3/$w.log 2>&1 || { tail -20 $R/gpurun_out/pmc_s3/$w.log; exit 1; }
  cd $R
done
for w in gemm fa fa32; do python scripts/pmc_summary.py "gemm_kernel|flashattn" $(find gpurun_out/pmc_s3/$w -name "*counter_collection.csv") > gpurun_out/pmc_s3/$w.md; tail -8 gpurun_out/pmc_s3/$w.md; done
