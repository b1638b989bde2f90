#!/bin/bash
# PMC passes (one counter set per run, each under its own time limit) for the round-6 versions of
# the secondary kernels: FA bwd (autograd path: dK/dV + dQ kernels), sparse MLA fwd, Mamba-2 chunk
# scan, and the bench's FA forward.   bash scripts/gpu_pmc_r6.sh [out_dir]
# Summaries: python scripts/pmc_summary.py <regex> <out_dir>/<name>_c*/*counter_collection.csv
set -o pipefail
OUT=${1:-gpurun_out/pmc_r6}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
C1=SQ_BUSY_CU_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_MFMA
C3=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_LDS,SQ_WAVE_CYCLES
cd /tmp
run() {  # name counters cmd...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $R/$OUT/$name -o $name --output-format csv -- "$@" > $R/$OUT/$name.log 2>&1
}
run fa_bwd_c1 $C1 python3 $R/scripts/prof_attn.py fa_bwd 10 && \
run fa_bwd_c3 $C3 python3 $R/scripts/prof_attn.py fa_bwd 10 && \
run smla_c1 $C1 python3 $R/scripts/prof_smla.py && \
run smla_c3 $C3 python3 $R/scripts/prof_smla.py && \
run mamba_c1 $C1 python3 $R/scripts/prof_attn.py mamba 10 && \
run mamba_c3 $C3 python3 $R/scripts/prof_attn.py mamba 10 && \
run fa_c1 $C1 python3 $R/scripts/pmc_driver.py fa 10 && \
run fa_c3 $C3 python3 $R/scripts/pmc_driver.py fa 10
rc=$?
echo "rc=$rc"
exit $rc
