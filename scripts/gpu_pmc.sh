# PMC passes (one counter set per rocprofv3 run, <= 8 SQ counters) for the bench FA kernel and the
# Mamba-2 chunk scan; summaries with scripts/pmc_summary.py.   bash scripts/gpu_pmc.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C=SQ_BUSY_CU_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_MFMA
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $R/$OUT/fa -o fa --output-format csv -- python3 $R/scripts/pmc_driver.py fa 10 > $R/$OUT/fa.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $C -d $R/$OUT/mamba -o mamba --output-format csv -- python3 $R/scripts/prof_mamba.py 4096 5 '{"block_M": 128, "block_N": 64, "block_K": 64, "threads": 256, "num_stages": 2, "xcd_group": true}' > $R/$OUT/mamba.log 2>&1
