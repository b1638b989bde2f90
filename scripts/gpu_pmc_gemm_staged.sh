#!/bin/bash
# MHA-sink GPU test + one PMC pass on the bench GEMM (staged epilogue). Each step time-limited.
set -o pipefail
mkdir -p gpurun_out/pmc_gemm
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_gpu_examples_misc.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mha_sink" > gpurun_out/t4.log 2>&1 || { tail -20 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
timeout -k 10 300 python examples/attention_sink/example_mha_sink_fwd_bhsd.py 2>&1 | grep -v amdgpu
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm -o p1 -- python3 $GRAFT_REPO_ROOT/scripts/gemm_epi_ab.py > $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm/run.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm/run.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/pmc_gemm -name "*counter_collection.csv"
