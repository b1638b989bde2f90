set -o pipefail
timeout -k 10 120 ./csrc/probes/mfma_fp6_probe > gpurun_out/fp6_probe.log 2>&1 && \
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mpmc
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/mpmc/p1 -o p -- python3 $R/scripts/prof_mamba.py 4096 5 > $R/gpurun_out/mpmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/mpmc/p2 -o p -- python3 $R/scripts/prof_mamba.py 4096 5 > $R/gpurun_out/mpmc/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $R/gpurun_out/mpmc/p3 -o p -- python3 $R/scripts/prof_mamba.py 4096 5 > $R/gpurun_out/mpmc/p3.log 2>&1 && \
cd $R && python scripts/pmc_summary.py "main_kernel|chunk" $(find gpurun_out/mpmc/p1 gpurun_out/mpmc/p2 gpurun_out/mpmc/p3 -name "*counter_collection.csv") > gpurun_out/mpmc/mamba.md && \
cd $R && timeout -k 10 600 python -u benchmarks/matmul_fp8/benchmark_matmul.py --out gpurun_out/benchmarks --rows 256,512,1024,4096 > gpurun_out/benchmarks/matmul_fp8_b.log 2>&1 && \
timeout -k 10 600 python -u benchmarks/mamba2/benchmark_mamba_chunk_scan.py --out gpurun_out/benchmarks --rows 1024,4096,16384 > gpurun_out/benchmarks/mamba2_b.log 2>&1
