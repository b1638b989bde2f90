#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job3.log
: > $O
timeout -k 10 200 python scripts/gpu_sweep.py mamba '{}' '{"block_K":64}' '{"block_M":64,"block_K":64,"threads":128}' '{"block_M":256,"block_K":32,"threads":512}' >> $O 2>&1 || exit $?
timeout -k 10 200 python scripts/gpu_sweep.py fa_bwd '{}' '{"dq_mode":"none"}' '{"block_M":128,"block_N":32,"threads":512}' '{"block_M":256,"block_N":32,"threads":512}' >> $O 2>&1 || exit $?
cat $O
