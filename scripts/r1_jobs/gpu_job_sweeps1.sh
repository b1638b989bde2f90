#!/bin/bash
# sweeps after the LDS-DMA-for-dynamic-loops fix
cd "$(dirname "$0")/.."
O=gpurun_out/sweeps1.log
: > $O
timeout -k 10 150 python scripts/gpu_sweep.py sink '{}' '{"block_M":128,"block_N":128,"threads":512}' '{"block_M":256,"block_N":128,"threads":512,"num_stages":1}' >> $O 2>&1 || exit $?
timeout -k 10 150 python scripts/gpu_sweep.py mamba '{}' '{"block_M":128,"block_N":64,"block_K":64}' '{"block_M":64,"block_N":64,"block_K":64,"threads":128}' '{"block_M":128,"block_N":64,"block_K":32,"threads":256}' >> $O 2>&1 || exit $?
timeout -k 10 200 python scripts/gpu_sweep.py fa_bwd '{}' '{"block_M":128,"block_N":64,"threads":256}' '{"block_M":128,"block_N":32,"threads":256}' '{"block_M":128,"block_N":64,"threads":512}' '{"block_M":64,"block_N":64,"threads":128}' >> $O 2>&1 || exit $?
timeout -k 10 150 python scripts/gpu_sweep.py decode '{}' '{"num_split":16}' '{"block_N":128}' '{"num_split":4,"block_N":128}' >> $O 2>&1 || exit $?
timeout -k 10 150 python scripts/gpu_sweep.py linear_attn '{}' '{"BV":128}' '{"threads":512}' >> $O 2>&1
cat $O
