#!/bin/bash
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 500 python -u scripts/sweep_gemm.py 2>&1 | grep -v amdgpu
