#!/bin/bash
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 200 python -u scripts/launch_overhead.py 2>&1 | grep -v amdgpu
