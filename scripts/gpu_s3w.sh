#!/bin/bash
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 400 python -u scripts/fa_staging_ab.py 2>&1 | grep -v amdgpu
