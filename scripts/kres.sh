#!/bin/bash
# Kernel resource usage (VGPR/AGPR/SGPR/spills/LDS/occupancy) of a generated HIP source: kres.sh file.hip
/opt/rocm/lib/llvm/bin/clang++ -x hip --offload-arch=gfx950 --offload-device-only --no-gpu-bundle-output \
  -I "$(dirname "$0")/../tilelang/include" -O3 -std=c++17 -ffp-contract=fast-honor-pragmas -w -c -o /tmp/kres.o "$1" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "remark" | sed -e 's/.*remark: //' | sort -u
