#!/bin/bash
# Build a wheel of the framework (reference: maint/scripts/local_distribution.sh).
# The wheel carries the Python package, the device headers (tilelang/include/tl) and the two
# native extensions built for this interpreter and ROCm; gfx950 kernels are compiled at run time
# (JIT, cached under $TILELANG_CACHE_DIR), so the wheel has no GPU build step.
set -euo pipefail
cd "$(dirname "$0")/../.."
rm -rf build dist
python3 setup.py build_ext --inplace
python3 -m pip wheel . --no-deps --no-build-isolation -w dist
ls -l dist
