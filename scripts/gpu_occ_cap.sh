#!/bin/bash
# The extract_kernel occupancy cap (dynamic LDS, 6 blocks per CU) against no
# cap (7), then the GPU tests with the cap.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
scripts/ab_env.sh "MAGOT_EXTRACT_BLOCKS_PER_CU=6" "MAGOT_EXTRACT_BLOCKS_PER_CU=0" || exit 1
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 300 --timeout-method thread > gpurun_out/abenv/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/abenv/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/abenv/pytest_gpu.log
