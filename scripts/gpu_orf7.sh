#!/bin/bash
# orf6_kernel at 7 blocks per CU (row cap 95, 32-word chunk bitmap: 23.0 KB of
# LDS per block) against the 6-block base, C5, then the C5 line with its
# oracle check and the GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
scripts/ab3.sh base orf7 -- --config C5 --steps 50 --warmup 10 || exit 1
timeout -k 10 300 python bench.py --config C5 > gpurun_out/ab3/orf7_c5_verify.json 2> gpurun_out/ab3/orf7_c5_verify.err || { tail -20 gpurun_out/ab3/orf7_c5_verify.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab3/orf7_c5_verify.json'));print(d['parity'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 300 --timeout-method thread > gpurun_out/ab3/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab3/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/ab3/pytest_gpu.log
