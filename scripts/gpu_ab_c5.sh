#!/bin/bash
# C5 A/B of two libmagot builds (scripts/lib_NAME.so), 3 alternating runs,
# then the B build's C5 line with the oracle check and the GPU tests.
#   usage: scripts/gpu_ab_c5.sh A B
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
A=$1; B=$2
scripts/ab3.sh $A $B -- --config C5 --steps 50 --warmup 10 || exit 1
MAGOT_LIB=$PWD/scripts/lib_$B.so timeout -k 10 300 python bench.py --config C5 > gpurun_out/ab3/${B}_c5_verify.json 2> gpurun_out/ab3/${B}_c5_verify.err || { tail -20 gpurun_out/ab3/${B}_c5_verify.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab3/${B}_c5_verify.json'));print(d['parity'], d['ms_per_step'], d['roofline']['frac'])"
MAGOT_LIB=$PWD/scripts/lib_$B.so timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 300 --timeout-method thread > gpurun_out/ab3/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab3/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/ab3/pytest_gpu.log
