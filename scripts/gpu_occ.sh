#!/bin/bash
# Occupancy / tile-size A/B on one box: base (5 chunk slots per lane, 7
# waves/SIMD), occ6 (same kernel, LDS padded to 6 blocks per CU), lc6 (6 chunk
# slots per lane: 6096-byte tiles, 76 VGPRs, 6 waves/SIMD); then lc6 once with
# the oracle byte check.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
scripts/ab3.sh base occ6 lc6 -- || exit 1
MAGOT_LIB=$PWD/scripts/lib_lc6.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab3/lc6_verify.json 2> gpurun_out/ab3/lc6_verify.err || { tail -20 gpurun_out/ab3/lc6_verify.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab3/lc6_verify.json'));print(d['parity'], d['ms_per_step'])"
