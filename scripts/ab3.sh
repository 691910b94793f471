#!/bin/bash
# A/B/C of libmagot.so builds on one box, alternated, 3 rounds (HIP-event kernel
# time and ms/step of bench.py).   usage: scripts/ab3.sh NAME1 NAME2 ... -- [bench args]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
names=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done; shift
OUT=gpurun_out/ab3; mkdir -p $OUT
for i in 1 2 3; do
  for v in "${names[@]}"; do
    MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -20 $OUT/$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v', '%.4f'%d['roofline']['kernel_ms'], '%.4f'%d['ms_per_step'])"
  done
done
