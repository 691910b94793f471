#!/bin/bash
# A/B/C... kernel variants on one box: bench lines alternated, three rounds.
#   usage: scripts/ab_multi.sh "LIB1 LIB2 ..." [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
LIBS=$1; shift
OUT=gpurun_out/abm; rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    MAGOT_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline "$@" > $OUT/$n.$i.json 2> $OUT/$n.$i.err || { tail -20 $OUT/$n.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$n.$i.json'));print('$n', d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
