#!/bin/bash
# A/B a kernel change on one box: two builds of libmagot.so, bench lines
# alternated (kernel time by HIP events), three rounds each.
#   usage: scripts/ab_bench.sh LIB_A LIB_B [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
A=$1; B=$2; shift 2
OUT=gpurun_out/ab; mkdir -p $OUT
for i in 1 2 3; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    MAGOT_LIB=$lib timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -20 $OUT/$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v', d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
