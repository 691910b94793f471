#!/bin/bash
# C5 "slow state" vs allocation: default hipMalloc arenas vs physically
# contiguous ones (MAGOT_ARENA_CONTIGUOUS=1), alternating, 3 rounds; C3 once each.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03t; rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
  for c in 0 1; do
    MAGOT_ARENA_CONTIGUOUS=$c timeout -k 10 300 python bench.py --config C5 --no-verify --no-cpu-baseline > $OUT/c5_$c.$i.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/c5_$c.$i.json'));print('C5 contig=$c', round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))"
  done
done
for c in 0 1; do
  MAGOT_ARENA_CONTIGUOUS=$c timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline --steps 300 > $OUT/c3_$c.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c3_$c.json'));print('C3 contig=$c', round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))"
done
