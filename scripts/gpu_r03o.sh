#!/bin/bash
# orf6_kernel v20: occupancy (blocks per CU: uncapped / 7 / 6), 3 alternating
# runs, then its PMC passes.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03o; rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
  for cap in 0 7 6; do
    MAGOT_ORF6_BLOCKS_PER_CU=$cap timeout -k 10 300 python bench.py --config C5 --steps 100 --no-verify --no-cpu-baseline > $OUT/cap$cap.$i.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/cap$cap.$i.json'));print('cap$cap', round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))"
  done
done
TAG=r03o_pmc bash scripts/gpu_pmc_c5.sh
