#!/bin/bash
# orf6_kernel (C5) occupancy: 6 blocks per CU (LDS-limited, no cap) against
# caps of 5 and 4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/occ_c5; mkdir -p $OUT
for i in 1 2 3; do
  for b in 0 5 4; do
    MAGOT_ORF6_BLOCKS_PER_CU=$b timeout -k 10 300 python bench.py --config C5 --steps 50 --warmup 10 --no-verify --no-cpu-baseline > $OUT/b$b-$i.json 2> $OUT/b$b-$i.err || { tail -20 $OUT/b$b-$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b$b-$i.json'));print('cap $b', '%.4f'%d['roofline']['kernel_ms'], '%.4f'%d['ms_per_step'])"
  done
done
