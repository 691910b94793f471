#!/bin/bash
# C2 tile size A/B (3 vs 5 chunk slots), then two C5 lines (box state).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03r; rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
  for lc in 5 3; do
    MAGOT_EXTRACT_LANE_CHUNKS=$lc timeout -k 10 300 python bench.py --config C2 --steps 300 --no-verify --no-cpu-baseline > $OUT/c2_lc$lc.$i.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/c2_lc$lc.$i.json'));print('C2 lc$lc', round(d['roofline']['kernel_ms'],5), round(d['ms_per_step'],5))"
  done
done
for lc in 5 3; do
  MAGOT_EXTRACT_LANE_CHUNKS=$lc timeout -k 10 300 python bench.py --rehearse-shard 2:0 --steps 300 --no-verify --no-cpu-baseline > $OUT/r20_lc$lc.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/r20_lc$lc.json'));print('2:0 lc$lc', round(d['roofline']['kernel_ms'],5), round(d['ms_per_step'],5))"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --config C5 --no-verify --no-cpu-baseline > $OUT/c5.$i.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c5.$i.json'));print('C5', round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))"
done
