#!/bin/bash
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 400 python scripts/debug_c5.py C5 $OUT/debug_c5.json > $OUT/debug.log 2>&1 || { tail -20 $OUT/debug.log; exit 1; }
cut -c1-600 $OUT/debug.log
for kr in 2:0 4:0 8:0 8:7; do
  timeout -k 10 300 python bench.py --rehearse-shard $kr --no-cpu-baseline > $OUT/rehearse_${kr/:/_}.json 2> $OUT/rehearse.err || { tail -20 $OUT/rehearse.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/rehearse_${kr/:/_}.json'));r=d['roofline'];print('$kr', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],4), d['parity'][:20])"
done
