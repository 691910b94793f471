#!/bin/bash
# Tile-size choice: every GPU test under both tile sizes (slow included), the
# C3 line, and the 8:0 / 4:0 / 2:0 shard rehearsals (auto choice).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03l; mkdir -p $OUT
bash scripts/gpu_round.sh r03l tests slow bench || exit 1
for kr in 2:0 4:0 8:0 8:7; do
  timeout -k 10 300 python bench.py --rehearse-shard $kr --steps 300 --no-cpu-baseline > $OUT/rehearse_${kr/:/_}.json 2> $OUT/rehearse.err || { tail -20 $OUT/rehearse.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/rehearse_${kr/:/_}.json'));r=d['roofline'];print('$kr', round(d['ms_per_step'],5), round(r['kernel_ms'],5), round(r['frac'],4), d['parity'][:20])"
done
