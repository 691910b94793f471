#!/bin/bash
# One GPU's share of the 8- and 4-GPU C4 job: 2-slot vs 3-slot small tiles.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/lc2; mkdir -p $OUT
MAGOT_LIB=$PWD/scripts/lib_lc2.so timeout -k 10 300 python bench.py --rehearse-shard 8:0 --steps 300 --no-cpu-baseline > $OUT/verify_8_0.json 2> $OUT/verify.err || { tail -20 $OUT/verify.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/verify_8_0.json'));print('lc2 8:0 verified', d['ms_per_step'], d['parity'])"
for kr in 8:0 4:0; do
  bash scripts/ab_multi.sh "scripts/lib_base2.so scripts/lib_lc2.so" --rehearse-shard $kr --steps 300 > $OUT/ab_${kr/:/_}.txt 2>&1 || { cat $OUT/ab_${kr/:/_}.txt; exit 1; }
  echo "== $kr"; cat $OUT/ab_${kr/:/_}.txt
done
