#!/bin/bash
# Round 3: slow tests (full C3, full C5 six frames), C5 / C2 lines, and the
# per-GPU share of the K-rank C4 job rehearsed on this one card.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03b; mkdir -p $OUT
bash scripts/gpu_round.sh r03b slow c5 c2 || exit 1
for kr in 2:0 4:0 8:0 8:7; do
  timeout -k 10 300 python bench.py --rehearse-shard $kr --no-cpu-baseline > $OUT/rehearse_${kr/:/_}.json 2> $OUT/rehearse.err || { tail -20 $OUT/rehearse.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/rehearse_${kr/:/_}.json'));r=d['roofline'];print('$kr', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],4), d['parity'][:20])"
done
