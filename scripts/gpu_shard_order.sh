#!/bin/bash
# The C4 shares with each shard in GFF order and in genome order, alternating.
#   usage: scripts/gpu_shard_order.sh TAG [R]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; R=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $R); do
  for o in gff genome; do
    timeout -k 10 300 python scripts/c4_shares.py --rounds 3 --order $o > $OUT/c4_$o$i.json 2> $OUT/c4_$o$i.err || { tail -20 $OUT/c4_$o$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/c4_$o$i.json'));p=d['plans']
print('$o', 'full', round(min(p['full']['ms']),5), ' '.join('%d:%.5f' % (n, max(min(p['%d:%d'%(n,r)]['ms']) for r in range(n))) for n in (2,4,8)), {k: round(v['mean'],3) for k,v in d['projected_speedup'].items()})"
  done
done
