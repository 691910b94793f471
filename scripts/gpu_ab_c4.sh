#!/bin/bash
# The C4 shares (scripts/c4_shares.py) of the product library and a variant,
# alternating: R runs each.   usage: scripts/gpu_ab_c4.sh TAG VARIANT_LIB [R]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; VAR=$2; R=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $R); do
  for v in base var; do
    lib=magot_amd/libmagot.so; [ $v = var ] && lib=$VAR
    MAGOT_LIB=$lib timeout -k 10 300 python scripts/c4_shares.py --rounds 3 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err || { tail -20 $OUT/c4_$v$i.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/c4_$v$i.json'));p=d['plans']
print('$v', 'full', round(min(p['full']['ms']),5), ' '.join('%d:%.5f' % (n, max(min(p['%d:%d'%(n,r)]['ms']) for r in range(n))) for n in (2,4,8)))"
  done
done
