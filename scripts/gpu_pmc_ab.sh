#!/bin/bash
# PMC passes (FETCH_SIZE; SQ_INSTS_VALU + SQ_WAVES; TCC_EA0_RDREQ) for two environments.
#   scripts/gpu_pmc_ab.sh "A_ENV" "B_ENV"
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcab; mkdir -p $OUT
i=0
for e in "$1" "$2"; do
  i=$((i+1)); j=0
  for grp in "FETCH_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    j=$((j+1)); rm -rf $OUT/v${i}_$j
    env $e timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/v${i}_$j -o pmc -- python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline > $OUT/v${i}_$j.log 2>&1 || { tail -5 $OUT/v${i}_$j.log; exit 1; }
  done
  echo "[$e]"; python scripts/pmc_summary.py $OUT | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in sorted(d.items()):
    if k.startswith('v${i}_'): print(k, v)"
done
