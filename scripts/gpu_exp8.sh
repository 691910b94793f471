#!/bin/bash
# Sparse-read request size calibration (membench2) with TCC request counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp8; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 ./scripts/membench2.bin | tee $OUT/timing.txt || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $OUT/p1 -o pmc -- ./scripts/membench2.bin > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p2 -o pmc -- ./scripts/membench2.bin > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ('p1', 'p2'):
    for f in glob.glob('gpurun_out/exp8/%s/**/*counter_collection.csv' % p, recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0][-12:]
            agg[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
        for (k, c), v in sorted(agg.items()):
            print(p, k, c, ['%.0f' % x for x in v[:3]])
PY
