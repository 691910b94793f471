#!/bin/bash
# WRITE_SIZE (one PMC pass each) of extract_kernel for A/B library variants.
#   usage: scripts/ab_write_size.sh "LIB1 LIB2 ..."
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/abw; rm -rf $OUT; mkdir -p $OUT
for lib in $1; do
  n=$(basename $lib .so)
  MAGOT_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$n -o pmc -- python bench.py --steps 5 --warmup 1 --no-verify --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; exit 1; }
  python3 - $n <<'PY'
import csv, glob, os, sys
KERNEL = os.environ.get('KERNEL', 'extract_kernel')
n = sys.argv[1]
v = [float(r['Counter_Value']) for f in glob.glob('gpurun_out/abw/%s/**/*counter_collection.csv' % n, recursive=True)
     for r in csv.DictReader(open(f)) if KERNEL in r['Kernel_Name']]
print(n, KERNEL, 'WRITE_SIZE GB per launch %.4f' % (sum(v) / len(v) * 1024 / 1e9))
PY
done
