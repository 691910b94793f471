#!/bin/bash
# Library variants of one kernel: HBM traffic per launch (FETCH_SIZE and
# WRITE_SIZE passes, separate runs) and time (alternating, 3 rounds).
#   scripts/ab_pmc_libs.sh OUTDIR KERNEL "lib_a.so lib_b.so ..." [bench args]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=$1; KERNEL=$2; LIBS=$3; shift 3
mkdir -p $OUT
for lib in $LIBS; do
  n=$(basename $lib .so)
  for grp in FETCH_SIZE WRITE_SIZE; do
    rm -rf $OUT/$n/$grp
    MAGOT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/$n/$grp -o pmc -- python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline --no-box-state "$@" > $OUT/$n.$grp.log 2>&1 || { echo "pmc $n $grp failed"; tail -3 $OUT/$n.$grp.log; exit 1; }
  done
  python3 scripts/pmc_json.py $OUT/$n X $KERNEL > $OUT/$n.pmc.json 2>/dev/null
  python3 -c "import json;d=json.load(open('$OUT/$n.pmc.json'));print('$n reads %.3f GB writes %.3f GB' % (d['hbm_read_bytes_per_launch']/1e9, d['write_size_bytes']/1e9))"
done
for rep in 1 2 3; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    MAGOT_LIB=$lib timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline --no-box-state "$@" > $OUT/$n.$rep.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$n.$rep.json'));print('$n', round(d['roofline']['kernel_ms'],5))"
  done
done
