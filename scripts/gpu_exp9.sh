#!/bin/bash
# Tile launch order experiment: identity vs genome-sorted schedule.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp9; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name order env
  MAGOT_TILE_ORDER=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o kt -- python scripts/prof_kernel.py --order $2 --iters 10 > $OUT/$1.log 2>&1 || exit 1
  echo "$1 order=$2 sched=$3 avg_ns=$(grep extract_kernel $OUT/$1/kt_kernel_stats.csv | cut -d, -f4)"
}
run rand_id random identity
run rand_gen random genome
run sort_id sorted identity
run sort_gen sorted genome
