#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp4; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 ./scripts/membench.bin || exit 1
run() {  # name outputs dbg grid
  MAGOT_GRID_BLOCKS=$4 MAGOT_DEBUG_PATHS=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o kt -- python scripts/prof_kernel.py --order sorted --outputs $2 --iters 10 > $OUT/$1.log 2>&1 || exit 1
  echo "$1 outputs=$2 dbg=$3 grid=$4 avg_ns=$(grep extract_kernel $OUT/$1/kt_kernel_stats.csv | cut -d, -f4)"
}
run full nuc+pep 0 0
run g256 nuc+pep 0 256
run g512 nuc+pep 0 512
run g1024 nuc+pep 0 1024
run g2048 nuc+pep 0 2048
run nuc nuc 0 0
run pep pep 0 0


