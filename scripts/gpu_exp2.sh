#!/bin/bash
# Attribution: kernel time with parts of the work switched off (timing only).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp2; rm -rf $OUT; mkdir -p $OUT
run() {  # name outputs dbg
  MAGOT_DEBUG_PATHS=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o kt -- python scripts/prof_kernel.py --order sorted --outputs $2 --iters 10 > $OUT/$1.log 2>&1 || exit 1
  echo "$1 outputs=$2 dbg=$3 avg_ns=$(grep extract_kernel $OUT/$1/kt_kernel_stats.csv | cut -d, -f4)"
}
run full nuc+pep 0
run nuc nuc 0
run pep pep 0
run noloads nuc+pep 4
run noloads_nuc nuc 4
run prologue nuc+pep 8
run slownuc_nuc nuc 1
