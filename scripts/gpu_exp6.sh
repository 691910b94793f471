#!/bin/bash
# Parity tests, then per-kernel timing for sorted/random orders and output splits.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp6; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() {  # name order outputs
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o kt -- python scripts/prof_kernel.py --order $2 --outputs $3 --iters 10 > $OUT/$1.log 2>&1 || exit 1
  echo "$1 order=$2 outputs=$3 avg_ns=$(grep extract_kernel $OUT/$1/kt_kernel_stats.csv | cut -d, -f4)"
}
run sorted sorted nuc+pep
run random random nuc+pep
run nuc random nuc
run pep random pep
