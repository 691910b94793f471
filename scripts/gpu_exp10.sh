#!/bin/bash
# XCD-aware schedule and DRAM-vs-MALL read requests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp10; rm -rf $OUT; mkdir -p $OUT
MAGOT_XCD_REMAP=1 timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # name order remap
  MAGOT_XCD_REMAP=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o kt -- python scripts/prof_kernel.py --order $2 --iters 10 > $OUT/$1.log 2>&1 || exit 1
  echo "$1 order=$2 remap=$3 avg_ns=$(grep extract_kernel $OUT/$1/kt_kernel_stats.csv | cut -d, -f4)"
}
run rand_0 random 0
run rand_1 random 1
run sort_0 sorted 0
run sort_1 sorted 1
for r in 0 1; do
  MAGOT_XCD_REMAP=$r timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc$r -o pmc -- python scripts/prof_kernel.py --order random --iters 5 > $OUT/pmc$r.log 2>&1 || exit 1
done
python scripts/pmc_summary.py $OUT
