#!/bin/bash
# Record order and L2 reuse: bench line and PMC traffic for --order sorted
# (records in genome order) against the default random order, one box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/sorted_pmc; mkdir -p $OUT
for o in random sorted; do
  timeout -k 10 300 python bench.py --order $o --no-cpu-baseline > $OUT/bench_$o.json 2> $OUT/bench_$o.err || { tail -20 $OUT/bench_$o.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$o.json'));print('$o', d['ms_per_step'], d['roofline']['kernel_ms'])"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1)); rm -rf $OUT/${o}_pmc$i
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/${o}_pmc$i -o pmc -- python bench.py --order $o --steps 5 --warmup 1 --no-verify --no-cpu-baseline > $OUT/${o}_pmc$i.log 2>&1 || { echo "pmc $o $i failed"; tail -3 $OUT/${o}_pmc$i.log; exit 1; }
  done
done
