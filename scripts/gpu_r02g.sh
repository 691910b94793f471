#!/bin/bash
# Round 2: C5 and C2 bench lines and the C5 kernel trace on the current kernels.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r02g; mkdir -p $OUT
timeout -k 10 600 python bench.py --config C5 --steps 30 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 300 python bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
rm -rf $OUT/kt5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- python bench.py --config C5 --steps 30 --no-cpu-baseline > $OUT/kt_c5.json 2> $OUT/kt_c5.err || { tail -30 $OUT/kt_c5.err; exit 1; }
grep -h "orf6_kernel\|extract_kernel" $OUT/kt5/kt_kernel_stats.csv
