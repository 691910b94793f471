#!/bin/bash
# GPU tests, then the C5 line (gather + six-frame translation) and its kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/c5; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 1000 python bench.py --config C5 --steps 10 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py --config C5 --steps 10 --warmup 2 --no-verify > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
grep -h "orf6\|extract_kernel" $OUT/kt/kt_kernel_stats.csv
