#!/bin/bash
# Re-verify HEAD on the GPU box: gpu parity tests, the default (C3) bench line
# and its kernel trace, then the C5 line and its kernel trace.  Each GPU step
# has its own limit; the chain stops at the first failure.
#   usage: scripts/gpu_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-check}
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py --no-cpu-baseline > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
grep -h extract_kernel $OUT/kt/kt_kernel_stats.csv
timeout -k 10 900 python bench.py --config C5 --steps 30 --warmup 10 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- python bench.py --config C5 --steps 30 --warmup 10 --no-verify > $OUT/kt5.json 2> $OUT/kt5.err || { tail -30 $OUT/kt5.err; exit 1; }
grep -h "orf6\|extract_kernel" $OUT/kt5/kt_kernel_stats.csv
