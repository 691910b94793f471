#!/bin/bash
# Kernel iteration loop for C5: gpu parity tests (orf6 first), the C5 line
# and its kernel trace.   usage: scripts/gpu_c5quick.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-c5q}
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k orf6 -x -q --timeout 120 --timeout-method thread > $OUT/pytest_orf6.log 2>&1 || { tail -40 $OUT/pytest_orf6.log; exit 1; }
tail -1 $OUT/pytest_orf6.log
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --config C5 --steps 10 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- python bench.py --config C5 --steps 10 --warmup 2 --no-verify > $OUT/kt5.json 2> $OUT/kt5.err || { tail -30 $OUT/kt5.err; exit 1; }
grep -h "orf6\|extract_kernel" $OUT/kt5/kt_kernel_stats.csv
