#!/bin/bash
# Kernel iteration loop for C3 (the default bench line): gpu parity tests, the
# bench line and its kernel trace.   usage: scripts/gpu_c3quick.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-c3q}
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('C3 kernel_ms %.4f frac %.4f parity %s' % (r['kernel_ms'], r['frac'], d['parity']))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py --no-cpu-baseline --no-verify > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
grep -h extract_kernel $OUT/kt/kt_kernel_stats.csv
