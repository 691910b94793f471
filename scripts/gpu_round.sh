#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile.  Each GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = slow ]; then
  timeout -k 10 600 python -m pytest tests -m "gpu and slow" -x -q > gpurun_out/pytest_gpu_slow.log 2>&1 || { tail -50 gpurun_out/pytest_gpu_slow.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_slow.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 3 --no-verify --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name '*stats*' | head
fi
