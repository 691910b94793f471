#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r02f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_slow.log 2>&1 || { tail -40 $OUT/pytest_slow.log; exit 1; }
tail -1 $OUT/pytest_slow.log
bash scripts/ab3.sh base vd -- --steps 300 || exit 1
bash scripts/gpu_pmc_ab.sh "MAGOT_LIB=$PWD/scripts/lib_base.so" "MAGOT_LIB=$PWD/scripts/lib_vd.so"
