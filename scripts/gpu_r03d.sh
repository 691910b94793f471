#!/bin/bash
# orf6 ballot fix: the upper-lane regression test, every orf6 test, the slow
# full-size C5 six-frame check, the C5 line (full six-frame verify).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "orf6 or c5" -x -q --timeout 500 --timeout-method thread > $OUT/pytest_orf6.log 2>&1 || { tail -30 $OUT/pytest_orf6.log; exit 1; }
tail -1 $OUT/pytest_orf6.log
bash scripts/gpu_round.sh r03d c5
