#!/bin/bash
# orf6_kernel v20 (2-bit code staging, codon indices in the chunk loop):
# orf6 / C5 GPU tests (slow full-size C5 included), then C5 A/B against the
# previous kernel, 3 alternating runs.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03n; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_translate_lib.py -m gpu -k "orf6 or c5 or kat or sequence_api or edge" -x -q --timeout 600 --timeout-method thread > $OUT/pytest_orf6.log 2>&1 || { tail -40 $OUT/pytest_orf6.log; exit 1; }
tail -1 $OUT/pytest_orf6.log
bash scripts/ab_multi.sh "scripts/lib_old.so scripts/lib_new.so" --config C5 --steps 100
