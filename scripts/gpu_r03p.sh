#!/bin/bash
# orf6 chunk pairs (q and q+64 per lane) vs single chunks, both at 7 blocks
# per CU; orf6 GPU tests first.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03p; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "orf6 or c5 or sequence_api" -x -q --timeout 600 --timeout-method thread > $OUT/pytest_orf6.log 2>&1 || { tail -40 $OUT/pytest_orf6.log; exit 1; }
tail -1 $OUT/pytest_orf6.log
export MAGOT_ORF6_BLOCKS_PER_CU=7
bash scripts/ab_multi.sh "scripts/lib_v20.so scripts/lib_pair.so" --config C5 --steps 100
