#!/bin/bash
# orf6 XCD order: gpu parity + C5 line; extract XCD-order A/B on C3.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/xcd2; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MAGOT_LIB=$PWD/scripts/lib_exx.so timeout -k 10 300 python -u -m pytest tests -m "gpu and not slow" -k "extract or gather or c3 or plan" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_exx.log 2>&1 || { tail -30 $OUT/pytest_exx.log; exit 1; }
tail -1 $OUT/pytest_exx.log
timeout -k 10 600 python bench.py --config C5 --steps 50 --warmup 20 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c5.json'));print('C5', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity'])"
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_exx.so scripts/lib_exxplain.so" --steps 200 --warmup 20
