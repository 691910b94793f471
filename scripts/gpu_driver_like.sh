#!/bin/bash
# What the driver runs at round end, in the same order: the whole -m gpu
# suite (slow tests included), smoke(), then the default bench line and the
# driver's 20/5 configuration.   usage: scripts/gpu_driver_like.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-driver_like}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('bench', round(d['ms_per_step'],5), '%.3e'%d['value'], round(r['kernel_ms'],5), round(r['frac'],4), d['parity'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err || { tail -30 $OUT/bench_20_5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_20_5.json'));r=d['roofline'];print('bench 20/5', round(d['ms_per_step'],5), '%.3e'%d['value'], round(r['kernel_ms'],5), round(r['frac'],4), d['parity'])"
