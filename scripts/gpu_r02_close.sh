#!/bin/bash
# Round-2 closing check on HEAD: GPU tests (incl. slow), smoke(), the C3 line
# (defaults and the driver's 20/5), C5 and C2 lines, kernel trace of the C3 line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r02_close; mkdir -p $OUT
bash scripts/gpu_round.sh r02_close tests slow bench kt || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_cfg_20_5.json 2> $OUT/driver.err || { tail -20 $OUT/driver.err; exit 1; }
timeout -k 10 400 python bench.py --config C5 > $OUT/bench_c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
timeout -k 10 300 python bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
for f in bench bench_driver_cfg_20_5 bench_c5 bench_c2 kt; do
  python3 -c "import json;d=json.load(open('$OUT/$f.json'));r=d['roofline'];print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['kernel_ms'],4), round(r['frac'],4), d['parity'][:24])"
done
