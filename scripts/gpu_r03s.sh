#!/bin/bash
# C5 slow state: three C5 bench processes under a GRBM_GUI_ACTIVE pass
# (engine clock per launch), then two plain ones.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03s; rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $OUT/clk$i -o pmc -- python bench.py --config C5 --no-verify --no-cpu-baseline > $OUT/clk$i.json 2> $OUT/clk$i.err || { tail -5 $OUT/clk$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/clk$i.json'));print('clk$i bench', round(d['ms_per_step'],4))"
  python3 scripts/clock_per_launch.py $OUT/clk$i orf6_kernel
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --config C5 --no-verify --no-cpu-baseline > $OUT/c5.$i.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c5.$i.json'));print('plain', round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))"
done
