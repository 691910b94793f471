#!/bin/bash
# Round-3 state: all GPU tests (slow included), C3 / driver / C5 / C2 lines,
# kernel traces of C3, C5, C2, smoke().
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/gpu_round.sh r03q tests slow bench driver c5 c2 kt kt5 kt2 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q/smoke.log 2>&1 || { tail -20 gpurun_out/r03q/smoke.log; exit 1; }
tail -1 gpurun_out/r03q/smoke.log
for f in bench bench_driver_cfg_20_5 bench_c5 bench_c2; do
  python3 -c "import json;d=json.load(open('gpurun_out/r03q/$f.json'));r=d['roofline'];print('$f', round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['kernel_ms'],4), round(r['frac'],4), d['parity'][:24])"
done
