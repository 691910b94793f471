#!/bin/bash
# Round-2 closing run on HEAD: every GPU test (slow included), the default
# bench line, the driver's configuration, the kernel trace and PMC passes.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r02_final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
scripts/gpu_round.sh $TAG tests slow bench || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_cfg_20_5.json 2> $OUT/bench_driver_cfg.err || { tail -20 $OUT/bench_driver_cfg.err; exit 1; }
cat $OUT/bench_driver_cfg_20_5.json
timeout -k 10 600 python bench.py --config C5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
scripts/gpu_round.sh $TAG kt pmc
