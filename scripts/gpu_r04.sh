#!/bin/bash
# Round-4 GPU steps, each under its own time limit, chained: stops at the first
# failure.   usage: scripts/gpu_r04.sh TAG step...
# steps: repl (replication/pack/segment tests), benchgpu (bench multi-rank tests),
#        ab5 / ab3 (scripts/lib_base.so vs the tree's library, C5 / C3, 3 alternating runs),
#        sharded (full-size sharded C3/C5 tests), bench (C3 line), c5 (C5 line),
#        gpu (every gpu test but slow), slow (slow gpu tests)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r04}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout-method thread"
for step in "$@"; do
  case $step in
    repl) timeout -k 10 600 $PYT --timeout 300 tests/test_gpu_replication.py > $OUT/repl.log 2>&1 || { tail -60 $OUT/repl.log; exit 1; }; tail -2 $OUT/repl.log ;;
    benchgpu) timeout -k 10 900 $PYT --timeout 400 tests/test_bench_gpu.py > $OUT/benchgpu.log 2>&1 || { tail -60 $OUT/benchgpu.log; exit 1; }; tail -2 $OUT/benchgpu.log ;;
    sharded) timeout -k 10 1000 $PYT --timeout 500 tests/test_gpu_sharded.py > $OUT/sharded.log 2>&1 || { tail -60 $OUT/sharded.log; exit 1; }; tail -2 $OUT/sharded.log ;;
    bench) timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }; cat $OUT/bench.json ;;
    c5) timeout -k 10 600 python bench.py --config C5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -30 $OUT/bench_c5.err; exit 1; }; cat $OUT/bench_c5.json ;;
    gpu) timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 300 --timeout-method thread > $OUT/gpu.log 2>&1 || { tail -60 $OUT/gpu.log; exit 1; }; tail -2 $OUT/gpu.log ;;
    slow) timeout -k 10 1100 python -u -m pytest tests -m "gpu and slow" -v -x --timeout 600 --timeout-method thread > $OUT/slow.log 2>&1 || { tail -60 $OUT/slow.log; exit 1; }; tail -3 $OUT/slow.log ;;
    ab5) bash scripts/ab_bench.sh scripts/lib_base.so magot_amd/libmagot.so --config C5 --steps 100 --no-box-state > $OUT/ab5.log 2>&1 || { tail -20 $OUT/ab5.log; exit 1; }; cp -r gpurun_out/ab $OUT/ab5; cat $OUT/ab5.log ;;
    ab3) bash scripts/ab_bench.sh scripts/lib_base.so magot_amd/libmagot.so --steps 300 --no-box-state > $OUT/ab3.log 2>&1 || { tail -20 $OUT/ab3.log; exit 1; }; cp -r gpurun_out/ab $OUT/ab3; cat $OUT/ab3.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
