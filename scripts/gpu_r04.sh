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
    probe5) timeout -k 10 600 python scripts/c5_state_probe.py > $OUT/c5_state.json 2> $OUT/c5_state.err || { tail -20 $OUT/c5_state.err; exit 1; }; cat $OUT/c5_state.err | grep '^{' ;;
    gloo2c5) MAGOT_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --config C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo2_c5.json 2> $OUT/gloo2_c5.err || { tail -30 $OUT/gloo2_c5.err; exit 1; }; grep '^{' $OUT/bench_gloo2_c5.json | cut -c1-600 ;;
    gloo8c5) MAGOT_DIST_BACKEND=gloo timeout -k 10 1000 python bench.py --gpus 8 --config C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo8_c5.json 2> $OUT/gloo8_c5.err || { tail -30 $OUT/gloo8_c5.err; exit 1; }; grep '^{' $OUT/bench_gloo8_c5.json | cut -c1-600 ;;
    gloo8c3) MAGOT_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 8 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo8_c3.json 2> $OUT/gloo8_c3.err || { tail -30 $OUT/gloo8_c3.err; exit 1; }; grep '^{' $OUT/bench_gloo8_c3.json | cut -c1-600 ;;
    packtime) MAGOT_GENOME_TIMING=1 timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $OUT/bench_packtime.json 2> $OUT/packtime.err || { tail -30 $OUT/packtime.err; exit 1; }; grep '^\[genome\]' $OUT/packtime.err ;;
    kt3) rm -rf $OUT/kt3; timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt3 -o kt -- python bench.py --no-box-state > $OUT/kt3.json 2> $OUT/kt3.err || { tail -30 $OUT/kt3.err; exit 1; }; python scripts/rocprof_summary.py --timed C3=$OUT/kt3/kt_kernel_trace.csv,$OUT/kt3.json | head -30 ;;
    kt5) rm -rf $OUT/kt5; timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- python bench.py --config C5 --no-cpu-baseline --no-box-state > $OUT/kt5.json 2> $OUT/kt5.err || { tail -30 $OUT/kt5.err; exit 1; }; python scripts/rocprof_summary.py --timed C5=$OUT/kt5/kt_kernel_trace.csv,$OUT/kt5.json | head -30 ;;
    state5)
      # C5 processes back to back: plain lines (box_state probes) and lines under
      # UTCL1 translation counters (+ kernel trace), to tell the fast and the slow
      # state apart by address translation
      mkdir -p $OUT/state
      for i in 1 2 3 4; do
        timeout -k 10 300 python bench.py --config C5 --steps 50 --warmup 5 --no-verify --no-cpu-baseline > $OUT/state/plain$i.json 2> $OUT/state/plain$i.err || { tail -20 $OUT/state/plain$i.err; exit 1; }
        python3 -c "import json;d=json.load(open('$OUT/state/plain$i.json'));b=d['box_state'];print('plain$i', round(d['roofline']['kernel_ms'],4), b['probe_before'], b['probe_after'])"
        rm -rf $OUT/state/pmc$i
        timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum --kernel-trace --output-format csv -d $OUT/state/pmc$i -o pmc -- python bench.py --config C5 --steps 30 --warmup 5 --no-verify --no-cpu-baseline --no-box-state > $OUT/state/pmc$i.json 2> $OUT/state/pmc$i.err || { tail -20 $OUT/state/pmc$i.err; exit 1; }
        python3 -c "import json;d=json.load(open('$OUT/state/pmc$i.json'));print('pmc$i', round(d['roofline']['kernel_ms'],4))"
      done ;;
    probeab)
      # does the memory probe before the six-frame plan decide C5's state?
      mkdir -p $OUT/probeab
      for i in 1 2 3; do
        for v in noprobe probe; do
          flag=""; [ $v = noprobe ] && flag="--no-probe"
          timeout -k 10 300 python scripts/c5_state_probe.py $flag --rounds 1 --spacers 0,0 > $OUT/probeab/$v$i.json 2> $OUT/probeab/$v$i.err || { tail -20 $OUT/probeab/$v$i.err; exit 1; }
          echo "$v$i $(grep '^{' $OUT/probeab/$v$i.err | tr '\n' ' ' | cut -c1-300)"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
