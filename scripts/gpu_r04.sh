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
    rehall)
      # every rank's share of the 2/4/8-GPU C3 job, one at a time on this GPU
      mkdir -p $OUT/rehearse
      for kr in 2:0 2:1 4:0 4:1 4:2 4:3 8:0 8:1 8:2 8:3 8:4 8:5 8:6 8:7; do
        timeout -k 10 300 python bench.py --rehearse-shard $kr --steps 300 --no-cpu-baseline --no-verify --no-box-state > $OUT/rehearse/r_${kr/:/_}.json 2> $OUT/rehearse/r.err || { tail -20 $OUT/rehearse/r.err; exit 1; }
        python3 -c "import json;d=json.load(open('$OUT/rehearse/r_${kr/:/_}.json'));r=d['roofline'];print('$kr', round(d['ms_per_step'],5), round(r['kernel_ms'],5), d['config']['cds_bases_rank0'], d['config']['exons_rank0'])"
      done ;;
    half)
      # why is half of C3 more than half the time?  tile sizes / caps on the 2:0 share
      mkdir -p $OUT/half
      for rep in 1 2; do
        for v in full:5 2_0:5 2_0:3 2_0:4 full:3 2_0:5:bpc5 2_0:5:bpc7; do
          IFS=: read what lc extra <<< "$v"
          args="--steps 300 --no-cpu-baseline --no-verify --no-box-state"
          [ $what = 2_0 ] && args="$args --rehearse-shard 2:0"
          envs="MAGOT_EXTRACT_LANE_CHUNKS=$lc"
          [ "$extra" = bpc5 ] && envs="$envs MAGOT_EXTRACT_BLOCKS_PER_CU=5"
          [ "$extra" = bpc7 ] && envs="$envs MAGOT_EXTRACT_BLOCKS_PER_CU=7"
          env $envs timeout -k 10 300 python bench.py $args > $OUT/half/$v.$rep.json 2> $OUT/half/err || { tail -20 $OUT/half/err; exit 1; }
          python3 -c "import json;d=json.load(open('$OUT/half/$v.$rep.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],5), round(r['kernel_ms'],5))"
        done
      done ;;
    halfpmc)
      mkdir -p $OUT/halfpmc
      for what in full 2_0; do
        args="--steps 20 --warmup 2 --settle-ms 0 --no-cpu-baseline --no-verify --no-box-state"
        [ $what = 2_0 ] && args="$args --rehearse-shard 2:0"
        i=0
        for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES"; do
          i=$((i+1))
          rm -rf $OUT/halfpmc/$what.$i
          timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/halfpmc/$what.$i -o pmc -- python bench.py $args > $OUT/halfpmc/$what.$i.log 2>&1 || { echo "pmc $what $i failed"; tail -5 $OUT/halfpmc/$what.$i.log; exit 1; }
        done
      done
      python3 scripts/pmc_summary.py $OUT/halfpmc 2>/dev/null | head -5; echo halfpmc done ;;
    abreh)
      # AB_B=scripts/lib_X.so: base vs variant on the full C3 job and one GPU's
      # share of the 2/4/8-GPU job, alternating, two rounds
      mkdir -p $OUT/abreh
      for rep in 1 2; do
        for what in full 2:0 4:0 8:0; do
          for v in A B; do
            lib=scripts/lib_base.so; [ $v = B ] && lib=$AB_B
            args="--steps 300 --no-cpu-baseline --no-verify --no-box-state"
            [ $what != full ] && args="$args --rehearse-shard $what"
            MAGOT_LIB=$lib timeout -k 10 300 python bench.py $args > $OUT/abreh/$v.${what/:/_}.$rep.json 2> $OUT/abreh/err || { tail -20 $OUT/abreh/err; exit 1; }
            python3 -c "import json;d=json.load(open('$OUT/abreh/$v.${what/:/_}.$rep.json'));r=d['roofline'];print('$v $what', round(d['ms_per_step'],5), round(r['kernel_ms'],5))"
          done
        done
      done ;;
    state2)
      # write-path probe, C5 line, C5 traffic replay, probe again: does C5's
      # slow state go with a slow tiled write stream on the same box?
      mkdir -p $OUT/state2
      /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 scripts/membench5.hip -o /tmp/membench5.bin || exit 1
      /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 scripts/solbench.hip -o /tmp/solbench.bin || exit 1
      MB5_PROBE=1 timeout -k 10 120 /tmp/membench5.bin > $OUT/state2/probe1.txt 2>&1 || exit 1
      timeout -k 10 300 python bench.py --config C5 --steps 50 --warmup 5 --no-verify --no-cpu-baseline > $OUT/state2/c5.json 2> $OUT/state2/c5.err || { tail -20 $OUT/state2/c5.err; exit 1; }
      timeout -k 10 300 /tmp/solbench.bin c5 > $OUT/state2/solbench_c5.txt 2>&1 || exit 1
      MB5_PROBE=1 timeout -k 10 120 /tmp/membench5.bin > $OUT/state2/probe2.txt 2>&1 || exit 1
      timeout -k 10 300 python bench.py --steps 100 --no-verify --no-cpu-baseline > $OUT/state2/c3.json 2> $OUT/state2/c3.err || { tail -20 $OUT/state2/c3.err; exit 1; }
      cat $OUT/state2/probe1.txt; python3 -c "import json;d=json.load(open('$OUT/state2/c5.json'));print('C5', round(d['roofline']['kernel_ms'],4), d['box_state']['probe_before'])"
      grep "scattered, buffer 1\|sequential runs " $OUT/state2/solbench_c5.txt | head -4; cat $OUT/state2/probe2.txt
      python3 -c "import json;d=json.load(open('$OUT/state2/c3.json'));print('C3', round(d['roofline']['kernel_ms'],5))" ;;
    orf6check) timeout -k 10 900 $PYT --timeout 400 tests/test_gpu_parity.py -k "orf6 or c5_full" tests/test_gpu_sharded.py::test_c5_shards_reassembled_six_frames_vs_c_oracle > $OUT/orf6check.log 2>&1 || { tail -40 $OUT/orf6check.log; exit 1; }; tail -2 $OUT/orf6check.log ;;
    abn)
      # ABN_LIBS="a.so b.so ..." ABN_ARGS="--config C5": the libraries alternated, 3 rounds
      mkdir -p $OUT/abn
      for rep in 1 2 3; do
        for lib in $ABN_LIBS; do
          n=$(basename $lib .so)
          MAGOT_LIB=$lib timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline --no-box-state $ABN_ARGS > $OUT/abn/$n.$rep.json 2> $OUT/abn/err || { tail -20 $OUT/abn/err; exit 1; }
          python3 -c "import json;d=json.load(open('$OUT/abn/$n.$rep.json'));print('$n', round(d['roofline']['kernel_ms'],5), round(d['ms_per_step'],5))"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
