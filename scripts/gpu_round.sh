#!/bin/bash
# One measured round on the GPU box: parity tests, the bench line, the bench
# under rocprofv3 kernel-trace (--stats), then PMC passes (one counter group
# per pass, never combined with other trace domains) over the same bench
# command.  Every GPU step has its own time limit; the chain stops at the
# first failure.   usage: scripts/gpu_round.sh TAG [stages...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r01}; shift
STAGES=${*:-tests slow bench kt pmc}
# stages: tests slow bench driver c2 c5 multi multi5 rehearse kt kt5 kt2 pmc traffic e2e smoke
#         dist dist5 fetchcal gloo8c3 gloo8c5 c4shares c4sharesg c5shares launchcost c2order planorder pytest:<file>
OUT=gpurun_out/$TAG; mkdir -p $OUT
BENCH="bench.py"
bash scripts/box_info.sh $OUT/box_before
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for st in $STAGES; do
  # pytest:<path>[::<test>] -- one test file (or test) under -m gpu
  if [[ $st == pytest:* ]]; then
    t=${st#pytest:}; n=$(echo "$t" | tr '/:' '__')
    timeout -k 10 900 python -u -m pytest "$t" -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_$n.log 2>&1 || { tail -40 $OUT/pytest_$n.log; exit 1; }
    tail -1 $OUT/pytest_$n.log
  fi
done
if has dist; then
  # the C3 job through the multi-GPU path at N=1: RCCL process group of one rank
  NCCL_DEBUG=INFO timeout -k 10 600 python $BENCH --dist --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_dist_c3.json 2> $OUT/dist_c3.err || { tail -30 $OUT/dist_c3.err; exit 1; }
  cut -c1-600 $OUT/bench_dist_c3.json
fi
if has dist5; then
  NCCL_DEBUG=INFO timeout -k 10 900 python $BENCH --dist --config C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_dist_c5.json 2> $OUT/dist_c5.err || { tail -30 $OUT/dist_c5.err; exit 1; }
  cut -c1-600 $OUT/bench_dist_c5.json
fi
if has fetchcal; then
  # FETCH_SIZE calibration for 12-byte buffer-load windows (scripts/fetchcal.hip)
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 scripts/fetchcal.hip -o /tmp/fetchcal.bin || exit 1
  timeout -k 10 120 /tmp/fetchcal.bin > $OUT/fetchcal_plain.jsonl || exit 1
  rm -rf $OUT/fetchcal_pmc $OUT/fetchcal_kt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetchcal_pmc -o pmc -- /tmp/fetchcal.bin > $OUT/fetchcal_pmc.jsonl 2> $OUT/fetchcal_pmc.err || { tail -5 $OUT/fetchcal_pmc.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/fetchcal_pmc2 -o pmc -- /tmp/fetchcal.bin > $OUT/fetchcal_pmc2.jsonl 2> $OUT/fetchcal_pmc2.err || { tail -5 $OUT/fetchcal_pmc2.err; }
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fetchcal_kt -o kt -- /tmp/fetchcal.bin > $OUT/fetchcal_kt.jsonl 2> $OUT/fetchcal_kt.err || { tail -5 $OUT/fetchcal_kt.err; exit 1; }
  cat $OUT/fetchcal_plain.jsonl
fi
for cfg in C3 C5; do
  if has gloo8${cfg,,}; then
    # the strong job over 8 ranks sharing this card (gloo, device tensors as under nccl)
    MAGOT_DIST_BACKEND=gloo MAGOT_COLLECTIVE_TENSORS=cuda timeout -k 10 900 python $BENCH --gpus 8 --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo8_$cfg.json 2> $OUT/gloo8_$cfg.err || { tail -30 $OUT/gloo8_$cfg.err; exit 1; }
    grep '^{' $OUT/bench_gloo8_$cfg.json | cut -c1-300
  fi
done
if has c4shares; then
  timeout -k 10 600 python scripts/c4_shares.py > $OUT/c4_shares.json 2> $OUT/c4_shares.err || { tail -20 $OUT/c4_shares.err; exit 1; }
  tail -8 $OUT/c4_shares.err
fi
if has c4sharesg; then
  timeout -k 10 600 python scripts/c4_shares.py --order genome > $OUT/c4_shares_genome.json 2> $OUT/c4_shares_genome.err || { tail -20 $OUT/c4_shares_genome.err; exit 1; }
  tail -8 $OUT/c4_shares_genome.err
fi
if has c5shares; then
  timeout -k 10 900 python scripts/c4_shares.py --config C5 --launches 50 > $OUT/c5_shares.json 2> $OUT/c5_shares.err || { tail -20 $OUT/c5_shares.err; exit 1; }
  tail -8 $OUT/c5_shares.err
fi
if has launchcost; then
  timeout -k 10 300 python scripts/launch_cost.py > $OUT/launch_cost.json 2> $OUT/launch_cost.err || { tail -20 $OUT/launch_cost.err; exit 1; }
  rm -rf $OUT/launch_kt
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/launch_kt -o kt -- python scripts/launch_cost.py > $OUT/launch_cost_kt.json 2> $OUT/launch_cost_kt.err || { tail -20 $OUT/launch_cost_kt.err; exit 1; }
  cat $OUT/launch_cost.json
fi
if has c2order; then
  timeout -k 10 300 python scripts/c2_draw_order.py > $OUT/c2_draw_order.json 2> $OUT/c2_draw_order.err || { tail -20 $OUT/c2_draw_order.err; exit 1; }
  cat $OUT/c2_draw_order.json
fi
if has planorder; then
  # record- vs genome-order extraction plans, alternating rounds (scripts/plan_order_ab.py)
  timeout -k 10 600 python scripts/plan_order_ab.py > $OUT/plan_order.json 2> $OUT/plan_order.err || { tail -20 $OUT/plan_order.err; exit 1; }
  tail -16 $OUT/plan_order.err
fi
if has slow; then
  timeout -k 10 900 python -u -m pytest tests -m "gpu and slow" -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1 || { tail -40 $OUT/pytest_gpu_slow.log; exit 1; }
  tail -1 $OUT/pytest_gpu_slow.log
fi
if has bench; then
  timeout -k 10 900 python $BENCH > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if has driver; then
  timeout -k 10 300 python $BENCH --steps 20 --warmup 5 > $OUT/bench_driver_cfg_20_5.json 2> $OUT/driver.err || { tail -30 $OUT/driver.err; exit 1; }
  cat $OUT/bench_driver_cfg_20_5.json
fi
if has c2; then
  timeout -k 10 300 python $BENCH --config C2 > $OUT/bench_c2.json 2> $OUT/c2.err || { tail -30 $OUT/c2.err; exit 1; }
  cat $OUT/bench_c2.json
fi
if has c5; then
  timeout -k 10 600 python $BENCH --config C5 > $OUT/bench_c5.json 2> $OUT/c5.err || { tail -30 $OUT/c5.err; exit 1; }
  cat $OUT/bench_c5.json
fi
if has multi5; then
  # the C5 job over two ranks sharing the card (gloo): six-frame outputs gathered back
  MAGOT_DIST_BACKEND=gloo MAGOT_COLLECTIVE_TENSORS=cuda timeout -k 10 900 python $BENCH --gpus 2 --config C5 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo2_c5.json 2> $OUT/gloo2_c5.err || { tail -30 $OUT/gloo2_c5.err; exit 1; }
  grep '^{' $OUT/bench_gloo2_c5.json | cut -c1-400
fi
if has e2e; then
  MAGOT_GENOME_TIMING=1 MAGOT_GFF_TIMING=1 timeout -k 10 900 python scripts/e2e_cli.py --config C3 --seq-type protein > $OUT/e2e_protein.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
  cat $OUT/e2e_protein.json
  rm -rf /tmp/magot_e2e
fi
if has gffab; then
  # host planner A/B on the box's CPUs: HEAD's gffplan.cpp against the copy
  # under scripts/ab_old/ (git-ignored), both built here
  bash scripts/gffplan_ab.sh build scripts/ab_old/magot_amd/csrc/gffplan.cpp > $OUT/gffab_build.log 2>&1 || { tail -20 $OUT/gffab_build.log; exit 1; }
  AB_TIMING=1 timeout -k 10 600 bash scripts/gffplan_ab.sh run $OUT/gffab 4 > $OUT/gffab.log 2>&1 || { tail -20 $OUT/gffab.log; exit 1; }
  grep plan_s $OUT/gffab/gffplan_ab.txt
fi
if has whole; then
  # the phase run (writes the C3 files and the reference out.fa; genome-order
  # plan as the CLI builds it), then three whole gff2fasta calls on those
  # files in fresh processes (the CLI's phase clock)
  MAGOT_GFF_TIMING=1 MAGOT_PLAN_TIMING=1 timeout -k 10 900 python scripts/e2e_cli.py --config C3 --seq-type protein --layout genome > $OUT/e2e_protein.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
  cat $OUT/e2e_protein.json
  for i in 1 2 3; do
    MAGOT_GFF_TIMING=1 timeout -k 10 300 python scripts/e2e_cli.py --config C3 --seq-type protein --whole > $OUT/e2e_whole$i.json 2> $OUT/e2e_whole$i.err || { tail -20 $OUT/e2e_whole$i.err; exit 1; }
    cat $OUT/e2e_whole$i.json
  done
  rm -rf /tmp/magot_e2e
fi
if has wholenuc; then
  # the same for seq_type=nucleotide (606 MB of text)
  MAGOT_GFF_TIMING=1 timeout -k 10 900 python scripts/e2e_cli.py --config C3 --seq-type nucleotide --layout genome > $OUT/e2e_nucleotide.json 2> $OUT/e2e_nuc.err || { tail -20 $OUT/e2e_nuc.err; exit 1; }
  cat $OUT/e2e_nucleotide.json
  for i in 1 2 3; do
    timeout -k 10 300 python scripts/e2e_cli.py --config C3 --seq-type nucleotide --whole > $OUT/e2e_whole_nuc$i.json 2> $OUT/e2e_whole_nuc$i.err || { tail -20 $OUT/e2e_whole_nuc$i.err; exit 1; }
    cat $OUT/e2e_whole_nuc$i.json
  done
  rm -rf /tmp/magot_e2e
fi
if has multi; then
  # two ranks launched by bench itself, sharing the one card over gloo (the
  # C4 orchestration; the driver's 8-GPU node runs it over RCCL)
  MAGOT_DIST_BACKEND=gloo MAGOT_COLLECTIVE_TENSORS=cuda timeout -k 10 600 python $BENCH --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/bench_gloo2.json 2> $OUT/gloo2.err || { tail -30 $OUT/gloo2.err; exit 1; }
  grep '^{' $OUT/bench_gloo2.json
fi
if has kt; then
  # the bench line under the kernel trace; rocprof_summary.py --timed averages
  # exactly the line's K timed dispatches (roofline.timed_launches)
  rm -rf $OUT/kt
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python $BENCH --no-box-state > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
  grep -h extract_kernel $OUT/kt/kt_kernel_stats.csv
  cat $OUT/kt.json
fi
if has rehearse; then
  # one GPU's share of the K-GPU C4 job (bench.py --rehearse-shard K:r)
  for kr in 2:0 4:0 8:0 8:7; do
    timeout -k 10 300 python $BENCH --rehearse-shard $kr --steps 300 --no-cpu-baseline > $OUT/rehearse_${kr/:/_}.json 2> $OUT/rehearse.err || { tail -20 $OUT/rehearse.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/rehearse_${kr/:/_}.json'));r=d['roofline'];print('$kr', round(d['ms_per_step'],5), round(r['kernel_ms'],5), round(r['frac'],4), d['parity'][:20])"
  done
fi
for cfg in C5 C2; do
  if has kt${cfg:1}; then
    rm -rf $OUT/kt_$cfg
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$cfg -o kt -- python $BENCH --config $cfg --no-cpu-baseline --no-box-state > $OUT/kt_$cfg.json 2> $OUT/kt_$cfg.err || { tail -30 $OUT/kt_$cfg.err; exit 1; }
    grep -h "orf6_kernel\|extract_kernel" $OUT/kt_$cfg/kt_kernel_stats.csv
  fi
done
if has pmc; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    rm -rf $OUT/pmc$i
    timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python bench.py --steps 5 --warmup 1 --no-verify --no-cpu-baseline --no-box-state --no-layout-compare > $OUT/pmc$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc group $i failed rc=$rc"; tail -3 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit 1; fi
  done
  python scripts/pmc_summary.py $OUT > $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
fi
if has traffic; then
  # HBM bytes per launch (FETCH_SIZE, WRITE_SIZE passes) of the C3, C5 and C2
  # lines: scripts/pmc_json.py DIR CONFIG KERNEL turns each into profiles/pmc_<config>.json
  for cfg in C3:extract_kernel C5:orf6_kernel C2:extract_kernel; do
    c=${cfg%%:*}
    for grp in FETCH_SIZE WRITE_SIZE; do
      rm -rf $OUT/traffic_$c/$grp
      timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/traffic_$c/$grp -o pmc -- python bench.py --config $c --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline --no-box-state --no-layout-compare > $OUT/traffic_$c.$grp.log 2>&1 || { echo "traffic $c $grp failed"; tail -3 $OUT/traffic_$c.$grp.log; exit 1; }
    done
  done
  echo traffic ok
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
bash scripts/box_info.sh $OUT/box_after
