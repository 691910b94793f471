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
OUT=gpurun_out/$TAG; mkdir -p $OUT
BENCH="bench.py"
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
if has slow; then
  timeout -k 10 900 python -u -m pytest tests -m "gpu and slow" -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1 || { tail -40 $OUT/pytest_gpu_slow.log; exit 1; }
  tail -1 $OUT/pytest_gpu_slow.log
fi
if has bench; then
  timeout -k 10 900 python $BENCH > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if has kt; then
  rm -rf $OUT/kt
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python $BENCH > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
  grep -h extract_kernel $OUT/kt/kt_kernel_stats.csv
  cat $OUT/kt.json
fi
if has pmc; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    rm -rf $OUT/pmc$i
    timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python bench.py --steps 5 --warmup 1 --no-verify --no-cpu-baseline > $OUT/pmc$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc group $i failed rc=$rc"; tail -3 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit 1; fi
  done
  python scripts/pmc_summary.py $OUT > $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
fi
