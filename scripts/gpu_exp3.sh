#!/bin/bash
# Instruction and wait counters per variant (PMC passes only).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp3; rm -rf $OUT; mkdir -p $OUT
run() {  # name outputs dbg counters...
  n=$1; o=$2; d=$3; shift 3
  MAGOT_DEBUG_PATHS=$d timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o pmc -- python scripts/prof_kernel.py --order sorted --outputs $o --iters 5 > $OUT/$n.log 2>&1 || exit 1
}
for v in "full nuc+pep 0" "nuc nuc 0" "noloads_nuc nuc 4" "prologue nuc+pep 8" "slownuc nuc 1"; do
  set -- $v
  run ${1}_ins $2 $3 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES
  run ${1}_wait $2 $3 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
done
python scripts/pmc_summary.py $OUT
