#!/bin/bash
# Issue/stall counters for the extraction kernel, full and nucleotide-only.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp7; rm -rf $OUT; mkdir -p $OUT
for outs in nuc+pep nuc; do
  P="python scripts/prof_kernel.py --order sorted --iters 5 --outputs $outs"
  i=0
  for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
             "SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_ACTIVE_INST_EXP"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/$outs/p$i -o pmc -- $P > $OUT/$outs.p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$outs pass $i failed rc=$rc"; grep -E "error|capab|not found|invalid" $OUT/$outs.p$i.log | head -3; [ $rc -ge 124 ] && exit 1; fi
  done
  python scripts/pmc_summary.py $OUT/$outs > $OUT/$outs.json
done
cat $OUT/nuc+pep.json $OUT/nuc.json
