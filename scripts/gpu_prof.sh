#!/bin/bash
# rocprofv3 passes over the extraction kernel: kernel trace + stats, then one
# PMC pass per counter group (never combined with any other trace domain).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=${1:-C3}
OUT=gpurun_out/prof_$CFG
rm -rf $OUT; mkdir -p $OUT
P="python scripts/prof_kernel.py --config $CFG --iters 10"
timeout -k 10 300 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $P > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- $P > $OUT/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc group $i failed rc=$rc"; tail -5 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit 1; fi
done
ls -R $OUT | head -50
