#!/bin/bash
# PMC counter passes (one group per run, no tracing domains) over the C5 bench;
# summary per orf6_kernel launch.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_c5}; rm -rf $OUT; mkdir -p $OUT
KERNEL=${KERNEL:-orf6_kernel}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python bench.py --config C5 --steps 3 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline > $OUT/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc group $i failed rc=$rc"; tail -3 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit 1; fi
done
python scripts/pmc_summary.py $OUT $KERNEL > $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
