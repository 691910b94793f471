#!/bin/bash
# Where orf6_kernel's VALU goes: SQ_INSTS_VALU / SQ_INSTS_LDS per launch for
# the full kernel and for the staging-only ablation (lib_nochunks: wrong
# output, no chunk loop), C5.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c5_split; mkdir -p $OUT
for v in head nochunks; do
  rm -rf $OUT/$v
  MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/$v -o pmc -- python bench.py --config C5 --steps 5 --warmup 1 --no-verify --no-cpu-baseline > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  python scripts/pmc_summary.py $OUT/$v orf6_kernel
done
