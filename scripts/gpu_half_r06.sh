#!/bin/bash
# extract_kernel's read bound under the genome-order layout (VERDICT r5 item
# 3): the half-density diagnostic (scripts/experiments/half_density.patch,
# -DMAGOT_EXP_HALF: every window read at half the plane density -- a forward
# 2-bit plane's line footprint -- with the VALU unchanged and the output
# wrong) against the product kernel: reads per launch (FETCH_SIZE /
# WRITE_SIZE passes) and kernel time (3 alternating rounds).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06half}; mkdir -p $OUT
python -m magot_amd.build > /dev/null || exit 1
cp magot_amd/libmagot.so scripts/lib_base.so
bash scripts/build_patch_variant.sh half scripts/experiments/half_density.patch -- -DMAGOT_EXP_HALF > $OUT/build.log 2>&1 || { tail -20 $OUT/build.log; exit 1; }
bash scripts/ab_pmc_libs.sh $OUT extract_kernel "scripts/lib_base.so scripts/lib_half.so" --no-layout-compare
