#!/bin/bash
# Large extraction tiles whose ends fall on 1 KB / 4 KB output boundaries
# (scripts/experiments/tile_align_1k.patch: whole aligned 1 KB store
# instructions; the store replay writes 4096- and 6144-byte tiles at
# 6.05 / 5.83 TB/s against 5.52 for unaligned 5072-byte ones), with 7-9
# chunk slots per lane so the tiles stay as long as today's.  Each variant's
# C3 line verified once, then traffic and time in alternating rounds.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06tile}; mkdir -p $OUT
python -m magot_amd.build > /dev/null || exit 1
cp magot_amd/libmagot.so scripts/lib_base.so
P=scripts/experiments/tile_align_1k.patch
bash scripts/build_patch_variant.sh lc7a128 $P -- -DMAGOT_EXP_LC=7 -DMAGOT_EXP_PPL=3 -DMAGOT_EXP_ALIGN=128 > $OUT/build.log 2>&1 &&
bash scripts/build_patch_variant.sh lc7a1k $P -- -DMAGOT_EXP_LC=7 -DMAGOT_EXP_PPL=3 -DMAGOT_EXP_ALIGN=1024 >> $OUT/build.log 2>&1 &&
bash scripts/build_patch_variant.sh lc8a1k $P -- -DMAGOT_EXP_LC=8 -DMAGOT_EXP_PPL=3 -DMAGOT_EXP_ALIGN=1024 >> $OUT/build.log 2>&1 &&
bash scripts/build_patch_variant.sh lc9a4k $P -- -DMAGOT_EXP_LC=9 -DMAGOT_EXP_PPL=3 -DMAGOT_EXP_ALIGN=4096 >> $OUT/build.log 2>&1 &&
bash scripts/build_patch_variant.sh lc6a1k $P -- -DMAGOT_EXP_LC=6 -DMAGOT_EXP_PPL=2 -DMAGOT_EXP_ALIGN=1024 >> $OUT/build.log 2>&1 || { tail -20 $OUT/build.log; exit 1; }
LIBS="scripts/lib_base.so scripts/lib_lc7a128.so scripts/lib_lc7a1k.so scripts/lib_lc8a1k.so scripts/lib_lc9a4k.so scripts/lib_lc6a1k.so"
for lib in $LIBS; do
  n=$(basename $lib .so)
  MAGOT_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-box-state --no-layout-compare > $OUT/verify_$n.json 2> $OUT/verify_$n.err || { tail -20 $OUT/verify_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/verify_$n.json'));print('$n', d['parity'], d['roofline']['kernel_ms'])"
done
bash scripts/ab_pmc_libs.sh $OUT extract_kernel "$LIBS" --no-layout-compare
