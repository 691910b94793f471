#!/bin/bash
# extract_kernel's output store policy (scripts/experiments/store_policy.patch):
# nt (the product) against sc1 (the line leaves the XCD's L2), nt sc1 and
# sc0 sc1; HBM traffic per launch and kernel time in alternating rounds.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06store}; mkdir -p $OUT
python -m magot_amd.build > /dev/null || exit 1
cp magot_amd/libmagot.so scripts/lib_base.so
for v in SC1 NT_SC1 SC0_SC1; do
  n=$(echo $v | tr 'A-Z' 'a-z')
  bash scripts/build_patch_variant.sh $n scripts/experiments/store_policy.patch -- -DMAGOT_EXP_STORE_$v > $OUT/build_$n.log 2>&1 || { tail -20 $OUT/build_$n.log; exit 1; }
done
# one verified line per variant first (same bytes, different cache policy)
for n in sc1 nt_sc1 sc0_sc1; do
  MAGOT_LIB=scripts/lib_$n.so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-box-state --no-layout-compare > $OUT/verify_$n.json 2> $OUT/verify_$n.err || { tail -20 $OUT/verify_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/verify_$n.json'));print('$n', d['parity'])"
done
bash scripts/ab_pmc_libs.sh $OUT extract_kernel "scripts/lib_base.so scripts/lib_sc1.so scripts/lib_nt_sc1.so scripts/lib_sc0_sc1.so" --no-layout-compare
