#!/bin/bash
# Upper bound of a 2-bit genome plane: the half-density window diagnostic
# (lib_half.so, wrong output, same VALU work) against the plain build, A/B
# alternated on one box, then one FETCH_SIZE pass each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab_bench.sh $PWD/scripts/lib_base.so $PWD/scripts/lib_half.so --steps 300 || exit 1
for v in base half; do
  rm -rf gpurun_out/ab/pmc_$v
  MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ab/pmc_$v -o pmc -- python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline > gpurun_out/ab/pmc_$v.log 2>&1 || exit 1
  echo $v; python scripts/pmc_summary.py gpurun_out/ab/pmc_$v | grep FETCH
done
