#!/bin/bash
# A/B of a variant library against the product one on one box: the variant's
# full bench line with the oracle check first, then R alternating rounds of
# both (kernel time by HIP events), then FETCH_SIZE / WRITE_SIZE passes of both.
#   usage: scripts/gpu_ab.sh TAG VARIANT_LIB CONFIG [ROUNDS]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; VAR=$2; CFG=$3; R=${4:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
B="python bench.py --config $CFG --no-cpu-baseline --no-box-state"
MAGOT_LIB=$VAR timeout -k 10 600 $B --steps 20 --warmup 5 > $OUT/var_verify.json 2> $OUT/var_verify.err || { tail -20 $OUT/var_verify.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/var_verify.json'));print('variant parity:', d['parity'])"
for i in $(seq 1 $R); do
  for v in base var; do
    lib=magot_amd/libmagot.so; [ $v = var ] && lib=$VAR
    MAGOT_LIB=$lib timeout -k 10 600 $B --no-verify > $OUT/ab_$v$i.json 2> $OUT/ab_$v$i.err || { tail -20 $OUT/ab_$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/ab_$v$i.json'));print('$v', d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
for v in base var; do
  lib=magot_amd/libmagot.so; [ $v = var ] && lib=$VAR
  for grp in FETCH_SIZE WRITE_SIZE; do
    rm -rf $OUT/pmc_$v/$grp
    MAGOT_LIB=$lib timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$v/$grp -o pmc -- python bench.py --config $CFG --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline --no-box-state --no-layout-compare > $OUT/pmc_$v.$grp.log 2>&1 || { echo "pmc $v $grp failed"; tail -3 $OUT/pmc_$v.$grp.log; exit 1; }
  done
done
echo done
