#!/bin/bash
# VERDICT r4 item 3 on one box: the structural attempt at extract_kernel's
# genome reads (scripts/experiments/xcd_contiguous.patch, one contiguous run
# of blocks per XCD) A/B'd against the product library, alternating, with
# FETCH_SIZE / WRITE_SIZE passes of both, and the product kernel on a
# coordinate-sorted record order (the locality bound).
#   usage: scripts/gpu_c3_reads.sh TAG VARIANT_LIB
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; VAR=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
B="python bench.py --no-verify --no-cpu-baseline --no-box-state"
for i in 1 2 3; do
  for v in base var; do
    lib=magot_amd/libmagot.so; [ $v = var ] && lib=$VAR
    MAGOT_LIB=$lib timeout -k 10 300 $B > $OUT/ab_$v$i.json 2> $OUT/ab_$v$i.err || { tail -20 $OUT/ab_$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/ab_$v$i.json'));print('$v', d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
timeout -k 10 300 $B --order sorted > $OUT/sorted.json 2> $OUT/sorted.err || { tail -20 $OUT/sorted.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/sorted.json'));print('sorted', d['roofline']['kernel_ms'], d['ms_per_step'])"
for v in base var sorted; do
  lib=magot_amd/libmagot.so; [ $v = var ] && lib=$VAR
  extra=""; [ $v = sorted ] && extra="--order sorted"
  for grp in FETCH_SIZE WRITE_SIZE; do
    rm -rf $OUT/pmc_$v/$grp
    MAGOT_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$v/$grp -o pmc -- python bench.py --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline --no-box-state $extra > $OUT/pmc_$v.$grp.log 2>&1 || { echo "pmc $v $grp failed"; tail -3 $OUT/pmc_$v.$grp.log; exit 1; }
  done
done
echo done
