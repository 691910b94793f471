#!/bin/bash
# Per-GPU share of the C4 job (rank 0 of 8, rehearsed on one card): tile size
# (5 / 4 / 3 chunk slots per lane) and the occupancy cap (6 blocks per CU vs
# none), 3 alternating runs each; then the same libraries at full C3 size.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03k; rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
  for v in base lc4 lc3 cap0; do
    lib=scripts/lib_$v.so; env=""
    [ $v = cap0 ] && { lib=scripts/lib_base.so; env="MAGOT_EXTRACT_BLOCKS_PER_CU=0"; }
    for kr in 8:0 4:0; do
      env $env MAGOT_LIB=$PWD/$lib timeout -k 10 300 python bench.py --rehearse-shard $kr --steps 300 --no-verify --no-cpu-baseline > $OUT/$v.$kr.$i.json 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/$v.$kr.$i.json'));print('$v $kr', round(d['roofline']['kernel_ms'],5), round(d['ms_per_step'],5))"
    done
  done
done
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_lc4.so" --steps 300
