set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sorder2; mkdir -p $OUT
for v in base sorder; do
  for grp in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    tag=$v.$(echo $grp | cut -c1-5)
    MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/$tag -o pmc -- python bench.py --config C5 --steps 5 --warmup 1 --settle-ms 0 --no-verify --no-cpu-baseline > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  done
done
python scripts/pmc_summary.py $OUT orf6_kernel > $OUT/pmc_summary.json && cat $OUT/pmc_summary.json
for i in 1 2 3 4; do
  for v in sorder base; do
    MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline --config C5 --steps 100 --warmup 20 > $OUT/$v.$i.json 2> $OUT/$v.$i.err || { tail -20 $OUT/$v.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v.$i.json'));print('$v', d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
