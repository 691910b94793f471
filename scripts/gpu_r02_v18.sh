#!/bin/bash
# Round-2 v18 (C5 kernel changes: DPP scans, exception-plane skip, multiply
# codon indices; C3 unchanged from v17): GPU tests, the C5 line with its
# kernel trace and traffic counters, the C3 line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r02_v18; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --config C5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
rm -rf $OUT/kt_c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c5 -o kt -- python bench.py --config C5 --no-cpu-baseline > $OUT/kt_c5.json 2> $OUT/kt_c5.err || { tail -20 $OUT/kt_c5.err; exit 1; }
grep -h "orf6" $OUT/kt_c5/kt_kernel_stats.csv
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1)); rm -rf $OUT/pmc_c5_$i
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c5_$i -o pmc -- python bench.py --config C5 --steps 3 --warmup 1 --no-verify --no-cpu-baseline > $OUT/pmc_c5_$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc_c5_$i.log; exit 1; }
done
python scripts/pmc_summary.py $OUT orf6_kernel > $OUT/pmc_summary_c5.json && cat $OUT/pmc_summary_c5.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
