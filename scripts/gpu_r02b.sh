#!/bin/bash
# Round 2: bench lines with the settle phase (defaults and the driver's
# --steps 20 --warmup 5), kernel trace --stats, and a clock pass: GRBM_GUI_ACTIVE
# and GRBM_COUNT per launch next to the kernel-trace durations of 200
# back-to-back launches (effective engine clock = cycles / duration).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02b}; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err || { tail -30 $OUT/bench_20_5.err; exit 1; }
cat $OUT/bench_20_5.json
rm -rf $OUT/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py --no-cpu-baseline > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
grep -h extract_kernel $OUT/kt/kt_kernel_stats.csv
rm -rf $OUT/clk
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --output-format csv -d $OUT/clk -o clk -- python bench.py --steps 200 --warmup 20 --settle-ms 0 --no-verify --no-cpu-baseline > $OUT/clk.json 2> $OUT/clk.err || { tail -30 $OUT/clk.err; exit 1; }
f=$(find $OUT/clk -name '*counter_collection.csv' | head -1)
head -2 "$f"
python3 - "$f" <<'PY'
import csv, sys, collections
rows = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    if 'extract_kernel' not in r['Kernel_Name']:
        continue
    k = r.get('Dispatch_Id') or r.get('Correlation_Id')
    d = rows.setdefault(k, dict(r))
    d[r['Counter_Name']] = float(r['Counter_Value'])
ds = list(rows.values())
print('launches', len(ds))
for i, d in enumerate(ds):
    if i % 20 == 0 or i < 3:
        dur = None
        if 'End_Timestamp' in d and 'Start_Timestamp' in d:
            dur = (int(d['End_Timestamp']) - int(d['Start_Timestamp'])) / 1e6
        print(i, dur, d.get('GRBM_GUI_ACTIVE'), d.get('GRBM_COUNT'), d.get('SQ_BUSY_CYCLES'))
PY
