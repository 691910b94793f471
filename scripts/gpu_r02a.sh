#!/bin/bash
# Round 2 first GPU pass: parity tests, bench at the defaults and at the
# driver's --steps 20 --warmup 5, a coordinate-sorted-record diagnostic, and a
# kernel trace of the driver configuration (per-launch durations in order).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r02a; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_20_5.json 2> $OUT/bench_20_5.err || { tail -30 $OUT/bench_20_5.err; exit 1; }
cat $OUT/bench_20_5.json
timeout -k 10 300 python bench.py --order sorted --no-cpu-baseline > $OUT/bench_sorted.json 2> $OUT/bench_sorted.err || { tail -30 $OUT/bench_sorted.err; exit 1; }
cat $OUT/bench_sorted.json
rm -rf $OUT/kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python bench.py --steps 300 --warmup 5 --no-cpu-baseline > $OUT/kt.json 2> $OUT/kt.err || { tail -30 $OUT/kt.err; exit 1; }
python3 - <<'PY'
import csv, glob
rows = [r for f in glob.glob('gpurun_out/r02a/kt/**/*kernel_trace.csv', recursive=True)
        for r in csv.DictReader(open(f)) if 'extract_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows]
t0 = int(rows[0]['Start_Timestamp'])
with open('gpurun_out/r02a/launch_order.txt', 'w') as fh:
    for r, x in zip(rows, d):
        fh.write('%.3f %.4f\n' % ((int(r['Start_Timestamp']) - t0) / 1e6, x))
print('launches', len(d), 'first 40:', ' '.join('%.3f' % x for x in d[:40]))
PY
