#!/bin/bash
# Diagnostic: does extra VALU work cost more back-to-back than in isolated
# launches?  (kernel trace of 200 back-to-back steps + 20 isolated launches)
# Needs scripts/experiments/dummy_valu.patch applied, then
#   scripts/build_variant.sh valu -DMAGOT_EXP_DUMMY_VALU=100 and lib_base.so = the plain build.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/valu; rm -rf $OUT; mkdir -p $OUT
for v in base valu base valu; do
  rm -rf $OUT/$v
  MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o kt -- python bench.py --steps 200 --warmup 20 --settle-ms 0 --no-verify --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  python3 - $v <<'PY'
import csv, glob, sys, json
v = sys.argv[1]
rows = [r for f in glob.glob('gpurun_out/valu/%s/**/*kernel_trace.csv' % v, recursive=True)
        for r in csv.DictReader(open(f)) if 'extract_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows]
W, S = 20, 200  # bench --warmup 20 --steps 200 --no-verify: W warm-up, S back-to-back, 20 isolated
assert len(d) == 8 + W + S + 20, len(d)  # 8: the minimum settle (bench.settle)
b2b, iso = d[8 + W:8 + W + S], d[8 + W + S:]
print(v, 'b2b %.4f' % (sum(b2b) / len(b2b)), 'isolated %.4f' % (sum(iso) / len(iso)))
PY
done
# round 2: the same with the bench's settle phase (100 ms of launches first)
for v in base valu base valu; do
  rm -rf $OUT/s$v
  MAGOT_LIB=$PWD/scripts/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/s$v -o kt -- python bench.py --steps 200 --warmup 20 --no-verify --no-cpu-baseline > $OUT/s$v.json 2> $OUT/s$v.err || { tail -5 $OUT/s$v.err; exit 1; }
  python3 - s$v <<'PY'
import csv, glob, sys
v = sys.argv[1]
rows = [r for f in glob.glob('gpurun_out/valu/%s/**/*kernel_trace.csv' % v, recursive=True)
        for r in csv.DictReader(open(f)) if 'extract_kernel' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows]
W, S = 20, 200
iso = d[-20:]
b2b = d[-20 - S:-20]  # the settle launches come before the warm-up
print(v, 'settled b2b %.4f' % (sum(b2b) / len(b2b)), 'isolated %.4f' % (sum(iso) / len(iso)), 'launches', len(d))
PY
done
