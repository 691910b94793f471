#!/bin/bash
# C5 run-to-run variation: two plain bench lines, one under the kernel trace,
# one more plain line, all on this box.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/r03h; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 400 python bench.py --config C5 --no-cpu-baseline --no-verify > $OUT/c5_$i.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c5_$i.json'));r=d['roofline'];print('plain$i', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['kernel_ms_isolated'],4))"
done
rm -rf $OUT/kt5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt5 -o kt -- python bench.py --config C5 --no-cpu-baseline --no-verify > $OUT/kt5.json 2> $OUT/kt5.err || { tail -20 $OUT/kt5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/kt5.json'));r=d['roofline'];print('kt', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['kernel_ms_isolated'],4))"
grep -h orf6 $OUT/kt5/kt_kernel_stats.csv
timeout -k 10 400 python bench.py --config C5 --no-cpu-baseline --no-verify > $OUT/c5_3.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5_3.json'));r=d['roofline'];print('plain3', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['kernel_ms_isolated'],4))"
