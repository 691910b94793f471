#!/bin/bash
# orf6_kernel counters on the C5 line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/exp11; rm -rf $OUT; mkdir -p $OUT
P="python bench.py --config C5 --steps 2 --warmup 0 --no-verify"
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- $P > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
agg = collections.defaultdict(list)
for f in glob.glob('gpurun_out/exp11/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'orf6_kernel' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
print(json.dumps({k: sum(v) / len(v) for k, v in sorted(agg.items())}, indent=1))
PY
