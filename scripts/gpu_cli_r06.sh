#!/bin/bash
# The non-slow GPU suite, then the gff2fasta CLI on C3 end to end: the phase
# run (record and genome layouts, plan_create's own phases), then three
# whole calls in fresh processes (the CLI's phase clock).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06cli}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
MAGOT_GFF_TIMING=1 MAGOT_PLAN_TIMING=1 timeout -k 10 900 python scripts/e2e_cli.py --config C3 --seq-type protein --layout genome > $OUT/e2e_protein.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
grep -E "plan|gffplan" $OUT/e2e.err
for i in 1 2 3; do
  MAGOT_GFF_TIMING=1 timeout -k 10 300 python scripts/e2e_cli.py --config C3 --seq-type protein --whole > $OUT/e2e_whole$i.json 2> $OUT/e2e_whole$i.err || { tail -20 $OUT/e2e_whole$i.err; exit 1; }
  cat $OUT/e2e_whole$i.json; grep gffplan $OUT/e2e_whole$i.err
done
rm -rf /tmp/magot_e2e
