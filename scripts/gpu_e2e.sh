#!/bin/bash
# End-to-end CLI path on C3 (native planner + one kernel launch).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/e2e; mkdir -p $OUT
MAGOT_GENOME_TIMING=1 MAGOT_GFF_TIMING=1 timeout -k 10 900 python scripts/e2e_cli.py --config C3 --seq-type protein > $OUT/e2e_protein.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
cat $OUT/e2e_protein.json; cat $OUT/e2e.err
MAGOT_GENOME_TIMING=1 MAGOT_GFF_TIMING=1 timeout -k 10 300 python scripts/e2e_cli.py --config C3 --seq-type protein --whole > $OUT/e2e_whole.json 2> $OUT/e2e_whole.err || { tail -20 $OUT/e2e_whole.err; exit 1; }
cat $OUT/e2e_whole.json; cat $OUT/e2e_whole.err
timeout -k 10 300 python scripts/e2e_variants.py > $OUT/e2e_variants.json 2> $OUT/e2e_variants.err || { tail -20 $OUT/e2e_variants.err; exit 1; }
cat $OUT/e2e_variants.json
rm -rf /tmp/magot_e2e
