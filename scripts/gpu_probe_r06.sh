#!/bin/bash
# Round 6 probes: the non-slow GPU suite, RCCL's INIT log file under
# bench.dist_setup, the counters rocprofv3 offers on this box, and the CLI's
# phase clock (plus plan_create's own phases) on C3.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06b}; mkdir -p $OUT
timeout -k 10 120 python scripts/rccl_log_probe.py > $OUT/rccl_log_probe.jsonl 2> $OUT/rccl_log_probe.err || { tail -20 $OUT/rccl_log_probe.err; exit 1; }
cat $OUT/rccl_log_probe.jsonl
MAGOT_GFF_TIMING=1 MAGOT_PLAN_TIMING=1 timeout -k 10 900 python scripts/e2e_cli.py --config C3 --seq-type protein > $OUT/e2e_protein.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
cat $OUT/e2e.err | grep plan
MAGOT_GFF_TIMING=1 MAGOT_PLAN_TIMING=1 timeout -k 10 300 python scripts/e2e_cli.py --config C3 --seq-type protein --layout genome > $OUT/e2e_protein_genome.json 2> $OUT/e2e_genome.err || { tail -20 $OUT/e2e_genome.err; exit 1; }
cat $OUT/e2e_genome.err | grep plan
for i in 1 2; do
  MAGOT_GFF_TIMING=1 timeout -k 10 300 python scripts/e2e_cli.py --config C3 --seq-type protein --whole > $OUT/e2e_whole$i.json 2> $OUT/e2e_whole$i.err || { tail -20 $OUT/e2e_whole$i.err; exit 1; }
  cat $OUT/e2e_whole$i.json; tail -5 $OUT/e2e_whole$i.err
done
rm -rf /tmp/magot_e2e
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
