#!/bin/bash
# One build under several environments, alternated, 3 rounds:
#   scripts/ab_envs.sh "ENV_A" "ENV_B" ... -- [bench args]
#   e.g. scripts/ab_envs.sh "X=0" "MAGOT_ORF6_ORDER=record" -- --config C5
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=${AB_OUT:-gpurun_out/abenvs}; mkdir -p $OUT
for i in 1 2 3; do
  k=0
  for e in "${ENVS[@]}"; do
    k=$((k+1))
    env $e timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline "$@" > $OUT/v$k.$i.json 2> $OUT/v$k.$i.err || { tail -20 $OUT/v$k.$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/v$k.$i.json'));print('[$e]', '%.4f'%d['roofline']['kernel_ms'], '%.4f'%d['ms_per_step'])"
  done
done
