#!/bin/bash
# A/B of one build under two environments, alternated, 3 rounds:
#   scripts/ab_env.sh "A_ENV" "B_ENV" [bench args]   e.g. "" "MAGOT_NO_CODE2=1" --steps 300
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
A=$1; B=$2; shift 2
OUT=gpurun_out/abenv; mkdir -p $OUT
for i in 1 2 3; do
  for v in A B; do
    e=$A; [ $v = B ] && e=$B
    env $e timeout -k 10 300 python bench.py --no-verify --no-cpu-baseline "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -20 $OUT/$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v [$e]', '%.4f'%d['roofline']['kernel_ms'], '%.4f'%d['ms_per_step'])"
  done
done
