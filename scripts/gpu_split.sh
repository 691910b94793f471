#!/bin/bash
# orf6_split_kernel (MAGOT_ORF6_SPLIT=1): orf6 GPU tests, a verified C5 line,
# then an alternating A/B against orf6_kernel.  Stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/split; mkdir -p $OUT
MAGOT_ORF6_SPLIT=1 timeout -k 10 240 python -u -m pytest tests -m "gpu and not slow" -x -q -k "orf6 or get_orfs or smoke" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MAGOT_ORF6_SPLIT=1 timeout -k 10 300 python bench.py --config C5 --steps 50 --no-cpu-baseline > $OUT/c5_verified.json 2> $OUT/c5.err || { tail -30 $OUT/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c5_verified.json'));print('split verified', d['ms_per_step'], d['parity'])"
bash scripts/ab_envs.sh "MAGOT_ORF6_SPLIT=0" "MAGOT_ORF6_SPLIT=1" -- --config C5 --steps 100 --warmup 20 > $OUT/ab.txt 2>&1; cat $OUT/ab.txt
