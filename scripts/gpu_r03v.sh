#!/bin/bash
# orf6_kernel v20 ablation (wrong output): no output stores; staging and
# segment tables only (no chunk loop); C5, 3 alternating rounds.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_nostore.so scripts/lib_stageonly.so" --config C5 --steps 100
