#!/bin/bash
# orf6_kernel v20 output stores: plain (base) vs non-temporal; C5, 3 rounds.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_nt.so" --config C5 --steps 100
