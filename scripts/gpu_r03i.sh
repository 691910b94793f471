#!/bin/bash
# A/B: current extract_kernel vs the 2-bit forward-plane diagnostic (D1, wrong
# output for lower case / exceptions), C3 default bench, 3 alternating runs.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_c2f.so" --steps 300
