#!/bin/bash
# Output-store cache policy A/B (C3, 300 steps, 3 alternating rounds):
# compiler nt (base), asm nt, nt sc0, nt sc1, sc0.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_ntasm.so scripts/lib_ntsc0.so scripts/lib_ntsc1.so scripts/lib_sc0.so" --steps 300
