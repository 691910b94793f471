#!/bin/bash
# Round 3, first GPU check: GPU tests (new bench/multi-rank tests included),
# the C3 line, the two-rank C4 rehearsal launched by bench itself.
cd "$(dirname "$0")/.."
bash scripts/gpu_round.sh r03a tests bench multi
