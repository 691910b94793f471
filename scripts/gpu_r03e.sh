#!/bin/bash
# Round 3 after the orf6 fix: all GPU tests (slow included), the C3 / driver /
# C5 / C2 lines, kernel traces of the C3, C5 and C2 lines.
cd "$(dirname "$0")/.."
bash scripts/gpu_round.sh r03e tests slow bench driver c5 c2 kt kt5 kt2
