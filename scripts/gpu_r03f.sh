#!/bin/bash
cd "$(dirname "$0")/.."
bash scripts/gpu_round.sh r03f c5 c2 kt kt5 kt2
