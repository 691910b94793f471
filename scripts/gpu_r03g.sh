#!/bin/bash
cd "$(dirname "$0")/.."
bash scripts/gpu_round.sh r03g tests
