#!/bin/bash
# Fresh PMC counters on the current kernels: C3 (extract_kernel) and C5 (orf6_kernel).
cd "$(dirname "$0")/.."
bash scripts/gpu_round.sh r03m pmc || exit 1
TAG=r03m_c5 bash scripts/gpu_pmc_c5.sh
