#!/bin/bash
# extract_kernel attribution (scripts/experiments/extract_attribution.patch,
# wrong output): without nucleotide stores, without peptide stores, without
# any store, without genome window loads; C3, 3 alternating runs.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_nonuc.so scripts/lib_nopep.so scripts/lib_nostore.so scripts/lib_noload.so" --steps 300
