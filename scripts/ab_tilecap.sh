#!/bin/bash
# Tile-count A/B for extract_kernel (apply scripts/experiments/tile_cap.patch
# first): MAGOT_EXTRACT_TILE_BYTES caps the tile
# below its slot size, so a plan's tile count lands just under a whole number
# of resident-wave rounds (6144 waves: 256 CUs x 6 blocks x 4).  One GPU's
# share of the 4- and 8-GPU jobs and the full C3 job, alternating, two rounds.
#   scripts/ab_tilecap.sh OUTDIR "8:0=0,2816,2560" "full=0,4864" ...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=$1; shift; mkdir -p $OUT
for rep in 1 2; do
  for spec in "$@"; do
    what=${spec%%=*}; caps=${spec#*=}
    for cap in ${caps//,/ }; do
      args="--steps 300 --no-cpu-baseline --no-verify --no-box-state"
      [ $what != full ] && args="$args --rehearse-shard $what"
      envs=""; [ $cap != 0 ] && envs="MAGOT_EXTRACT_TILE_BYTES=$cap"
      f=$OUT/${what/:/_}.$cap.$rep.json
      env $envs timeout -k 10 300 python bench.py $args > $f 2> $OUT/err || { tail -20 $OUT/err; exit 1; }
      python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$what cap=$cap', round(d['ms_per_step'],5), round(r['kernel_ms'],5))"
    done
  done
done
