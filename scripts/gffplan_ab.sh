#!/bin/bash
# A/B of the host gff2fasta planner on the C3 GFF3 (no GPU): two binaries
# built from two versions of gffplan.cpp, run alternately on the same file.
#   build here:  scripts/gffplan_ab.sh build OLD_GFFPLAN_CPP
#   run:         scripts/gffplan_ab.sh run OUT_DIR [ROUNDS]   (AB_TIMING=1: phase times)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
F="-std=c++17 -O3 --offload-arch=gfx950 -x hip --offload-host-only -I$ROOT/include"
if [ "$1" = build ]; then
  OLD=$2
  /opt/rocm/bin/hipcc $F -I$ROOT/magot_amd/csrc -c "$ROOT/scripts/gffplan_bench.cpp" -o /tmp/gb_main.o
  /opt/rocm/bin/hipcc $F -I$ROOT/magot_amd/csrc -c "$ROOT/magot_amd/csrc/gffplan.cpp" -o /tmp/gb_new.o
  /opt/rocm/bin/hipcc $F -I$(dirname "$OLD") -c "$OLD" -o /tmp/gb_old.o
  /opt/rocm/bin/hipcc -o "$ROOT/scripts/gffplan_new.bin" /tmp/gb_main.o /tmp/gb_new.o -lpthread
  /opt/rocm/bin/hipcc -o "$ROOT/scripts/gffplan_old.bin" /tmp/gb_main.o /tmp/gb_old.o -lpthread
  exit 0
fi
OUT=$2; ROUNDS=${3:-4}
mkdir -p "$OUT"
D=$(mktemp -d)
python - "$D" <<'PY'
import os, sys
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
from magot_amd import synth
d = sys.argv[1]
w = synth.make('C3')
with open(os.path.join(d, 'ann.gff3'), 'w') as fh:
    fh.write(w.gff3_text())
with open(os.path.join(d, 'ctgs.txt'), 'w') as fh:
    fh.write('\n'.join('%s %d' % (n, l) for n, l in zip(w.contig_names, w.contig_len)))
PY
for i in $(seq "$ROUNDS"); do
  for v in old new; do
    env ${AB_TIMING:+MAGOT_GFF_TIMING=1} "$ROOT/scripts/gffplan_$v.bin" "$D/ann.gff3" "$D/ctgs.txt" 3 2>&1 |
      sed "s/^/$v /" | tee -a "$OUT/gffplan_ab.txt"
  done
done
rm -rf "$D"
