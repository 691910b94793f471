#!/bin/bash
# Build an A/B variant of libmagot.so from the current sources with patches
# from scripts/experiments applied (in a scratch copy; the tree is untouched):
#   scripts/build_patch_variant.sh NAME PATCH... [-- -DFLAG...]  -> scripts/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
PATCHES=(); FLAGS=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; FLAGS=("$@"); break; fi
  PATCHES+=("$1"); shift
done
python -m magot_amd.build > /dev/null
W=/tmp/magot_variant_$NAME; rm -rf $W; mkdir -p $W
cp -r magot_amd include $W/
ROOT=$(pwd)
for p in "${PATCHES[@]}"; do (cd $W && patch -p1 -s < "$ROOT/$p"); done
objs=""
hdr=0  # a changed header recompiles every translation unit
for h in $W/magot_amd/csrc/*.h $W/include/*.h; do
  cmp -s $h ${h#$W/} || hdr=1
done
for s in $W/magot_amd/csrc/*.hip $W/magot_amd/csrc/*.cpp; do
  b=$(basename $s)
  if [ $hdr = 1 ] || ! cmp -s $s magot_amd/csrc/$b || [ ${#FLAGS[@]} -gt 0 ]; then
    lang=""; [[ $b == *.hip ]] && lang="-x hip"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -I$W/include "${FLAGS[@]}" $lang -c $s -o $W/$b.o
    objs="$objs $W/$b.o"
  else
    objs="$objs magot_amd/_build/$b.o"
  fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o scripts/lib_$NAME.so $objs -lpthread
echo scripts/lib_$NAME.so
