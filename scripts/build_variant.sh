#!/bin/bash
# Build an A/B variant of libmagot.so with extra compile definitions, e.g.
#   scripts/build_variant.sh nt -DMAGOT_EXP_NT_STORE   -> scripts/lib_nt.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
python -m magot_amd.build > /dev/null
D=magot_amd/_build/var_$NAME; mkdir -p $D
objs=""
for f in magot_amd/_build/*.o; do
  b=$(basename $f)
  if [ $b = extract.hip.o ] || [ $b = seqops.hip.o ] || [ $b = abi.hip.o ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude "$@" -x hip -c magot_amd/csrc/${b%.o} -o $D/$b
    objs="$objs $D/$b"
  else
    objs="$objs $f"
  fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o scripts/lib_$NAME.so $objs -lpthread
echo scripts/lib_$NAME.so
