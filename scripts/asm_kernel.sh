#!/bin/bash
# Device assembly of one kernel from a csrc file, with a short resource and
# memory-instruction summary (no GPU needed).
#   usage: scripts/asm_kernel.sh SRC.hip MANGLED_PREFIX [OUT_DIR=/tmp/asm]
set -o pipefail
SRC=$1; SYM=$2; OUT=${3:-/tmp/asm}
mkdir -p $OUT
ROOT=$(cd "$(dirname "$0")/.." && pwd)
base=$(basename $SRC .hip)
timeout 300 /opt/rocm/bin/hipcc $EXTRA -O3 -std=c++17 -I$ROOT/include --offload-arch=gfx950 -x hip \
  --cuda-device-only -S $SRC -o $OUT/$base.s 2>&1 | grep -v hip-link
s=$(grep -n "^${SYM}" $OUT/$base.s | head -1 | cut -d: -f1)
e=$(awk -v s=$s 'NR>s && /^\.Lfunc_end/ {print NR; exit}' $OUT/$base.s)
sed -n "${s},${e}p" $OUT/$base.s > $OUT/kernel.s
echo "kernel lines $s-$e -> $OUT/kernel.s"
echo "VALU $(grep -c '^\s*v_' $OUT/kernel.s)  SALU $(grep -c '^\s*s_' $OUT/kernel.s)  DS $(grep -c '^\s*ds_' $OUT/kernel.s)  VMEM $(grep -c '^\s*buffer_\|^\s*global_' $OUT/kernel.s)  scratch $(grep -c 'scratch_' $OUT/kernel.s)"
grep -A40 "\.name:\s*${SYM}" $OUT/$base.s | grep -m4 "vgpr_count\|sgpr_count\|private_segment_fixed_size\|spill"
