#!/bin/bash
# Multi-rank rehearsal on one GPU: C4 strong mode at world 1 (nccl = RCCL), then
# world 2 with the gloo backend (two ranks sharing the card) for both modes.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/multi; mkdir -p $OUT
timeout -k 10 600 python bench.py --mode strong --steps 5 --warmup 1 > $OUT/strong_n1.json 2> $OUT/strong_n1.err || { tail -30 $OUT/strong_n1.err; exit 1; }
cat $OUT/strong_n1.json
MAGOT_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode strong --gpus 2 --steps 3 --warmup 1 > $OUT/strong_n2_gloo.json 2> $OUT/strong_n2_gloo.err || { tail -30 $OUT/strong_n2_gloo.err; exit 1; }
cat $OUT/strong_n2_gloo.json
MAGOT_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/weak_n2_gloo.json 2> $OUT/weak_n2_gloo.err || { tail -30 $OUT/weak_n2_gloo.err; exit 1; }
cat $OUT/weak_n2_gloo.json
