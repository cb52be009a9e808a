#!/bin/bash
# Weak-scaling projections at the bench default (16 x N frames per step):
# rank 0's share of N = 8 at 128 frames per step against one GPU at 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-weak}; mkdir -p $OUT
for cfg in C2 C3 C5; do
  timeout -k 10 240 python3 scripts/tile_scaling.py $cfg 16 0 1 > $OUT/ts_${cfg}_1.log 2>&1 || exit $?
  timeout -k 10 240 python3 scripts/tile_scaling.py $cfg 128 0 8 > $OUT/ts_${cfg}_8w.log 2>&1 || exit $?
  grep -h "N=" $OUT/ts_${cfg}_1.log $OUT/ts_${cfg}_8w.log
done
exit 0
