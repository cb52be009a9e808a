#!/bin/bash
# Projected band-sharding scaling (one GPU): tile_scaling.py over configs x path splits.
#   bash scripts/gpu_scaling.sh "C2 C3" "1 0 4 8"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
CFGS=${1:-"C2 C3 C4"}; SPLITS=${2:-"1 0"}
for c in $CFGS; do
  for s in $SPLITS; do
    timeout -k 10 200 python3 scripts/tile_scaling.py $c 8 $s 2>&1 | grep -v amdgpu.ids || exit $?
  done
done 2>&1 | tee gpurun_out/scaling.log
