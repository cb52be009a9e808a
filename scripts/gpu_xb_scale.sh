#!/bin/bash
# XCD band-size A/B (variants/), then the one-GPU 8-rank weak-scaling
# projection of the in-tree library (tile_scaling.py, 16 x N frames per step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_ab_r02.sh ab_xb base xb512 xb32 || exit $?
mkdir -p gpurun_out/scale_r02i
for c in C2 C3 C5; do
  timeout -k 10 240 python3 scripts/tile_scaling.py $c w16 0 1,2,4,8 > gpurun_out/scale_r02i/$c.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/scale_r02i/$c.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
