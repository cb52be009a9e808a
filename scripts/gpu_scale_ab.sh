#!/bin/bash
# Projected tile scaling (tile_scaling.py) of several builds:
#   bash scripts/gpu_scale_ab.sh "r0 r8" "C2 16;C5 4" "1,8"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS=$1; RUNS=${2:-"C2 16;C3 16"}; NS=${3:-"1,8"}
IFS=';' read -ra R <<< "$RUNS"
for v in $VARS; do
  for a in "${R[@]}"; do
    set -- $a
    VRHIP_LIB=$PWD/variants/libvrhip_$v.so timeout -k 10 200 python3 scripts/tile_scaling.py $1 $2 0 $NS 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit $?
  done
done | tee gpurun_out/scale_ab.log
