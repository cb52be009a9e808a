#!/bin/bash
# Per library: one-frame critical path against image size and the A/B rates
# (16-frame steps + one frame per call):  bash scripts/gpu_libs.sh <tag> "<cfgs>" "<sizes>" lib...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFGS=$2; SIZES=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
for lib in "$@"; do
  n=$(basename $lib .so)
  VRHIP_LIB=$PWD/$lib timeout -k 10 150 python3 -u scripts/critical_path.py $CFGS $SIZES 2>&1 | grep -v amdgpu.ids | sed "s/^/$n /" | tee -a $OUT/critical.log || exit $?
done
for c in $(echo $CFGS | tr ',' ' '); do
  timeout -k 10 300 python3 -u scripts/ab.py --cfg $c --frames 16 --steps 3 --interactive 30 "$@" 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.log || exit $?
done
exit 0
