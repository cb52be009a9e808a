#!/bin/bash
# A/B of one environment knob of the in-tree library on C2/C3/C5 (16 frames per step).
# Usage: bash scripts/gpu_env_ab.sh <tag> <VAR> <value...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in C2 C3 C5; do
  for v in "$@" "$@"; do
    env $VAR=$v timeout -k 10 300 python3 scripts/ab.py --cfg $cfg --frames 16 vrenderer_pathtracer_amd/libvrhip.so > $OUT/ab_${cfg}_$v.log 2>&1
    rc=$?; echo "$cfg $VAR=$v rc=$rc $(grep Mpaths $OUT/ab_${cfg}_$v.log)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
