#!/bin/bash
# A/B of the production library against variant libraries on C2 / C3 / C5
# (scripts/ab.py, 16 frames per step, each library twice, images must match):
#   bash scripts/gpu_ab3.sh <tag> "<configs>" variant.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
LIBS=""
for v in "$@"; do LIBS="$LIBS vrenderer_pathtracer_amd/libvrhip.so $v"; done
for cfg in $CFGS; do
  timeout -k 10 400 python3 -u scripts/ab.py --cfg $cfg --frames 16 --steps 6 $LIBS $LIBS > $OUT/ab_$cfg.log 2>&1 || exit $?
  echo "== $cfg"; grep -v amdgpu.ids $OUT/ab_$cfg.log | tail -$((2 * $# * 2 + 1))
done
