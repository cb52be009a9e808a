#!/bin/bash
# A/B of the production library against variants on several configs:
#   bash scripts/gpu_abx.sh <tag> "<configs>" variant.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-abx}; CFGS=${2:-C2}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for cfg in $CFGS; do
  timeout -k 10 240 python3 scripts/ab.py --cfg $cfg --frames 16 --steps ${AB_STEPS:-6} vrenderer_pathtracer_amd/libvrhip.so "$@" > $OUT/ab_$cfg.log 2>&1
  rc=$?
  echo "ab_$cfg rc=$rc"; grep -v amdgpu.ids $OUT/ab_$cfg.log | tail -n 5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
exit 0
