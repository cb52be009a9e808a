#!/bin/bash
# A/B of launch overlap modes (vrhip_set_overlap -1 automatic vs 1 always) at
# bench.py's 16 frames per step.  Usage: bash scripts/gpu_ovl.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in C2 C3 C5; do
  timeout -k 10 400 python3 scripts/ab.py --cfg $cfg --frames 16 --overlap=-1,1,-1,1 vrenderer_pathtracer_amd/libvrhip.so > $OUT/ovl_$cfg.log 2>&1
  rc=$?; echo "ovl $cfg rc=$rc"; cat $OUT/ovl_$cfg.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
