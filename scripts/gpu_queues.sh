#!/bin/bash
# Work-queue head count sweep (VRHIP_QUEUES, runtime) on the production library.
#   bash scripts/gpu_queues.sh <tag> "<configs>" "<queue counts>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-queues}; CFGS=${2:-C3 C5}; QS=${3:-16 32 64}
mkdir -p $OUT
for cfg in $CFGS; do
  for q in $QS; do
    timeout -k 10 240 env VRHIP_QUEUES=$q python3 scripts/ab.py --cfg $cfg --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so > $OUT/ab_${cfg}_q$q.log 2>&1
    rc=$?; echo "$cfg q=$q: $(grep -v amdgpu.ids $OUT/ab_${cfg}_q$q.log | grep Mpaths)"
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  done
done
exit 0
