#!/bin/bash
# r05f: GPU tests + smoke + C2/C3/C5 bench lines, then the create_multi
# cadence projection (TS_SYNC=1: 1 and 4 frames per synchronous call).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_quick.sh r05f C2 C3 C5 || exit $?
OUT=gpurun_out/r05f
for cfg in C2 C3; do
  for F in 1 4; do
    TS_SYNC=1 TS_STEPS=30 timeout -k 10 200 python3 -u scripts/tile_scaling.py $cfg $F 0 1,2,4,8 > $OUT/ts_sync_${cfg}_$F.log 2>&1 || exit $?
    grep -v amdgpu.ids $OUT/ts_sync_${cfg}_$F.log
  done
done
