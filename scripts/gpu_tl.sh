#!/bin/bash
# Kernel timelines of back-to-back shard steps (tile_scaling.py at one N):
#   bash scripts/gpu_tl.sh <tag> "<cfg> <frames> <N>" [lib ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; read -r CFG F N <<< "$2"; shift 2
LIBS=${@:-vrenderer_pathtracer_amd/libvrhip.so}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for lib in $LIBS; do
  n=$(basename $lib .so)
  VRHIP_LIB=$PWD/$lib timeout -k 10 120 python3 -u scripts/tile_scaling.py $CFG $F 0 1,$N 2>&1 | grep -v amdgpu.ids | tee $OUT/scal_$n.log || exit $?
  VRHIP_LIB=$PWD/$lib timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl_$n -o run -- \
    python3 -u scripts/tile_scaling.py $CFG $F 0 $N > $OUT/tl_$n.log 2>&1 || exit $?
  python3 scripts/trace_timeline.py $OUT/tl_$n 30 | tee $OUT/tl_$n.txt
done
exit 0
