#!/bin/bash
# Builder sweep: max leaf size x SAH node cost for the scene BVH, current library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${1:-bvhsweep}; mkdir -p $OUT
for cfg in C2 C3 C5; do
  F=16; [ $cfg = C5 ] && F=4
  for leaf in 2 3 4 6; do
    for nc in 0.5 1.0 2.0; do
      timeout -k 10 200 python3 scripts/ab.py --cfg $cfg --frames $F --leaf $leaf --node-cost $nc vrenderer_pathtracer_amd/libvrhip.so > $OUT/${cfg}_${leaf}_${nc}.log 2>&1
      rc=$?; echo "$cfg leaf=$leaf nc=$nc rc=$rc $(grep -o '[0-9.]* Mpaths/s' $OUT/${cfg}_${leaf}_${nc}.log)"
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
