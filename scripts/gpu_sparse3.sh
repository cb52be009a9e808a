#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sparse3}; shift
mkdir -p $OUT
timeout -k 10 480 python3 -u -m pytest tests -m gpu -rA -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -n 8
[ $rc -ne 0 ] && exit $rc
for cfg in C3 C5 C3D; do
  timeout -k 10 240 python3 scripts/ab.py --cfg $cfg --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so "$@" > $OUT/ab_$cfg.log 2>&1
  rc=$?; echo "ab_$cfg rc=$rc"; grep -v amdgpu.ids $OUT/ab_$cfg.log | tail -3
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
for cfg in C3 C5; do
  timeout -k 10 240 env TS_SERVICE=-1 python3 scripts/tile_scaling.py $cfg 16 0 1,8 > $OUT/ts_${cfg}.log 2>&1
  rc=$?; echo "ts_$cfg rc=$rc"; grep -v amdgpu.ids $OUT/ts_${cfg}.log | tail -2
  [ $rc -ne 0 ] && exit $rc
done
exit 0
