#!/bin/bash
# Drain diagnostics (one GPU call): dependent-load latency micro, one-frame
# critical path against image size, one-frame call time against the path
# kernel's resident waves per SIMD, per-path timelines (variants/libvrhip_pt.so).
#   bash scripts/gpu_drain.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-drain}; OUT=gpurun_out/$TAG; mkdir -p $OUT
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ -x scripts/micro/chase ] && step chase 60 scripts/micro/chase
step critical 200 python3 -u scripts/critical_path.py C2,C3 160x96,320x192,640x368,1280x720
for w in 0 3 4 5; do
  for c in C2 C3; do
    VRHIP_WAVES_PER_SIMD=$w step inter_${c}_w$w 200 python3 -u scripts/ab.py --cfg $c --frames 16 --steps 3 --interactive 30 vrenderer_pathtracer_amd/libvrhip.so
  done
done
for c in C2 C3 C5; do
  step strong16_$c 200 python3 -u scripts/tile_scaling.py $c 16 0
done
if [ -f variants/libvrhip_pt.so ]; then
  for a in "C2 1" "C3 1" "C2 1 320 192"; do
    n=$(echo $a | tr ' ' '_')
    VRHIP_LIB=$PWD/variants/libvrhip_pt.so step pt_$n 150 python3 -u scripts/path_times.py $a
  done
fi
exit 0
