#!/bin/bash
# Feature-class kernels: the GPU tests, then A/B of the class kernels
# against the generic kernel (variants/libvrhip_noclass.so, -DVR_FEATURE_CLASSES=0),
# the non-BASELINE configs against their nearest exact specialisation, and
# optional variants on C3.
#   bash scripts/gpu_cls.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-cls}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest 480 python3 -u -m pytest tests -m gpu -rA -v --timeout 300 --timeout-method thread
for cfg in ${CFGS:-C2D C3D}; do
  step ab_$cfg 240 python3 scripts/ab.py --cfg $cfg --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_noclass.so
done
step ab_C2 240 python3 scripts/ab.py --cfg C2 --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so
step ab_C3 240 python3 scripts/ab.py --cfg C3 --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_w7h.so
exit 0
