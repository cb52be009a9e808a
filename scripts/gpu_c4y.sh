#!/bin/bash
# Sphere path pool checks: sphere/split/class/golden GPU tests, C4 A/B against
# variants, and the C4 split probe.   bash scripts/gpu_c4y.sh <tag> [variant.so ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c4y}; shift
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_classes.py tests/test_golden.py -m gpu -k "C4 or C1 or split or CB or C4D or C1T or golden or profiled" -rA -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" $OUT/pytest.log | tail -n 8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python3 scripts/ab.py --cfg C4 --frames 16 --steps 8 vrenderer_pathtracer_amd/libvrhip.so "$@" > $OUT/ab_C4.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab_C4.log | tail -4
# coherence probe curve on C2 (variants/libvrhip_pc*.so, invalid images)
if [ -f variants/libvrhip_pc1.so ]; then
  timeout -k 10 300 python3 scripts/ab.py --cfg C2 --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_pc1.so variants/libvrhip_pc4.so variants/libvrhip_pc16.so > $OUT/ab_C2_probe.log 2>&1
  rc=$?; echo "probe ab rc=$rc"; grep -v amdgpu.ids $OUT/ab_C2_probe.log | tail -6
fi
exit 0
