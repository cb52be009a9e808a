#!/bin/bash
# C4 / sphere-scene checks: the sphere, split and class GPU tests, the C4
# split probe, and the class-scene rates of the production library and any
# variants given.   bash scripts/gpu_quick_c4.sh <tag> [variant.so ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c4}; shift
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_classes.py tests/test_golden.py -m gpu -k "C4 or C1 or split or CB or C4D or C1T or golden" -rA -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 -u scripts/c4_probe.py > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids $OUT/probe.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u scripts/class_probe.py vrenderer_pathtracer_amd/libvrhip.so "$@" > $OUT/class_probe.log 2>&1
rc=$?; echo "class_probe rc=$rc"; grep -v amdgpu.ids $OUT/class_probe.log
exit 0
