#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-spp}; shift
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_classes.py tests/test_golden.py -m gpu -k "C4 or C1 or split or sphere or CB or C4D or C1T or golden or profiled" -rA -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -n 8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python3 scripts/ab.py --cfg C4 --frames 16 --steps 8 vrenderer_pathtracer_amd/libvrhip.so "$@" > $OUT/ab_C4.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab_C4.log | tail -4
exit 0
