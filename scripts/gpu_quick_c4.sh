#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-c4}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_classes.py -m gpu -k "C4 or C1 or split or CB or C4D or C1T" -rA -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 -u scripts/c4_probe.py > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat $OUT/probe.log | grep -v amdgpu.ids
exit 0
