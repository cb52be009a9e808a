#!/bin/bash
# Render-service pass: its GPU tests, then the fixed-cadence projection
# (scripts/tile_scaling.py, 16 frames per step) with and without the service.
#   bash scripts/gpu_svc.sh <tag> [configs...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-svc}; shift
CFGS=${@:-C3 C2 C5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$NO_TESTS" ]; then
  step pytest_svc 300 python3 -u -m pytest tests/test_gpu_service.py -m gpu -rA -v -x --timeout 120 --timeout-method thread
fi
for cfg in $CFGS; do
  step ts_${cfg}_svc 240 env TS_SERVICE=-1 python3 scripts/tile_scaling.py $cfg 16 0 1,4,8
  step ts_${cfg}_base 240 env TS_SERVICE=0 python3 scripts/tile_scaling.py $cfg 16 0 1,4,8
done
exit 0
