#!/bin/bash
# Quick GPU pass: parity tests, smoke, bench lines (no profiler passes).
#   bash scripts/gpu_quick.sh <tag> [configs...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03q}; shift
CFGS=${@:-C2 C3 C5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -z "$NO_TESTS" ]; then
  step pytest 480 python3 -u -m pytest tests -m gpu -rA -v --timeout 300 --timeout-method thread
  step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
for cfg in $CFGS; do
  step bench_$cfg 300 python3 bench.py --config $cfg --no-cpu
done
exit 0
