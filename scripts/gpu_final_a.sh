#!/bin/bash
# Final pass, part A: GPU tests, smoke, bench lines of every config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-final}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest 480 python3 -u -m pytest tests -m gpu -rA -v --timeout 300 --timeout-method thread
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_C2 300 python3 bench.py
for cfg in C1 C3 C4 C5 C2D C3D; do
  step bench_$cfg 300 python3 bench.py --config $cfg --no-cpu
done
exit 0
