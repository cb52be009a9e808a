#!/bin/bash
# Round GPU pass: parity tests, smoke, bench lines for C1-C5, and for every
# config a rocprofv3 kernel trace (--stats) plus separate FETCH_SIZE /
# WRITE_SIZE passes of the same bench command.
#   bash scripts/gpu_round.sh <tag> [--no-tests]
# then: python3 scripts/summarize_round.py gpurun_out/<tag> <round-name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>; stops the script on a crash / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}

if [ "$2" != "--no-tests" ]; then
  step pytest 480 python3 -u -m pytest tests -m gpu -rA -v --timeout 300 --timeout-method thread
  step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_C2 300 python3 bench.py
for cfg in C1 C3 C4 C5 C2D C3D; do
  step bench_$cfg 300 python3 bench.py --config $cfg --no-cpu
done
PB="bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 --strong-steps 0"
for cfg in C1 C2 C3 C4 C5; do
  step trace_$cfg 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$cfg -o run -- python3 $PB --config $cfg
  step fetch_$cfg 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$cfg -o run -- python3 $PB --config $cfg
  step write_$cfg 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$cfg -o run -- python3 $PB --config $cfg
done
exit 0
