#!/bin/bash
# Round GPU pass: parity tests, smoke, bench lines for C1-C5, and for
# C2/C3/C5 a rocprofv3 kernel trace plus separate FETCH_SIZE / WRITE_SIZE
# passes of the same bench command.  Usage: bash scripts/gpu_round.sh <tag> [--no-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>; stops the script on a crash / timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}

if [ "$2" != "--no-tests" ]; then
  step pytest 420 python3 -u -m pytest tests -m gpu -rA -v --timeout 300 --timeout-method thread
  step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_C2 240 python3 bench.py
for cfg in C1 C3 C4 C5; do
  step bench_$cfg 240 python3 bench.py --config $cfg --no-cpu
done
PB="bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0"
for cfg in C2 C3 C5; do
  step trace_$cfg 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$cfg -o run -- python3 $PB --config $cfg
  step fetch_$cfg 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$cfg -o run -- python3 $PB --config $cfg
  step write_$cfg 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$cfg -o run -- python3 $PB --config $cfg
done
exit 0
