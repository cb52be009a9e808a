#!/bin/bash
# Full GPU check on the box: parity tests, smoke, bench, rocprofv3 summaries.
# Usage: bash scripts/gpu_round.sh <tag> [--no-prof]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>; stops the script on a crash/timeout
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}

step pytest_gpu 900 python3 -m pytest tests -q -m gpu -rA
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
if [ "$2" != "--no-prof" ]; then
  step prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu
  step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu
  step prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu
  step prof_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/prof_sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu
fi
exit 0
