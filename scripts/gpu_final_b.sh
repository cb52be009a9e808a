#!/bin/bash
# Final pass, part B: for C1-C5 a rocprofv3 kernel trace (--stats) and separate
# FETCH_SIZE / WRITE_SIZE passes of the same bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-final}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
PB="bench.py --steps 5 --warmup 1 --no-cpu --no-roof --no-verify --interactive-frames 0 --strong-steps 0"
for cfg in ${CFGS:-C1 C2 C3 C4 C5}; do
  for kind in trace fetch write; do
    case $kind in
      trace) args="--kernel-trace --stats";; fetch) args="--pmc FETCH_SIZE";; write) args="--pmc WRITE_SIZE";;
    esac
    timeout -k 10 200 rocprofv3 $args --output-format csv -d $OUT/${kind}_$cfg -o run -- python3 $PB --config $cfg > $OUT/${kind}_$cfg.log 2>&1
    rc=$?; echo "${kind}_$cfg rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 $OUT/${kind}_$cfg.log; exit $rc; fi
  done
done
exit 0
