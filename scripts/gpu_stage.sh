#!/bin/bash
# Result-staging A/B plus WRITE_SIZE of each variant on C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${1:-stage}; mkdir -p $OUT; export TMPDIR=/tmp
shift
for cfg in C2 C3; do
  timeout -k 10 300 python3 scripts/ab.py --cfg $cfg --frames 16 $(for v in "$@"; do echo variants/libvrhip_$v.so; done) > $OUT/ab_$cfg.log 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cat $OUT/ab_$cfg.log; [ $rc -ne 0 ] && exit $rc
done
for v in "$@"; do
  VRHIP_LIB=$PWD/variants/libvrhip_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 > $OUT/write_$v.log 2>&1
  echo "write $v rc=$?"
done
exit 0
