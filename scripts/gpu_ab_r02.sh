#!/bin/bash
# A/B of libvrhip.so variants (variants/*.so from scripts/build_variants.sh) on C2/C3/C5,
# then WRITE_SIZE of the nt-store variant.  Usage: bash scripts/gpu_ab_r02.sh <tag> <variant names...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
LIBS=""; for v in "$@"; do LIBS="$LIBS variants/libvrhip_$v.so"; done
for cfg in C2 C3 C5; do
  F=16; [ $cfg = C5 ] && F=4
  timeout -k 10 400 python3 scripts/ab.py --cfg $cfg --frames $F $LIBS > $OUT/ab_$cfg.log 2>&1
  rc=$?; echo "ab $cfg rc=$rc"; cat $OUT/ab_$cfg.log
  [ $rc -ne 0 ] && exit $rc
done
if [ -f variants/libvrhip_nt.so ]; then
  VRHIP_LIB=$PWD/variants/libvrhip_nt.so timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_nt_C2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 > $OUT/write_nt_C2.log 2>&1
  echo "write_nt rc=$?"
fi
exit 0
