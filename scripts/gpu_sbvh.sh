#!/bin/bash
# A/B of the spatial-split builder (VRHIP_SBVH_ALPHA) on C2/C3/C5, then the GPU
# parity tests on spatial-split trees.  Usage: bash scripts/gpu_sbvh.sh <tag> <alpha...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in C2 C3 C5; do
  F=16; [ $cfg = C5 ] && F=4
  for al in 0 "$@"; do
    VRHIP_SBVH_ALPHA=$al timeout -k 10 400 python3 scripts/ab.py --cfg $cfg --frames $F vrenderer_pathtracer_amd/libvrhip.so > $OUT/ab_${cfg}_$al.log 2>&1
    rc=$?; echo "sbvh $cfg alpha=$al rc=$rc"; cat $OUT/ab_${cfg}_$al.log
    [ $rc -ne 0 ] && exit $rc
  done
done
VRHIP_SBVH_ALPHA=$1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
exit $rc
