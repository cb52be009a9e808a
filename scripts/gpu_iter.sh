#!/bin/bash
# One build -> measure iteration on the box: GPU parity tests, A/B of
# variants/*.so on C2/C3/C5 (16 frames per step), projected tile scaling.
#   bash scripts/gpu_iter.sh "variants/libvrhip_base.so variants/libvrhip_new.so" [--no-tests] [--scaling]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
LIBS=$1; shift
OUT=gpurun_out/iter.log; : > $OUT
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a $OUT; tail -4 gpurun_out/pytest_gpu.log | tee -a $OUT
  [ $rc -ne 0 ] && exit $rc
else shift; fi
for cfg in C2 C3 C5; do
  fr=16; [ $cfg = C5 ] && fr=4
  timeout -k 10 400 python3 scripts/ab.py --cfg $cfg --frames $fr --steps 5 $LIBS 2>&1 | grep -v amdgpu.ids | tee -a $OUT || exit $?
done
if [ "$1" = "--scaling" ]; then
  for lib in $LIBS; do
    for cfg in C2 C3; do
      VRHIP_LIB=$PWD/$lib timeout -k 10 200 python3 scripts/tile_scaling.py $cfg 16 0 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $lib) |" | tee -a $OUT || exit $?
    done
  done
fi
exit 0
